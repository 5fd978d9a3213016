#!/bin/bash
# GPU A/B round: kernel parity tests, then the kernel A/B bench over the given columns.
# usage: tools/run_ab.sh "<pytest -k expr>" COL...   (COL as in tools/bench_kernels.py)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
k=$1; shift
if [ -n "$k" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "$k" > gpurun_out/kt.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/kt.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 480 python -u tools/bench_kernels.py "$@" > gpurun_out/kb2.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/kb2.log; exit $rc
