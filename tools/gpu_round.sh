#!/bin/bash
# One GPU session: tests, bench, kernel-trace profile (+ HIP API trace), each step under its own limit.
# usage: tools/gpu_round.sh <tag> [skip_tests]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=${1:-run}
mkdir -p gpurun_out/$tag
if [ "$2" != "skip_tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$tag/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$tag/pytest.log
  if [ $rc -ge 2 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/$tag/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/$tag/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv \
  -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0 > gpurun_out/$tag/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/$tag/prof.log
exit $rc
