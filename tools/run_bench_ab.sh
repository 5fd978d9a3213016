#!/bin/bash
# GPU: the train-step bench once per library build (VJ_LIB), 1 GPU, no CPU baseline.
# usage: tools/run_bench_ab.sh lib.so ...
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename "$lib" .so)
  VJ_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 > "gpurun_out/bench_$n.log" 2>&1
  rc=$?; echo "[$n] rc=$rc"; python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$n.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'])" 2>/dev/null
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/bench_$n.log"; exit $rc; fi
done
