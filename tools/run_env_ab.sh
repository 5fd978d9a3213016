#!/bin/bash
# GPU: the train-step bench once per environment setting, 1 GPU, no CPU baseline.
# usage: tools/run_env_ab.sh "ENV=V [ENV2=V2]" ...   ("" = defaults)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i + 1))
  env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 > "gpurun_out/bench_env$i.log" 2>&1
  rc=$?; echo "[$e] rc=$rc"; python -c "import json,sys; d=json.loads(open('gpurun_out/bench_env$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'])" 2>/dev/null
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/bench_env$i.log"; exit $rc; fi
done
