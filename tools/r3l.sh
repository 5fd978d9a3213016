#!/bin/bash
# Step A/B of the batched W^T refresh (2 runs each, alternating), then the ViT-g bench lines
export TMPDIR=/tmp
o=gpurun_out/r3l; mkdir -p $o
for r in 1 2; do
  for b in 1 0; do
    VJ_WT_BATCH=$b timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_b${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_b${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_b${b}_$r.log') if l.startswith('{')][-1]); print('WT_BATCH=$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
bash tools/vitg_final.sh r03vitg
timeout -k 10 200 python -u tools/blaslt_probe.py > gpurun_out/r3n/blaslt.log 2>&1 || { echo "blaslt probe failed"; tail -5 gpurun_out/r3n/blaslt.log; exit 6; }
cat gpurun_out/r3n/blaslt.log
