#!/bin/bash
# A/B of two library builds on the full bench (alternating runs): tools/ab_bench.sh <variant.so> [runs]
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/abb
n=${2:-2}
for i in $(seq 1 $n); do
  for lib in "$1" ""; do
    tag=$( [ -n "$lib" ] && basename "$lib" .so || echo current )
    VJ_LIB=$lib timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --kernel-events 0 > gpurun_out/abb/$tag.$i.log 2>&1 || { echo "$tag failed"; exit 3; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/abb/$tag.$i.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
  done
done
