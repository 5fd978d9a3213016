#!/bin/bash
# One-GPU price of the N > 1 machinery: bench.py plain vs --arm-reducer 1 (the
# bucketed gradient all-reduce over a one-rank RCCL process group: the same buckets, stream joins,
# RCCL stream and kernels as a DP run, minus the xGMI transfer), interleaved, every run under a limit.
# usage: TAG=name RUNS=n bash tools/arm_ab.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
o=gpurun_out/${TAG:-arm}; mkdir -p "$o"
for r in $(seq 1 "${RUNS:-2}"); do
  for arm in ${ARMS:-0 1}; do  # 0: unarmed, 1: armed, 2: process group only; suffix q: GPU_MAX_HW_QUEUES=$QN
    a=${arm%q}; qenv=(); [ "$a" != "$arm" ] && qenv=(GPU_MAX_HW_QUEUES=${QN:-8})
    env "${qenv[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 \
      --arm-reducer $a > "$o/arm${arm}_$r.log" 2>&1 || { echo "bench failed (arm $arm)"; tail -5 "$o/arm${arm}_$r.log"; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/arm${arm}_$r.log') if l.startswith('{')][-1]); print('arm $arm', d.get('reducer_armed'), d.get('dist_backend'), 'run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'], 'allreduce_exposed_ms', d['allreduce_exposed_ms'])"
  done
done
