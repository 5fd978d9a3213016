#!/bin/bash
# step A/B: attention forward priority (default build) vs none (noprio build)
export TMPDIR=/tmp
o=gpurun_out/r3af; mkdir -p $o
for r in 1 2; do
  for b in noprio prio; do
    if [ $b = noprio ]; then L=vjepa2_amd/libvjepa_hip_noprio.so; else L=vjepa2_amd/libvjepa_hip.so; fi
    VJ_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_${b}_$r.log') if l.startswith('{')][-1]); print('$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
# GEMM: s_setprio around each phase's MFMAs (gprio) / static priority for waves 4-7 (gsprio)
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_gprio.so vjepa2_amd/libvjepa_hip_gsprio.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
