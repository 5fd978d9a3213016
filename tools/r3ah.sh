#!/bin/bash
# step A/B: GEMM DMA by waves 0-3 only (dmaw4 build) vs all 8 waves (default); RoPE / GELU shapes again
export TMPDIR=/tmp
o=gpurun_out/r3ah; mkdir -p $o
for r in 1 2; do
  for b in base dmaw4; do
    if [ $b = base ]; then L=vjepa2_amd/libvjepa_hip.so; else L=vjepa2_amd/libvjepa_hip_dmaw4.so; fi
    VJ_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_${b}_$r.log') if l.startswith('{')][-1]); print('$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=9 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_dmaw4.so > $o/bkg.log 2>&1 || { echo "bench failed"; tail -5 $o/bkg.log; exit 3; }
cat $o/bkg.log
