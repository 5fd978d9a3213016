#!/bin/bash
# attention forward VALU upper bounds: no row sums / no exp-argument fma (measurement builds, wrong results)
export TMPDIR=/tmp
o=gpurun_out/r3aa; mkdir -p $o
VJ_BENCH_KIND=attn VJ_BENCH_ROUNDS=9 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_nolsum.so vjepa2_amd/libvjepa_hip_nofma.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
