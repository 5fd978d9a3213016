#!/bin/bash
# attention forward head dim 32: priority around the PV (p32a) / S (p32b) MFMA clusters
export TMPDIR=/tmp
o=gpurun_out/r3an; mkdir -p $o
VJ_BENCH_KIND=attn VJ_BENCH_ONLY=hd32 VJ_BENCH_ROUNDS=11 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_p32a.so vjepa2_amd/libvjepa_hip_p32b.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
