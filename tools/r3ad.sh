#!/bin/bash
# attention forward: s_setprio around the S (1) / PV (2) / both (3) MFMA clusters, head dim 64
export TMPDIR=/tmp
o=gpurun_out/r3ad; mkdir -p $o
VJ_BENCH_KIND=attn VJ_BENCH_ONLY=fwd VJ_BENCH_ROUNDS=11 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_prio1.so vjepa2_amd/libvjepa_hip_prio2.so vjepa2_amd/libvjepa_hip_prio3.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
