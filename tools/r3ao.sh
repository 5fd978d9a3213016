#!/bin/bash
# attention forward with the MFMA priority: V-tile DMA under the softmax (fsp) / K,V ring fragments (ring)
export TMPDIR=/tmp
o=gpurun_out/r3ao; mkdir -p $o
VJ_BENCH_KIND=attn VJ_BENCH_ONLY=fwd VJ_BENCH_ROUNDS=11 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_fsp.so vjepa2_amd/libvjepa_hip_ring.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
