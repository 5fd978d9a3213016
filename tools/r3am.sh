#!/bin/bash
# with 4 DMA waves: B pieces after 2 / 1 of the last phase's m-tiles (sp2 / sp1), A pieces after the first (spr2)
export TMPDIR=/tmp
o=gpurun_out/r3am; mkdir -p $o
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 400 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_sp2.so vjepa2_amd/libvjepa_hip_sp1.so vjepa2_amd/libvjepa_hip_spr2.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
