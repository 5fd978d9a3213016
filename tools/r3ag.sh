#!/bin/bash
# attention forward at 2 workgroups per CU (with the MFMA priority); GEMM DMA issued by waves 0-3 only
export TMPDIR=/tmp
o=gpurun_out/r3ag; mkdir -p $o
VJ_BENCH_KIND=attn VJ_BENCH_ONLY=fwd VJ_BENCH_ROUNDS=9 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_occ2.so > $o/bka.log 2>&1 || { echo "bench failed"; tail -5 $o/bka.log; exit 3; }
cat $o/bka.log
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_dmaw4.so > $o/bkg.log 2>&1 || { echo "bench failed"; tail -5 $o/bkg.log; exit 3; }
cat $o/bkg.log
