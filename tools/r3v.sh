#!/bin/bash
# predictor GEMM shapes (K = 384 / N = 384): two-workgroup kernel and block stagger
export TMPDIR=/tmp
o=gpurun_out/r3v; mkdir -p $o
VJ_BENCH_ONLY=pred VJ_BENCH_ROUNDS=9 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so @VJ_GEMM_2W=1 @VJ_GEMM_STAGGER=2 @VJ_GEMM_STAGGER=6 @VJ_GEMM_2W=1,VJ_GEMM_STAGGER=2 > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
