#!/bin/bash
# ping-pong GEMM forms on the short-K predictor / context shapes
export TMPDIR=/tmp
o=gpurun_out/r3y; mkdir -p $o
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so @VJ_GEMM_PP=1 @VJ_GEMM_PP=2 > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
