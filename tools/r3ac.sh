#!/bin/bash
# tile-order group sweep on the target / predictor GEMM shapes
export TMPDIR=/tmp
o=gpurun_out/r3ac; mkdir -p $o
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 400 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so @VJ_GEMM_GROUP=4 @VJ_GEMM_GROUP=12 @VJ_GEMM_GROUP=16 @VJ_GEMM_GROUP=32 > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
