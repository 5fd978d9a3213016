#!/bin/bash
# 32x32x16 ping-pong GEMM: parity (PP tests), then kernel A/B of one-tile / PP16 / PP32
export TMPDIR=/tmp
o=gpurun_out/r3k; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "pingpong or fused_rope or transpose" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -5 $o/kt.log; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_ROUNDS=5 timeout -k 10 400 python -u tools/bench_kernels.py @VJ_GEMM_PP=0 @VJ_GEMM_PP=1 @VJ_GEMM_PP=2 > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
head -34 $o/bk.log
