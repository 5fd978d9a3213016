# ping-pong GEMM (3-stage ring) parity + A/B against the one-tile kernel
export TMPDIR=/tmp
o=gpurun_out/r3c; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "pingpong or fused_rope or epilogues or gemm_layouts" --timeout 120 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -4 $o/kt.log; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_ONLY=${VJ_BENCH_ONLY:-} timeout -k 10 300 python -u tools/bench_kernels.py @VJ_GEMM_PP=0 @VJ_GEMM_PP=1 > $o/bk.log 2>&1 || { echo "bench_kernels failed"; tail -5 $o/bk.log; exit 3; }
head -33 $o/bk.log
