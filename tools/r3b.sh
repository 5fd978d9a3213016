# round 3: ping-pong GEMM parity + A/B, launcher tests, bench (each GPU step under its own limit)
export TMPDIR=/tmp
o=gpurun_out/r3b; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "pingpong or fused_rope or epilogues or gemm_layouts" --timeout 120 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -4 $o/kt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_kernels.py @VJ_GEMM_PP=0 @VJ_GEMM_PP=1 > $o/bk.log 2>&1 || { echo "bench_kernels failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $o/bench.log 2>&1 || { echo "bench failed"; tail -5 $o/bench.log; exit 4; }
tail -c 1200 $o/bench.log
VJ_GEMM_PP=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_pp0.log 2>&1 || { echo "bench pp0 failed"; exit 5; }
tail -c 300 $o/bench_pp0.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_launcher.py -x -v --timeout 300 --timeout-method thread > $o/launch.log 2>&1
echo "launcher rc=$?"; tail -5 $o/launch.log
