export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 500 python -u -m pytest tests/test_gpu_launcher.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a/launch.log 2>&1
echo "launcher rc=$?"; tail -5 gpurun_out/r3a/launch.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r3a/bench.log 2>&1 && tail -c 1500 gpurun_out/r3a/bench.log
