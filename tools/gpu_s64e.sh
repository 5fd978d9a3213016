cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/s64e && mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "gemm or gelu" > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -ne 0 ] && { tail -30 $o/tests.log; exit $rc; }
TAG=s64e STEPS="VJ_GEMM_STG64=0 - VJ_GEMM_STG64=1" RUNS=2 bash tools/gpu_ab.sh || exit 4
for r in 1 2; do for arm in "0 0" "16 0" "16 1" "16 2"; do
  set -- $arm; n=$1; m=$2
  VJ_RCCL_PROXY_MODE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/proxy_${n}_${m}_$r.log 2>&1 || { echo "proxy $n $m failed"; tail -5 $o/proxy_${n}_${m}_$r.log; exit 5; }
  python3 -c "import json; d=json.loads([l for l in open('$o/proxy_${n}_${m}_$r.log') if l.startswith('{')][-1]); print('proxy cus $n mode $m run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['allreduce_exposed_ms'], d['dist_backend'])"
done; done
