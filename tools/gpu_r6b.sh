# full GPU tests (S64 default everywhere), then the RCCL proxy modes (16 CUs) with / without CU reservation
cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/r6b && mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -ne 0 ] && { tail -30 $o/tests.log; exit $rc; }
for r in 1 2; do for arm in "0 0 0" "16 0 0" "16 1 0" "16 2 0" "16 2 16"; do
  set -- $arm; n=$1; m=$2; res=$3
  VJ_RCCL_RESERVE_CUS=$res VJ_RCCL_PROXY_MODE=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/proxy_${n}_${m}_${res}_$r.log 2>&1 || { echo "proxy $arm failed"; tail -5 $o/proxy_${n}_${m}_${res}_$r.log; exit 5; }
  python3 -c "import json; d=json.loads([l for l in open('$o/proxy_${n}_${m}_${res}_$r.log') if l.startswith('{')][-1]); print('proxy cus $n mode $m reserve $res run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['allreduce_exposed_ms'], d['dist_backend'])"
done; done
