# GPU tests after the 192-row routing change, then the 16-CU RCCL hold proxy with the all-reduce overlapped
# vs issued at the end of the backward (VJ_ALLREDUCE=end)
cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/r6d && mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -ne 0 ] && { tail -30 $o/tests.log; exit $rc; }
for r in 1 2; do for arm in "0 overlap" "0 end" "16 overlap" "16 end"; do
  set -- $arm; n=$1; mode=$2
  VJ_ALLREDUCE=$mode VJ_RCCL_PROXY_MODE=2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/p_${n}_${mode}_$r.log 2>&1 || { echo "arm $arm failed"; tail -5 $o/p_${n}_${mode}_$r.log; exit 5; }
  python3 -c "import json; d=json.loads([l for l in open('$o/p_${n}_${mode}_$r.log') if l.startswith('{')][-1]); print('proxy hold cus $n allreduce $mode run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['allreduce_exposed_ms'])"
done; done
