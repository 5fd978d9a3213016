# full GPU tests with the S64 default, then kernel traces of the step with / without the RCCL proxy
cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/r6a && mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -ne 0 ] && { tail -30 $o/tests.log; exit $rc; }
for arm in "0 0" "16 2"; do
  set -- $arm; n=$1; m=$2
  VJ_RCCL_PROXY_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_${n}_$m -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/prof_${n}_$m.log 2>&1 || { echo "prof $arm failed"; tail -5 $o/prof_${n}_$m.log; exit 4; }
  python3 tools/prof_summary.py "$(find $o/prof_${n}_$m -name '*kernel_trace.csv' | head -1)" 4 $o/stats_${n}_$m.txt "proxy $n mode $m" || exit 5
  head -30 $o/stats_${n}_$m.txt
done
