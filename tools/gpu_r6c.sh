# kernel traces of the step with / without the 16-CU RCCL proxy (hold mode: CUs held, no bytes)
cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/r6c && mkdir -p $o
for arm in "0 0" "16 2"; do
  set -- $arm; n=$1; m=$2
  VJ_RCCL_PROXY_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_${n}_$m -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/prof_${n}_$m.log 2>&1 || { echo "prof $arm failed"; tail -5 $o/prof_${n}_$m.log; exit 4; }
  python3 tools/prof_summary.py "$(find $o/prof_${n}_$m -name '*kernel_trace.csv' | head -1)" 4 $o/stats_${n}_$m.txt "proxy $n mode $m" || exit 5
  grep -o '"value": [0-9.]*' $o/prof_${n}_$m.log
done
