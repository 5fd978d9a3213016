# update-envelope test + a kernel-trace profile of the default step
export TMPDIR=/tmp
o=gpurun_out/r3g; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -q -s -k "train_steps_match or attention_fwd_bwd" --timeout 300 --timeout-method thread > $o/t.log 2>&1
rc=$?; grep -E "passed|failed|all updates|Error|assert" $o/t.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0 > $o/prof.log 2>&1 || { echo "prof failed"; tail -5 $o/prof.log; exit 4; }
echo prof ok
timeout -k 10 120 ./tools/peak_bin > $o/peak.json 2>&1 || { echo "peak failed"; cat $o/peak.json; exit 5; }
cat $o/peak.json
