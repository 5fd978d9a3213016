# delta fused into the dQ sweep: parity, kernel A/B, step A/B; peak probe (16x16 fixed)
export TMPDIR=/tmp
o=gpurun_out/r3h; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -3 $o/kt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_vs_oracle.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread > $o/kt2.log 2>&1
rc=$?; tail -3 $o/kt2.log; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_ONLY="attn" timeout -k 10 300 python -u tools/bench_kernels.py @VJ_ATTN_DELTA=1 @VJ_ATTN_DELTA=0 > $o/bk.log 2>&1 || { echo "bench attn failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
for d in 1 0 1 0; do
  VJ_ATTN_DELTA=$d timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_d$d.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_d$d.log; exit 4; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/bench_d$d.log') if l.startswith('{')][-1]); print('DELTA=$d', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
timeout -k 10 120 ./tools/peak_bin > $o/peak.json 2>&1 || { echo "peak failed"; cat $o/peak.json; exit 5; }
cat $o/peak.json
