# attention backward with the stored dS^T: parity, kernel A/B, step A/B
export TMPDIR=/tmp
o=gpurun_out/r3f; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention or fused_rope or layernorm" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -3 $o/kt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_vs_oracle.py tests/test_gpu_model.py -q -k "fpc_groups or autocast or wide_head" --timeout 300 --timeout-method thread > $o/kt2.log 2>&1
rc=$?; grep -E "passed|failed|rel_l1 [0-9]|G\)|worst|fpc" $o/kt2.log | tail -40; [ $rc -ge 2 ] && exit $rc
VJ_BENCH_ONLY="attn" timeout -k 10 300 python -u tools/bench_kernels.py @VJ_ATTN_DS=0 @VJ_ATTN_DS=1 > $o/bk.log 2>&1 || { echo "bench attn failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
for ds in 0 1 0 1; do
  VJ_ATTN_DS=$ds timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_ds$ds.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_ds$ds.log; exit 4; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/bench_ds$ds.log') if l.startswith('{')][-1]); print('DS=$ds', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
