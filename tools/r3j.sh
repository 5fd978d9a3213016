# fused attention backward, interleaved: parity, kernel A/B, step A/B
export TMPDIR=/tmp
o=gpurun_out/r3j; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -3 $o/kt.log; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_ONLY="attn bwd" timeout -k 10 300 python -u tools/bench_kernels.py @VJ_ATTN_FUSED=0 @VJ_ATTN_FUSED=1 > $o/bk.log 2>&1 || { echo "bench attn failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
for d in 0 1; do
  VJ_ATTN_FUSED=$d timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_f$d.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_f$d.log; exit 4; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/bench_f$d.log') if l.startswith('{')][-1]); print('FUSED=$d', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
for dl in 1 0; do
  VJ_ATTN_FUSED=0 VJ_ATTN_DELTA=$dl timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_d$dl.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_d$dl.log; exit 4; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/bench_d$dl.log') if l.startswith('{')][-1]); print('FUSED=0 DELTA=$dl', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
timeout -k 10 200 python -u tools/blaslt_probe.py > $o/blaslt.log 2>&1 || { echo "blaslt probe failed"; tail -5 $o/blaslt.log; exit 6; }
cat $o/blaslt.log
