# new GPU tests + PP variants A/B (kernels) + LN A/B + step-level A/B (PP for RoPE only vs off)
export TMPDIR=/tmp
o=gpurun_out/r3d; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train_vs_oracle.py tests/test_gpu_model.py -q -k "pingpong or fused_rope or fpc_groups or autocast or residual_precision or train_step_vs_oracle or test_gemm or layernorm or block_matches" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; grep -E "passed|failed|rel_l1|mean\|" $o/kt.log | tail -20; [ $rc -ge 2 ] && exit $rc
VJ_BENCH_ONLY="ln " timeout -k 10 200 python -u tools/bench_kernels.py @VJ_LN_V1=1 @VJ_LN_V1=0 > $o/bk_ln.log 2>&1 || { echo "bench ln failed"; tail -5 $o/bk_ln.log; exit 3; }
cat $o/bk_ln.log
timeout -k 10 400 python -u tools/bench_kernels.py @VJ_GEMM_PP=0 @VJ_GEMM_PP=1 vjepa2_amd/libvjepa_hip_prio0.so@VJ_GEMM_PP=1 > $o/bk.log 2>&1 || { echo "bench_kernels failed"; tail -5 $o/bk.log; exit 3; }
head -33 $o/bk.log
for pp in 0 "" 0 ""; do
  VJ_GEMM_PP=$pp timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_pp$pp.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_pp$pp.log; exit 4; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$o/bench_pp$pp.log') if l.startswith('{')][-1]); print('PP=${pp:-default}', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
