#!/bin/bash
# GEMM main-loop variants: DMA spread around the last phase's MFMAs, no SLP packing
export TMPDIR=/tmp
o=gpurun_out/r3q; mkdir -p $o
for v in spread noslp; do
  VJ_LIB=vjepa2_amd/libvjepa_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 200 --timeout-method thread > $o/kt_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $o/kt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
VJ_BENCH_ROUNDS=7 timeout -k 10 500 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_spread.so vjepa2_amd/libvjepa_hip_noslp.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_optim.py tests/test_gpu_train_vs_oracle.py -x -q -k "adamw or ema or optim or train" --timeout 200 --timeout-method thread > $o/kt_opt.log 2>&1
rc=$?; echo "optim: $(tail -1 $o/kt_opt.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for b in 1 0; do
    VJ_FUSED_EMA=$b timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_e${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_e${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_e${b}_$r.log') if l.startswith('{')][-1]); print('FUSED_EMA=$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
