#!/bin/bash
# spread 1 (default) vs 0 vs 2: GEMM parity for the default, kernel A/B, step A/B 1 vs 0
export TMPDIR=/tmp
o=gpurun_out/r3r; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm or adamw" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; echo "default: $(tail -1 $o/kt.log)"; [ $rc -ne 0 ] && exit $rc
VJ_LIB=vjepa2_amd/libvjepa_hip_spread2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 200 --timeout-method thread > $o/kt2.log 2>&1
rc=$?; echo "spread2: $(tail -1 $o/kt2.log)"; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 500 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip_spread0.so vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_spread2.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
head -34 $o/bk.log
for r in 1 2; do
  for b in spread0 default; do
    lib=vjepa2_amd/libvjepa_hip.so; [ $b = spread0 ] && lib=vjepa2_amd/libvjepa_hip_spread0.so
    VJ_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_${b}_$r.log') if l.startswith('{')][-1]); print('$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
