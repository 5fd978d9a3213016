#!/bin/bash
# attention forward addressing (no spills): parity, kernel A/B vs the committed build, step A/B
export TMPDIR=/tmp
o=gpurun_out/r3m; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ac.py -x -q -k "attention or attn or fused_rope or frame" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; tail -3 $o/kt.log; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_ONLY="attn" VJ_BENCH_ROUNDS=7 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip_base.so vjepa2_amd/libvjepa_hip.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
for r in 1 2; do
  for b in base new; do
    lib=vjepa2_amd/libvjepa_hip.so; [ $b = base ] && lib=vjepa2_amd/libvjepa_hip_base.so
    VJ_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_${b}_$r.log') if l.startswith('{')][-1]); print('$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
