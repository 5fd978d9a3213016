#!/bin/bash
# DMA hi: A pieces from waves 0-3, B pieces from waves 4-7 (hi build) vs both from waves 0-3
export TMPDIR=/tmp
o=gpurun_out/r3al; mkdir -p $o
VJ_LIB=vjepa2_amd/libvjepa_hip_hi.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm or linear or rope or pingpong or 192" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; echo "tests hi: $(tail -1 $o/kt.log)"; [ $rc -ne 0 ] && { tail -30 $o/kt.log; exit $rc; }
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_hi.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
for r in 1 2; do
  for b in base hi; do
    if [ $b = base ]; then L=vjepa2_amd/libvjepa_hip.so; else L=vjepa2_amd/libvjepa_hip_hi.so; fi
    VJ_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_${b}_$r.log') if l.startswith('{')][-1]); print('$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
