#!/bin/bash
# VALU cross-lane exchanges (DPP / permlane swaps instead of ds_bpermute): full GPU tests, kernel
# A/B (GEMM epilogues, attention, LayerNorm), step A/B; hipBLASLt kernel names
export TMPDIR=/tmp
o=gpurun_out/r3p; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_ROUNDS=5 timeout -k 10 400 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip_base.so vjepa2_amd/libvjepa_hip.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
for r in 1 2; do
  for b in base new; do
    lib=vjepa2_amd/libvjepa_hip.so; [ $b = base ] && lib=vjepa2_amd/libvjepa_hip_base.so
    VJ_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 > $o/bench_${b}_$r.log 2>&1 || { echo "bench failed"; tail -5 $o/bench_${b}_$r.log; exit 4; }
    python3 -c "import json; d=json.loads([l for l in open('$o/bench_${b}_$r.log') if l.startswith('{')][-1]); print('$b run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/blt -o run --output-format csv -- python3 tools/blaslt_probe.py > $o/blt.log 2>&1 || { echo "blaslt prof failed"; tail -3 $o/blt.log; exit 5; }
echo "blaslt prof ok"
