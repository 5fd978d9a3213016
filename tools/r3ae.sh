#!/bin/bash
# attention backward: s_setprio around the S / dP (1), dV / dK or dQ (2), both (3) MFMA clusters;
# attention parity tests with the default build (forward priority on)
export TMPDIR=/tmp
o=gpurun_out/r3ae; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention or attn" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; echo "tests: $(tail -1 $o/kt.log)"; [ $rc -ne 0 ] && { tail -30 $o/kt.log; exit $rc; }
VJ_BENCH_KIND=attn VJ_BENCH_ONLY=bwd VJ_BENCH_ROUNDS=9 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_bprio1.so vjepa2_amd/libvjepa_hip_bprio2.so vjepa2_amd/libvjepa_hip_bprio3.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
