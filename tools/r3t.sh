#!/bin/bash
# attention forward: V tile DMA spread under the softmax
export TMPDIR=/tmp
o=gpurun_out/r3t; mkdir -p $o
VJ_LIB=vjepa2_amd/libvjepa_hip_afs.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ac.py -x -q -k "attention or attn or frame" --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; echo "afs: $(tail -1 $o/kt.log)"; [ $rc -ne 0 ] && exit $rc
VJ_BENCH_KIND=attn VJ_BENCH_ROUNDS=9 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_afs.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
