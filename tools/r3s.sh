#!/bin/bash
# B-piece split point (1 / 2 = default / 3 m-tiles) and the 32-deep 2W kernel spread
export TMPDIR=/tmp
o=gpurun_out/r3s; mkdir -p $o
for v in split1 split3 s32; do
  VJ_LIB=vjepa2_amd/libvjepa_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 200 --timeout-method thread > $o/kt_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $o/kt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 500 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_split1.so vjepa2_amd/libvjepa_hip_split3.so vjepa2_amd/libvjepa_hip_s32.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
