#!/bin/bash
# upper bound of deeper DMA lookahead: main-loop DMA wait removed (measurement build, wrong results)
export TMPDIR=/tmp
o=gpurun_out/r3z; mkdir -p $o
VJ_BENCH_KIND=gemm VJ_BENCH_ROUNDS=7 timeout -k 10 300 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_nowait.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
