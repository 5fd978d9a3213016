#!/bin/bash
# A/B of the two-workgroup GEMM (with / without the per-CU stagger) against the 8-wave kernel
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/ab2w
VJ_BENCH_ROUNDS=5 timeout -k 10 400 python -u tools/bench_kernels.py "" "@VJ_GEMM_2W=1" "@VJ_GEMM_2W=1,VJ_GEMM_STAGGER=4" "@VJ_GEMM_2W=1,VJ_GEMM_STAGGER=10" > gpurun_out/ab2w/k.log 2>&1
echo rc=$?
