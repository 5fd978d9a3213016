#!/bin/bash
# GEMM / model parity with the DMA issued by waves 0-3 on the 256-wide tiles (new default)
export TMPDIR=/tmp
o=gpurun_out/r3ai; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_fp8.py -x -q --timeout 200 --timeout-method thread > $o/kt.log 2>&1
rc=$?; echo "tests: $(tail -1 $o/kt.log)"; [ $rc -ne 0 ] && { tail -30 $o/kt.log; exit $rc; }
exit 0
