#!/bin/bash
# per-tile stamps (main loop / epilogue cycles) of the predictor and context GEMM shapes
export TMPDIR=/tmp
o=gpurun_out/r3w; mkdir -p $o
timeout -k 10 200 python -u tools/gemm_stamps.py pred > $o/st_pred.log 2>&1 || { echo "stamps failed"; tail -5 $o/st_pred.log; exit 3; }
timeout -k 10 200 python -u tools/gemm_stamps.py tgt > $o/st_tgt.log 2>&1 || { echo "stamps failed"; tail -5 $o/st_tgt.log; exit 3; }
cat $o/st_pred.log $o/st_tgt.log
