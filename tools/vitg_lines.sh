#!/bin/bash
# BASELINE configs[3] / [4] bench lines (single GPU): ViT-g/16 16x384^2 B=24 bf16, ViT-g/16 64x256^2 B=6
# bf16 and with the fp8 target encoder. Each run under its own limit; stop at the first failure.
cd "$(dirname "$0")/.." || exit 2
out=gpurun_out/vitg; mkdir -p $out
timeout -k 10 400 python -u bench.py --model vit_giant_xformers --crop 384 --frames 16 --batch 24 --steps 3 --warmup 2 --cpu-baseline 0 > $out/g384.log 2>&1 || { echo "g384 failed"; tail -3 $out/g384.log; exit 3; }
grep '^{' $out/g384.log | tail -1 | cut -c1-400
for fp8 in 0 1; do
  timeout -k 10 400 python -u bench.py --model vit_giant_xformers --crop 256 --frames 64 --batch 6 --steps 3 --warmup 2 --cpu-baseline 0 --fp8-target $fp8 > $out/g64_fp8$fp8.log 2>&1 || { echo "g64 fp8=$fp8 failed"; tail -3 $out/g64_fp8$fp8.log; exit 4; }
  grep '^{' $out/g64_fp8$fp8.log | tail -1 | cut -c1-400
done
