# BASELINE configs[4] (ViT-g 64x256^2 B=6): bf16 vs fp8-target lines with the serialised per-kernel breakdown
cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/${1:-fp8} && mkdir -p $o
for f8 in 0 1; do
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --model vit_giant_xformers --crop 256 --frames 64 --batch 6 --fp8-target $f8 > $o/g64_f8$f8.log 2>&1 || { echo "fp8=$f8 failed"; tail -5 $o/g64_f8$f8.log; exit 3; }
  grep '^{' $o/g64_f8$f8.log | tail -1 > $o/g64_f8$f8.json
  python3 -c "import json; d=json.load(open('$o/g64_f8$f8.json')); print('fp8', $f8, d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
