#!/bin/bash
# BASELINE configs[3] / [4] bench lines with roofline.traffic: for each ViT-g config, a bench run (its
# dominant kernel), FETCH_SIZE / WRITE_SIZE PMC passes over the same bench, tools/traffic.py into
# profiles/traffic.json (one entry per kernel + workload), then the final bench line.
# usage: tools/vitg_final.sh <tag>
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=${1:-vitg}
out=gpurun_out/$tag; mkdir -p "$out"
# traffic entries go to a copy under gpurun_out (merged back by gpurun; profiles/ on the box is not):
# copy $out/traffic.json to profiles/traffic.json afterwards
cp profiles/traffic.json "$out/traffic.json"
run() {  # name workload bench-args...
  local name=$1 wl=$2; shift 2
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --cpu-baseline 0 "$@" > "$out/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$out/$name.log"; return 3; }
  local dom
  dom=$(python3 -c "import json; print(json.loads([l for l in open('$out/$name.log') if l.startswith('{')][-1])['roofline']['kernel'])") || return 3
  echo "$name dominant: $dom"
  local i=0
  for p in FETCH_SIZE WRITE_SIZE; do
    i=$((i + 1))
    VJ_TGT_STREAM=0 VJ_WGRAD_STREAM=0 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $p -d "$out/${name}_p$i" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 "$@" > "$out/${name}_p$i.log" 2>&1 || { echo "$name pmc $p failed"; tail -3 "$out/${name}_p$i.log"; return 4; }
  done
  python3 tools/traffic.py "$out/${name}_p1" "$out/${name}_p2" "$dom" "$out/traffic.json" "$wl" || return 5
  cp "$out/traffic.json" profiles/traffic.json  # the final line below reads it
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 "$@" > "$out/${name}_final.log" 2>&1 || { echo "$name final failed"; return 3; }
  grep '^{' "$out/${name}_final.log" | tail -1 > "$out/${name}.json"
  cut -c1-600 "$out/${name}.json"
}
run g384 "vit_giant_xformers 16x384^2 B=24" --model vit_giant_xformers --crop 384 --frames 16 --batch 24 || exit $?
run g64 "vit_giant_xformers 64x256^2 B=6" --model vit_giant_xformers --crop 256 --frames 64 --batch 6 --fp8-target 0 || exit $?
run g64f8 "vit_giant_xformers 64x256^2 B=6" --model vit_giant_xformers --crop 256 --frames 64 --batch 6 --fp8-target 1 || exit $?
