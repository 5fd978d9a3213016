#!/bin/bash
# End-of-round measurement: full GPU tests, bench, kernel-trace stats, PMC passes (MFMA busy, HBM
# fetch / write) and the dominant kernel's traffic; every GPU step under its own limit, stop at the
# first failure. usage: tools/gpu_final.sh <tag>
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$out/pytest.log"; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -u bench.py > "$out/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$out/bench.log"; exit 3; }
tail -c 600 "$out/bench.log"
VJ_TGT_STREAM=0 VJ_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 > "$out/prof.log" 2>&1 || { echo "prof failed"; tail -5 "$out/prof.log"; exit 4; }
echo "prof ok"
# per-step kernel table from the trace's steady-state window (tools/prof_summary.py: setup excluded)
python3 tools/prof_summary.py "$(find "$out/prof" -name '*kernel_trace.csv' | head -1)" 4 "$out/kernel_stats.txt" \
  "VJ_TGT_STREAM=0 VJ_WGRAD_STREAM=0 python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 (serialised)" \
  || { echo "prof summary failed"; exit 4; }
bash tools/pmc_bench.sh "$tag" > "$out/pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "$out/pmc.log"; exit 5; }
echo "pmc ok"
# the bench's own dominant kernel (roofline.kernel of its JSON line)
dom=$(python3 -c "import json,sys; print(json.loads([l for l in open('$out/bench.log') if l.startswith('{')][-1])['roofline']['kernel'])")
echo "dominant: $dom"
cp profiles/traffic.json "$out/traffic.json"  # merged: this entry replaced, the ViT-g entries kept
python3 tools/traffic.py gpurun_out/pmc_bench/$tag/p2 gpurun_out/pmc_bench/$tag/p3 "$dom" "$out/traffic.json"
