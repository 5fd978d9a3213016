#!/bin/bash
# rocprofv3 PMC passes over a short bench.py run (each pass its own process, under a hard limit):
# MFMA busy + clock, HBM-side fetch, HBM-side write. Then tools/pmc_report.py summarises the top
# kernels. usage: tools/pmc_bench.sh <tag> [bench.py args...]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmc_bench/$tag
mkdir -p "$out"
passes=("SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE")
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  VJ_TGT_STREAM=0 VJ_WGRAD_STREAM=0 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $p -d "$out/p$i" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
done
python3 tools/pmc_report.py "$out" > "$out/report.txt"; cat "$out/report.txt"
