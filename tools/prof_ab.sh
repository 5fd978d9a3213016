#!/bin/bash
# Per-kernel step profile of several env arms (rocprofv3 --kernel-trace --stats over a short bench.py
# run per arm, each under its own limit), summarised per step by tools/prof_summary.py.
#   TAG=name ARMS="- VJ_X=1,VJ_Y=2 ..." bash tools/prof_ab.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
o=gpurun_out/${TAG:-profab}; mkdir -p "$o"
i=0
for arm in ${ARMS:--}; do
  i=$((i + 1))
  envs=()
  [ "$arm" != "-" ] && IFS=',' read -r -a envs <<< "$arm"
  env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/p$i" -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 > "$o/p$i.log" 2>&1 \
    || { echo "prof failed ($arm)"; tail -5 "$o/p$i.log"; exit 3; }
  f=$(find "$o/p$i" -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] || f=$(find "$o/p$i" -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" 4 "$o/arm$i.txt" "VJ env: $arm" > /dev/null
  echo "arm $i ($arm): $(grep TOTAL "$o/arm$i.txt")"
done
