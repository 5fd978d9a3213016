#!/bin/bash
# HBM-side bytes (FETCH_SIZE / WRITE_SIZE, separate passes) of one tools/bench_kernels.py case per
# library build. usage: tools/pmc_bytes.sh <tag> <lib.so ...>   (env VJ_BENCH_ONLY selects the case)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmcb/$tag
mkdir -p "$out"
for lib in "$@"; do
  b=$(basename "$lib" .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    VJ_BENCH_ROUNDS=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d "$out/$b/$c" -o run --output-format csv -- python3 tools/bench_kernels.py "$lib" > "$out/$b.$c.log" 2>&1
    rc=$?
    echo "$b $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 "$out/$b.$c.log"; exit $rc; fi
  done
  python3 tools/pmc_summary.py "$out/$b" > "$out/$b.summary.txt"; echo "== $b"; cat "$out/$b.summary.txt"
done
