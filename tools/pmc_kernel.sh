#!/bin/bash
# PMC counters (two SQ passes) for one tools/bench_kernels.py case, each pass under a hard limit.
# usage: tools/pmc_kernel.sh <tag> <bench_kernels args...>   (env VJ_BENCH_ONLY selects the case)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmc/$tag
mkdir -p "$out"
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  VJ_BENCH_ROUNDS=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $p -d "$out/p$i" -o run --output-format csv -- python3 tools/bench_kernels.py "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -2 "$out/p$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py "$out" > "$out/summary.txt"; cat "$out/summary.txt"
