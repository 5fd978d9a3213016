#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own hard time limit) over a
# command, results under gpurun_out/pmc/<tag>/pN/. Stops at the first failing pass.
# usage: tools/pmc_passes.sh <tag> <cmd...>
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/pmc/$tag
mkdir -p "$out"
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  echo "=== pass $i: $p"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $p -d "$out/p$i" -o run --output-format csv -- "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -2 "$out/p$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
