#!/bin/bash
# One parameterised GPU A/B session (replaces the round-3 one-off r3*.sh scripts). Every GPU step
# runs under its own time limit; the script stops at the first failing step.
#
#   TAG=name                       output directory gpurun_out/<name>
#   TESTS="expr"                   pytest -k expression over tests/test_gpu_kernels.py ("all": every
#                                  -m gpu test; unset: no tests)
#   KCOLS="col col ..."            tools/bench_kernels.py columns (lib.so | lib.so@ENV=V | @ENV=V);
#   KIND=gemm|attn|ln|...          VJ_BENCH_KIND for it; ROUNDS (default 7); ONLY -> VJ_BENCH_ONLY
#   STEPS="arm arm ..."            bench.py step A/B: each arm "-" (defaults) or "ENV=V,ENV2=V2";
#   RUNS=n                         interleaved rounds of the arms (default 2)
#
# usage: TAG=x TESTS=gemm KCOLS="@VJ_GEMM_BM192=0 vjepa2_amd/libvjepa_hip.so" STEPS="- VJ_GEMM_BM192=0" \
#          bash tools/gpu_ab.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
o=gpurun_out/${TAG:-ab}; mkdir -p "$o"
if [ -n "$TESTS" ]; then
  if [ "$TESTS" = all ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$o/tests.log" 2>&1
  else
    timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
      -k "$TESTS" > "$o/tests.log" 2>&1
  fi
  rc=$?; echo "tests: $(tail -1 "$o/tests.log")"; [ $rc -ne 0 ] && { tail -40 "$o/tests.log"; exit $rc; }
fi
if [ -n "$KCOLS" ]; then
  # shellcheck disable=SC2086
  VJ_BENCH_KIND=${KIND:-} VJ_BENCH_ONLY=${ONLY:-} VJ_BENCH_ROUNDS=${ROUNDS:-7} timeout -k 10 480 \
    python -u tools/bench_kernels.py $KCOLS > "$o/bk.log" 2>&1 || { echo "kernel bench failed"; tail -8 "$o/bk.log"; exit 3; }
  cat "$o/bk.log"
fi
if [ -n "$STEPS" ]; then
  for r in $(seq 1 "${RUNS:-2}"); do
    i=0
    for arm in $STEPS; do
      i=$((i + 1))
      envs=()
      [ "$arm" != "-" ] && IFS=',' read -r -a envs <<< "$arm"
      env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 \
        > "$o/step_${i}_$r.log" 2>&1 || { echo "bench failed ($arm)"; tail -5 "$o/step_${i}_$r.log"; exit 4; }
      python3 -c "import json; d=json.loads([l for l in open('$o/step_${i}_$r.log') if l.startswith('{')][-1]); print('arm $arm run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
    done
  done
fi
