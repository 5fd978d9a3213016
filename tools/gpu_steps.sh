#!/bin/bash
# Run GPU steps in order; each under its own timeout. Continue past ordinary test failures (rc 1),
# stop at anything that looks like a crash, abort or timeout (rc >= 2).
# usage: tools/gpu_steps.sh "<timeout_s> <logname> <cmd...>" ...
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for spec in "$@"; do
  t=$(echo "$spec" | awk '{print $1}'); log=$(echo "$spec" | awk '{print $2}'); cmd=$(echo "$spec" | cut -d' ' -f3-)
  echo "=== [$log] $cmd (timeout ${t}s)"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$log.log" 2>&1
  rc=$?
  echo "=== [$log] rc=$rc"; tail -5 "gpurun_out/$log.log"
  if [ $rc -ge 2 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
