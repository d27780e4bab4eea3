#!/bin/bash
# Run GPU steps in sequence, each under its own time limit, stopping at the first failure.
#   bash tools/gpu_run.sh NAME SECONDS "COMMAND" [NAME SECONDS "COMMAND" ...]
# Each step's output goes to gpurun_out/NAME.log; the tail (TAILN lines, default 6) and any
# JSON bench line are echoed.
cd "$(dirname "$0")/.." 2>/dev/null || cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
  name=$1; to=$2; cmd=$3; shift 3
  echo "=== $name ($cmd)"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "rc=$rc"
  tail -"${TAILN:-6}" "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
