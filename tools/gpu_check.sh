#!/bin/bash
# First-contact GPU check: kernel tests, model tests, quick perf, rocprof stats.
# Each GPU step has its own time limit; a crash/fault (rc>1) stops the script.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "rc=$rc"; tail -25 gpurun_out/$name.log
  if [ $rc -gt 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
run kernels 400 python -m pytest tests/test_kernels_gpu.py -x -q
run model 300 python -m pytest tests/test_model_gpu.py -x -q
run perf 300 python tools/quick_perf.py
