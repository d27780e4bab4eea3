#!/bin/bash
# patch-row sampler state: tests, then A/B of the sampler bench (rows on/off) and the head microbench
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log | cut -c1-900
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run rows_tests 300 python -u -m pytest tests/test_sampler_rows_gpu.py tests/test_sampler_gpu.py -x -v --timeout 120 --timeout-method thread
run s_rows_ab 300 python tools/ub_sampler.py ROWS 30 4
run ends 120 python tools/ub_sampler_ends.py
run bench 400 python bench.py --no-eager-baseline
