#!/bin/bash
# LayerNorm fold: new kernel tests first, then the whole GPU suite, bench (fold on / off)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
TAILN=25 run foldtests 300 python -u -m pytest tests/test_ln_fold_gpu.py -x -v --timeout 120 --timeout-method thread
run gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 300 python bench.py
DDIM_COLD_LN_FOLD=0 run bench_nofold 300 python bench.py
