#!/bin/bash
# GPU validation pass: new-kernel tests first (short limit), microbench, smoke, all GPU tests
# (with their printed measurements), numerical error report, bench
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log | cut -c1-800
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run gputests 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread
run grad_error 300 python tools/grad_error_report.py
run bench 400 python bench.py
grep -h "^{" gpurun_out/bench.log | cut -c1-2000
