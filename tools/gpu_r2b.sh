#!/bin/bash
# data-parallel step topology A/B (tools/gpu_fork.sh), then the full GPU suite + bench
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_fork.sh 2>&1 | tee gpurun_out/fork.txt || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 || { tail -5 gpurun_out/r2_bench.log; exit 1; }
grep "^{" gpurun_out/r2_bench.log | cut -c1-400
