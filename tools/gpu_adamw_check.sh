#!/bin/bash
# fused AdamW numerics + engine parity, then the headline bench (vectorised optimizer pass)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k adamw tests/test_engine_gpu.py > gpurun_out/adamw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/adamw_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-eager-baseline > gpurun_out/adamw_bench.log 2>&1
rc=$?; grep "^{" gpurun_out/adamw_bench.log | cut -c1-400; [ $rc -eq 0 ] || { tail -5 gpurun_out/adamw_bench.log; exit $rc; }
timeout -k 10 200 python bench.py --no-eager-baseline --no-sampler > gpurun_out/adamw_bench2.log 2>&1
rc=$?; grep "^{" gpurun_out/adamw_bench2.log | cut -c1-300; exit $rc
