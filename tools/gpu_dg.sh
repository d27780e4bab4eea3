#!/bin/bash
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ln_fold_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dg_tests.log 2>&1
rc=$?; tail -4 gpurun_out/dg_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_bench.sh DDIM_COLD_DGRAD_BF16 1 0
