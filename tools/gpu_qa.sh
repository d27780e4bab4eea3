#!/bin/bash
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ln_fold_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qa_tests.log 2>&1
rc=$?; tail -25 gpurun_out/qa_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_bench.sh DDIM_COLD_QKV_ATTN 1 0
