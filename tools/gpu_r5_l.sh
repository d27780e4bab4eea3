#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5l
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k lnbwd_dgrad > gpurun_out/r5l/pytest.log 2>&1 || { tail -5 gpurun_out/r5l/pytest.log; exit 1; }
timeout -k 10 120 python -u tools/ub_gemm_stamps.py 2080 > gpurun_out/r5l/stamps_tiny.txt 2>&1
