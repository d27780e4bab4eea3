#!/bin/bash
# GEMM ordering experiment: tile tests only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5i
timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gemm_tiles_gpu.py > gpurun_out/r5i/pytest.log 2>&1; rc=$?
tail -12 gpurun_out/r5i/pytest.log | grep -v "^$"; exit $rc
