#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_mlp_gpu.py tests/test_kernels_gpu.py -k "mlp or head_step" -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mlp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/ub_mlp.py > gpurun_out/ub_mlp.log 2>&1; rc=$?; cat gpurun_out/ub_mlp.log | grep -v amdgpu.ids; exit $rc
