#!/bin/bash
# GEMM phase stamps at the vit_small_200 and ViT-tiny shapes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5g
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/ub_gemm_stamps.py 20032 > gpurun_out/r5g/stamps_small.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/ub_gemm_stamps.py 2080 > gpurun_out/r5g/stamps_tiny.txt 2>&1
