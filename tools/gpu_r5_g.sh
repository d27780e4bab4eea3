#!/bin/bash
# GEMM phase stamps at the vit_small_200 shapes for several tile configs, and ViT-tiny
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5g
export PYTHONUNBUFFERED=1
timeout -k 10 180 python -u tools/ub_gemm_stamps.py 20032 -1,4,5,3,2,1 > gpurun_out/r5g/stamps_small_tiles.txt 2>&1
