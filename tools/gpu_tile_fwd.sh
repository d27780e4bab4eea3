#!/bin/bash
# forward GEMMs (ViT-tiny shapes, M=2080 / 4160) under each forced tile
cd $GRAFT_REPO_ROOT
for tile in -1 0 1 2 3; do
  if [ $tile -ge 0 ]; then export DDIM_COLD_GEMM_TILE=$tile; else unset DDIM_COLD_GEMM_TILE; fi
  timeout -k 5 120 python tools/ub_gemm_phase.py 2>/dev/null || exit 1
done
