#!/bin/bash
# vit_small_200 training step under each forced GEMM tile (large-M shapes: M = 20,032)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
for tile in -1 1 2 3; do
  if [ $tile -ge 0 ]; then export DDIM_COLD_GEMM_TILE=$tile; else unset DDIM_COLD_GEMM_TILE; fi
  timeout -k 10 200 python bench.py --model vit_small_200 --steps 20 --warmup 5 --no-sampler --no-gaussian > gpurun_out/th.log 2>&1 || { tail -3 gpurun_out/th.log; exit 1; }
  echo "tile=$tile $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/th.log)"
done
