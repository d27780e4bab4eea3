#!/bin/bash
# A/B of the fused cold batch, 1000 timed steps per run, interleaved
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for env in X=1 DDIM_COLD_FUSE_BATCH=0 X=2 DDIM_COLD_FUSE_BATCH=0 X=3 DDIM_COLD_FUSE_BATCH=0; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 50 > gpurun_out/fb_bench.log 2>&1 || { tail -5 gpurun_out/fb_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/fb_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
