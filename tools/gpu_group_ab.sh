#!/bin/bash
# group forward vs per-op forward: interleaved train-step A/B (1000 steps each)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for env in DDIM_COLD_GROUP_FWD=1 DDIM_COLD_GROUP_FWD=0 DDIM_COLD_GROUP_FWD=1 DDIM_COLD_GROUP_FWD=0 DDIM_COLD_GROUP_FWD=1 DDIM_COLD_GROUP_FWD=0; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/gab.log 2>&1 || { tail -5 gpurun_out/gab.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/gab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
done
