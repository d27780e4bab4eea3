#!/bin/bash
# QKV input-gradient K-split count A/B (DDIM_COLD_QKV_DGRAD_SPLITS)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for q in 1 2 3 4; do
    DDIM_COLD_QKV_DGRAD_SPLITS=$q timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler > gpurun_out/qs_b.log 2>&1 || { tail -5 gpurun_out/qs_b.log; exit 1; }
    echo "splits $q step $(grep '^{' gpurun_out/qs_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  done
done
