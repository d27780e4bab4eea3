#!/bin/bash
# sampler A/B: current tree vs ab_old/ (a previous commit's package + its _C.so), interleaved
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  for d in . ab_old; do
    (cd $d && timeout -k 10 200 python bench.py --steps 2 --warmup 2 --no-eager-baseline) > gpurun_out/sab.log 2>&1 || { tail -5 gpurun_out/sab.log; exit 1; }
    echo "$d $(grep "^{" gpurun_out/sab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sampler ms', d['ddim_sampler_ms_per_batch'])")"
  done
done
