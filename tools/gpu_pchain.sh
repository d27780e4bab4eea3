#!/bin/bash
# sampler patch-row chain: tests, then sampler ms/batch with the chain on / off (interleaved)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_sampler_gpu.py tests/test_group_fwd_gpu.py > gpurun_out/pchain_test.log 2>&1 || { tail -30 gpurun_out/pchain_test.log; exit 1; }
tail -1 gpurun_out/pchain_test.log
for rep in 1 2 3; do
  for on in 1 0; do
    DDIM_COLD_SAMPLER_PATCH_CHAIN=$on timeout -k 10 200 python bench.py --steps 2 --warmup 2 --no-eager-baseline > gpurun_out/pchain_b.log 2>&1 || { tail -5 gpurun_out/pchain_b.log; exit 1; }
    echo "chain=$on $(grep '^{' gpurun_out/pchain_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sampler ms', d['ddim_sampler_ms_per_batch'])")"
  done
done
