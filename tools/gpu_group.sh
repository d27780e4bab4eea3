#!/bin/bash
# image-group persistent forward: bit-exactness tests, then train/sampler A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_group_fwd_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/group_tests.log 2>&1
rc=$?; tail -12 gpurun_out/group_tests.log; [ $rc -eq 0 ] || exit $rc
for env in DDIM_COLD_GROUP_FWD=1 DDIM_COLD_GROUP_FWD=0 DDIM_COLD_GROUP_FWD=1 DDIM_COLD_GROUP_FWD=0; do
  env $env timeout -k 10 200 python bench.py --steps 500 --warmup 20 --no-eager-baseline > gpurun_out/group_bench.log 2>&1 || { tail -5 gpurun_out/group_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/group_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train', d['ms_per_step'], 'sampler ms', d['ddim_sampler_ms_per_batch'])")"
done
