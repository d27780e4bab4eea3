#!/bin/bash
# data-parallel path at 1 rank: per-bucket weight-gradient launches vs riders
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_dist_gpu.py tests/test_engine_gpu.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dpwg_tests.log 2>&1
rc=$?; echo "$(tail -1 gpurun_out/dpwg_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/dpwg_tests.log; exit $rc; }
for rep in 1 2; do
for env in "DDIM_COLD_WGRAD_BUCKET=1" "DDIM_COLD_WGRAD_BUCKET=0"; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 --force-dist > gpurun_out/dpwg_bench.log 2>&1 || { tail -5 gpurun_out/dpwg_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/dpwg_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['allreduce'])")"
done; done
