#!/bin/bash
# cold batch fused into the patch embedding: op/engine parity tests, then A/B bench (fused vs DDIM_COLD_FUSE_BATCH=0)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_engine_gpu.py > gpurun_out/fb_tests.log 2>&1
rc=$?; tail -4 gpurun_out/fb_tests.log; [ $rc -eq 0 ] || exit $rc
for env in X=1 DDIM_COLD_FUSE_BATCH=0 X=2 DDIM_COLD_FUSE_BATCH=0; do
  env $env timeout -k 10 200 python bench.py --no-sampler > gpurun_out/fb_bench.log 2>&1 || { tail -5 gpurun_out/fb_bench.log; exit 1; }
  echo "$env $(grep '^{' gpurun_out/fb_bench.log | cut -c1-160)"
done
