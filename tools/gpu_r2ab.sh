#!/bin/bash
# tests for the wgrad tail tiles + fused attention/proj backward, then interleaved A/Bs
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 128 64; do
  DDIM_COLD_WGRAD_MULTI_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or backward or attn" > gpurun_out/r2ab_tests.log 2>&1
  rc=$?; echo "tile $t: $(tail -1 gpurun_out/r2ab_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r2ab_tests.log; exit $rc; }
done
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2ab_tests2.log 2>&1
rc=$?; echo "engine: $(tail -1 gpurun_out/r2ab_tests2.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for env in "X=1" "DDIM_COLD_WGRAD_MULTI_TILE=64" "DDIM_COLD_ATTN_PROJ=0"; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/r2ab_bench.log 2>&1 || { tail -5 gpurun_out/r2ab_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/r2ab_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done; done
