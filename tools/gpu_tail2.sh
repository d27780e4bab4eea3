#!/bin/bash
# whole-backward wgrad tile: tests (both tiles), then interleaved A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 128 64; do
  DDIM_COLD_WGRAD_MULTI_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or backward" > gpurun_out/tail2_tests.log 2>&1
  rc=$?; echo "tile $t: $(tail -1 gpurun_out/tail2_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
for env in DDIM_COLD_WGRAD_MULTI_TILE=128 DDIM_COLD_WGRAD_MULTI_TILE=64 DDIM_COLD_WGRAD_MULTI_TILE=128 DDIM_COLD_WGRAD_MULTI_TILE=64 DDIM_COLD_WGRAD_MULTI_TILE=128 DDIM_COLD_WGRAD_MULTI_TILE=64; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/tail2_bench.log 2>&1 || { tail -5 gpurun_out/tail2_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/tail2_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
