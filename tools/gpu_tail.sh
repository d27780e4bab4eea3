#!/bin/bash
# whole-backward weight-gradient launch: tests, then interleaved A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or backward or engine or graph" > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
for env in DDIM_COLD_WGRAD_TAIL=1 DDIM_COLD_WGRAD_TAIL=0 DDIM_COLD_WGRAD_MULTI_S=4 DDIM_COLD_WGRAD_TAIL=1 DDIM_COLD_WGRAD_TAIL=0 DDIM_COLD_WGRAD_MULTI_S=4; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/tail_bench.log 2>&1 || { tail -5 gpurun_out/tail_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/tail_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
