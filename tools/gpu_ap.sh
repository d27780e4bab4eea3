#!/bin/bash
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "attn or backward" > gpurun_out/ap_tests.log 2>&1
rc=$?; echo "$(tail -1 gpurun_out/ap_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ap_tests.log; exit $rc; }
for rep in 1 2 3; do
for env in "DDIM_COLD_ATTN_PROJ=1" "DDIM_COLD_ATTN_PROJ=0"; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/ap_bench.log 2>&1 || { tail -5 gpurun_out/ap_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/ap_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done; done
