#!/bin/bash
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ln_fold_gpu.py tests/test_sampler_gpu.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s2_tests.log 2>&1
rc=$?; echo "$(tail -1 gpurun_out/s2_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/s2_tests.log; exit $rc; }
for rep in 1 2 3; do
for env in "DDIM_COLD_GEMM_S2=1" "DDIM_COLD_GEMM_S2=0"; do
  env $env timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-eager-baseline > gpurun_out/s2_bench.log 2>&1 || { tail -5 gpurun_out/s2_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/s2_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train', d['ms_per_step'], 'sampler ms', d['ddim_sampler_ms_per_batch'])")"
done; done
