#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wg
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_gemm_tiles_gpu.py tests/test_engine_gpu.py -x -q -m gpu > gpurun_out/wg/pytest.log 2>&1 || { tail -40 gpurun_out/wg/pytest.log; exit 1; }
tail -1 gpurun_out/wg/pytest.log
DDIM_COLD_WGRAD_GROUP_SPLITS=1 timeout -k 10 120 python tools/ub_wgrad_k.py > gpurun_out/wg/k.log 2>&1 || { tail -20 gpurun_out/wg/k.log; exit 1; }
grep T= gpurun_out/wg/k.log
for s in 1 2 3; do
  DDIM_COLD_WGRAD_GROUP_SPLITS=$s timeout -k 10 120 python tools/ub_wgrad.py > gpurun_out/wg/u.log 2>&1 || { tail -20 gpurun_out/wg/u.log; exit 1; }
  grep splits gpurun_out/wg/u.log
done
timeout -k 10 120 python tools/ubench.py > gpurun_out/wg/ubench.log 2>&1 || { tail -20 gpurun_out/wg/ubench.log; exit 1; }
grep -i "dgrad\|wgrad\|resid\|qkv\|gelu" gpurun_out/wg/ubench.log
timeout -k 10 300 python bench.py --steps 200 --warmup 30 --no-sampler > gpurun_out/wg/bench.log 2>&1 || { tail -30 gpurun_out/wg/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/wg/bench.log
