#!/bin/bash
# dynamic-LDS attention / LayerNorm backward: kernel tests, micro-benchmarks, step time
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/dl_t.log 2>&1 || { tail -20 gpurun_out/dl_t.log; exit 1; }
tail -1 gpurun_out/dl_t.log
(cd tools && timeout -k 10 120 python -u ub_drop.py) > gpurun_out/dl_ub.log 2>&1 || { tail -5 gpurun_out/dl_ub.log; exit 1; }
grep "ln bwd\|attn bwd" gpurun_out/dl_ub.log | head -4
for rep in 1 2 3; do
  for c in 0 2 3; do
    DDIM_COLD_LN_BWD_CFG=$c timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler > gpurun_out/dl_b.log 2>&1 || { tail -5 gpurun_out/dl_b.log; exit 1; }
    echo "ln_bwd cfg $c step $(grep '^{' gpurun_out/dl_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  done
done
