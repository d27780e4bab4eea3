#!/bin/bash
# fused QKV projection + attention (DDIM_COLD_QKV_ATTN=1) on dynamic LDS: tests + step / sampler A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DDIM_COLD_QKV_ATTN=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "qkv or program" > gpurun_out/qa_t.log 2>&1 || { tail -20 gpurun_out/qa_t.log; exit 1; }
tail -1 gpurun_out/qa_t.log
for rep in 1 2; do
  for q in 1 0; do
    DDIM_COLD_QKV_ATTN=$q timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-eager-baseline > gpurun_out/qa_b.log 2>&1 || { tail -5 gpurun_out/qa_b.log; exit 1; }
    echo "qkv_attn=$q $(grep '^{' gpurun_out/qa_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'sampler', d['ddim_sampler_ms_per_batch'])")"
  done
done
