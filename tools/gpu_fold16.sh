#!/bin/bash
# 16-byte LayerNorm fold kernel: fold tests, step A/B, sampler unaffected
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ln_fold_gpu.py tests/test_group_fwd_gpu.py tests/test_engine_gpu.py > gpurun_out/f16_t.log 2>&1 || { tail -20 gpurun_out/f16_t.log; exit 1; }
tail -1 gpurun_out/f16_t.log
for rep in 1 2 3; do
  for f in 1 0; do
    DDIM_COLD_FOLD16=$f timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler > gpurun_out/f16_b.log 2>&1 || { tail -5 gpurun_out/f16_b.log; exit 1; }
    echo "fold16=$f step $(grep '^{' gpurun_out/f16_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  done
done
