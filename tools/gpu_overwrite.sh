#!/bin/bash
# gradient overwrite (single writer per range, AdamW zeroes only the embeddings): tests + step A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "engine or overwrite or wgrad_multi or replica or graph" > gpurun_out/ow_test.log 2>&1 || { tail -30 gpurun_out/ow_test.log; exit 1; }
tail -1 gpurun_out/ow_test.log
for rep in 1 2 3; do
  for k in 1 0; do
    DDIM_COLD_GRAD_OVERWRITE=$k timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler > gpurun_out/ow_b.log 2>&1 || { tail -5 gpurun_out/ow_b.log; exit 1; }
    echo "overwrite=$k $(grep '^{' gpurun_out/ow_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['final_loss'])")"
  done
done
