#!/bin/bash
# attention keep flags stored by the forward: kernel tests, micro-benchmark, interleaved step A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/keep_tests.log 2>&1 || { tail -20 gpurun_out/keep_tests.log; exit 1; }
tail -2 gpurun_out/keep_tests.log
(cd tools && timeout -k 10 200 python -u ub_drop.py) > gpurun_out/keep_ub.log 2>&1 || { tail -5 gpurun_out/keep_ub.log; exit 1; }
grep " us " gpurun_out/keep_ub.log
for rep in 1 2 3; do
  for k in 1 0; do
    DDIM_COLD_ATTN_KEEP=$k timeout -k 10 200 python bench.py --steps 1000 --warmup 50 --no-sampler > gpurun_out/keep_b.log 2>&1 || { tail -5 gpurun_out/keep_b.log; exit 1; }
    echo "keep=$k $(grep '^{' gpurun_out/keep_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['final_loss'])")"
  done
done
