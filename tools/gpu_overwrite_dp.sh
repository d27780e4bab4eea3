#!/bin/bash
# gradient overwrite in the data-parallel step (1-rank RCCL group): parity + step A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_dist_gpu.py tests/test_engine_gpu.py > gpurun_out/owdp_test.log 2>&1 || { tail -30 gpurun_out/owdp_test.log; exit 1; }
tail -1 gpurun_out/owdp_test.log
for rep in 1 2 3; do
  for k in 1 0; do
    DDIM_COLD_GRAD_OVERWRITE=$k timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler --force-dist > gpurun_out/owdp_b.log 2>&1 || { tail -5 gpurun_out/owdp_b.log; exit 1; }
    echo "dp overwrite=$k $(grep '^{' gpurun_out/owdp_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['allreduce'], d['config']['final_loss'])")"
  done
done
