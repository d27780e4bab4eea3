#!/bin/bash
# data-parallel path: parity tests, then single-process vs 1-rank data-parallel step time
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_dist_gpu.py tests/test_model_gpu.py > gpurun_out/dpab_test.log 2>&1 || { tail -20 gpurun_out/dpab_test.log; exit 1; }
tail -1 gpurun_out/dpab_test.log
for rep in 1 2 3; do
  for a in "" "--force-dist"; do
    timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler $a > gpurun_out/dpab.log 2>&1 || { tail -5 gpurun_out/dpab.log; exit 1; }
    echo "[$a] $(grep '^{' gpurun_out/dpab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['allreduce'], d['config']['final_loss'])")"
  done
done
