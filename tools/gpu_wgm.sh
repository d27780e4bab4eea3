#!/bin/bash
# whole-backward weight-gradient launch: tile configs (correctness, micro-benchmark, step A/B)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 64 12864 128642; do
  DDIM_COLD_WGRAD_MULTI_TILE=$c timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k wgrad_multi > gpurun_out/wgm_t_$c.log 2>&1 || { echo "tile $c test FAILED"; tail -20 gpurun_out/wgm_t_$c.log; exit 1; }
  echo "tile $c: $(tail -1 gpurun_out/wgm_t_$c.log)"
  DDIM_COLD_WGRAD_MULTI_TILE=$c timeout -k 10 200 python -u tools/ub_wgrad_multi.py > gpurun_out/wgm_u_$c.log 2>&1 || { tail -5 gpurun_out/wgm_u_$c.log; exit 1; }
  grep "full\|1 block" gpurun_out/wgm_u_$c.log | sed "s/^/tile $c: /"
done
for rep in 1 2 3; do
  for c in 64 12864 128642; do
    DDIM_COLD_WGRAD_MULTI_TILE=$c timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler > gpurun_out/wgm_b.log 2>&1 || { tail -5 gpurun_out/wgm_b.log; exit 1; }
    echo "tile $c step $(grep '^{' gpurun_out/wgm_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  done
done
