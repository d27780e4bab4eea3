#!/bin/bash
# sampler / train time vs forced GEMM tile config (DDIM_COLD_GEMM_TILE) and the cost model
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
one() {
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-eager-baseline > gpurun_out/ts.log 2>&1 || { tail -3 gpurun_out/ts.log; return 1; }
  grep "^{" gpurun_out/ts.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', 'train', d['ms_per_step'], 'sampler', d.get('ddim_sampler_ms_per_batch'))"
}
one X=0 && one DDIM_COLD_GEMM_TILE=0 && one DDIM_COLD_GEMM_TILE=1 && one DDIM_COLD_GEMM_TILE=2 && one DDIM_COLD_GEMM_TILE=3 && one DDIM_COLD_GEMM_TILE_MODEL=1
