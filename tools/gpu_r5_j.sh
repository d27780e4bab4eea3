#!/bin/bash
# LayerNorm backward as the consumer GEMM's prologue: numerics, then same-box A/Bs and a step table
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5j
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pytest 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_model_gpu.py -k "lnbwd_dgrad or prologue or program or layernorm" > gpurun_out/r5j/pytest.log 2>&1
step ab_tiny 300 python tools/ab_module_constant.py ddim_cold_amd.models.program FUSE_LN_PRO 1,0 2 -- \
  --steps 300 --warmup 30 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5j/ab_tiny.txt 2>&1
step ab_small 400 python tools/ab_module_constant.py ddim_cold_amd.models.program FUSE_LN_PRO 1,0 2 -- \
  --model vit_small_200 --steps 40 --warmup 8 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5j/ab_small.txt 2>&1
step prof_tiny 200 bash tools/gpu_prof_step.sh r5j/prof_tiny --steps 30 --warmup 10
