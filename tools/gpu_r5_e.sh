#!/bin/bash
# round-5 state check: the whole GPU test suite, both benches, step tables of both models
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5e
export PYTHONUNBUFFERED=1
step() {  # name, timeout, command...; stops the script on a fault / abort / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pytest 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5e/pytest_gpu.log 2>&1
step bench 300 python bench.py --steps 200 --warmup 20 --no-vendor > gpurun_out/r5e/bench.json 2> gpurun_out/r5e/bench.err
step bench_small 300 python bench.py --model vit_small_200 --steps 40 --warmup 8 --no-vendor --no-sampler > gpurun_out/r5e/bench_small.json 2> gpurun_out/r5e/bench_small.err
step prof_tiny 200 bash tools/gpu_prof_step.sh r5e/prof_tiny --steps 30 --warmup 10
step prof_small 200 bash tools/gpu_prof_step.sh r5e/prof_small --model vit_small_200 --steps 20 --warmup 5
