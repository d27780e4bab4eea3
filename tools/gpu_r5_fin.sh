#!/bin/bash
# round-5 final validation (after the attention dropout changes): the whole GPU suite, the default bench,
# the vit_small_200 bench, and step tables of both models
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5fin
export PYTHONUNBUFFERED=1
step() {  # name, timeout, command...; stops the script on a fault / abort / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pytest 700 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5fin/pytest_gpu.log 2>&1
tail -2 gpurun_out/r5fin/pytest_gpu.log
step bench 400 python bench.py > gpurun_out/r5fin/bench.json 2> gpurun_out/r5fin/bench.err
step bench200 400 python bench.py --steps 200 --warmup 20 > gpurun_out/r5fin/bench200.json 2> gpurun_out/r5fin/bench200.err
step small 400 python bench.py --model vit_small_200 --steps 30 --warmup 5 > gpurun_out/r5fin/small.json 2> gpurun_out/r5fin/small.err
step proftiny 450 bash tools/gpu_prof_step.sh r5fin/prof_tiny --steps 40 --warmup 10
step profsmall 450 bash tools/gpu_prof_step.sh r5fin/prof_small --model vit_small_200 --steps 15 --warmup 3
