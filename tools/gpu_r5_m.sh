#!/bin/bash
# round-5 validation: the whole GPU suite, the default bench, a launch-path env A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5m
export PYTHONUNBUFFERED=1
step() {  # name, timeout, command...; stops the script on a fault / abort / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pytest 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5m/pytest_gpu.log 2>&1
step bench 400 python bench.py --steps 200 --warmup 20 > gpurun_out/r5m/bench.json 2> gpurun_out/r5m/bench.err
for rep in 1 2; do
  step kern1 200 env HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 300 --warmup 30 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5m/kernarg1_$rep.json 2>/dev/null
  step kern0 200 env HIP_FORCE_DEV_KERNARG=0 python bench.py --steps 300 --warmup 30 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5m/kernarg0_$rep.json 2>/dev/null
done
