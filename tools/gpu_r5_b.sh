#!/bin/bash
# round-5 validation on one GPU: the whole GPU test suite, the fp32-oracle error report
# of the round-5 configs, the full bench (new vendor img2img key), the e2e trainer demo
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5b
export PYTHONUNBUFFERED=1
step() {  # name, timeout, command...; stops the script on a fault / abort / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pytest 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5b/pytest_gpu.log 2>&1
step report 300 python -u tools/grad_error_report.py r5 > gpurun_out/r5b/grad_error_r5.txt 2>&1
step bench 400 python bench.py --steps 200 --warmup 20 > gpurun_out/r5b/bench.json 2> gpurun_out/r5b/bench.err
step e2e 600 bash tools/gpu_e2e_demo.sh > gpurun_out/r5b/e2e.log 2>&1
