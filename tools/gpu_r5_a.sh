#!/bin/bash
# round-5 data-parallel checks on one GPU: new hand-off tests, --force-dist bench
# (autotune incl. the captured inline layout), a forced hand-off failure, single process
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5a
export PYTHONUNBUFFERED=1
step() {  # name, timeout, command...; stops the script on a fault / abort / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pytest 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pair_handoff_gpu.py \
  tests/test_engine_gpu.py -k "pair or stepped or multi_step" > gpurun_out/r5a/pytest_new.log 2>&1
step force_dist 300 python bench.py --force-dist --steps 200 --warmup 20 --no-sampler --no-vendor --no-gaussian \
  > gpurun_out/r5a/bench_force_dist.json 2> gpurun_out/r5a/bench_force_dist.err
DDIM_COLD_TEST_HANDOFF_SKEW=1 step skew 300 python bench.py --force-dist --steps 100 --warmup 10 --no-sampler \
  --no-vendor --no-gaussian > gpurun_out/r5a/bench_skew.json 2> gpurun_out/r5a/bench_skew.err
step single 300 python bench.py --steps 200 --warmup 20 --no-sampler --no-vendor --no-gaussian \
  > gpurun_out/r5a/bench_single.json 2> gpurun_out/r5a/bench_single.err
