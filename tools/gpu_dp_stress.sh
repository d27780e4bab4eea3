#!/bin/bash
# repeated data-parallel bench runs (1-rank RCCL group, collectives captured): every run must
# exit 0 with the collectives captured (no watchdog abort, no capture fallback)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/dps_test.log 2>&1 || { tail -20 gpurun_out/dps_test.log; exit 1; }
tail -1 gpurun_out/dps_test.log
for i in $(seq 1 ${N:-8}); do
  timeout -k 10 150 python bench.py --steps 30 --warmup 10 --no-sampler --force-dist $EXTRA > gpurun_out/dps_$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc $(grep -o '"allreduce": "[a-z-]*"' gpurun_out/dps_$i.log) fallback=$(grep -c 'falling back' gpurun_out/dps_$i.log) watchdog=$(grep -c 'watchdog' gpurun_out/dps_$i.log)"
  [ $rc -eq 0 ] || exit $rc
done
