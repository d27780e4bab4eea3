#!/bin/bash
# atomic-add throughput for the dQ accumulation idea; re-run of the tests fixed after r5e
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5f
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./tools/ub_atomic.bin > gpurun_out/r5f/ub_atomic.txt 2>&1; rc=$?; echo "ub_atomic rc=$rc"; cat gpurun_out/r5f/ub_atomic.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_engine_gpu.py \
  tests/test_trainer_overlap_gpu.py -k "stepped or overlapped" > gpurun_out/r5f/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r5f/pytest.log; exit $rc
