#!/bin/bash
# K-step graphs: engine parity tests, then interleaved A/B of --graph-steps 1 / 4 / 8 (1000 timed steps each)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_engine_gpu.py > gpurun_out/gs_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gs_tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 4 8 1 4 8; do
  timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 --graph-steps $k > gpurun_out/gs_bench.log 2>&1 || { tail -5 gpurun_out/gs_bench.log; exit 1; }
  echo "K=$k $(grep "^{" gpurun_out/gs_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
