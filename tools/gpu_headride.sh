#!/bin/bash
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_engine_gpu.py -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hr_tests.log 2>&1
rc=$?; echo "$(tail -1 gpurun_out/hr_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/hr_tests.log; exit $rc; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/hr_bench.log 2>&1 || { tail -5 gpurun_out/hr_bench.log; exit 1; }
  echo "head-rider $(grep "^{" gpurun_out/hr_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
