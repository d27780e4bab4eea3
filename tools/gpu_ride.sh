#!/bin/bash
# Weight-gradient riders in the dgrad launches: new tests, interleaved A/B, kernel profile
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ride_tests.log 2>&1
rc=$?; tail -4 gpurun_out/ride_tests.log; [ $rc -eq 0 ] || exit $rc
for env in DDIM_COLD_WGRAD_RIDE=1 DDIM_COLD_WGRAD_RIDE=0 DDIM_COLD_WGRAD_RIDE=1 DDIM_COLD_WGRAD_RIDE=0 DDIM_COLD_WGRAD_RIDE=1 DDIM_COLD_WGRAD_RIDE=0 ${EXTRA_AB}; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/ride_bench.log 2>&1 || { tail -5 gpurun_out/ride_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/ride_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ride
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ride -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph > gpurun_out/prof_ride.log 2>&1
echo "prof rc=$?"
