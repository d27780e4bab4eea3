#!/bin/bash
# full GPU suite + bench + data-parallel wire variants at 1 rank
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 || { tail -5 gpurun_out/r2_bench.log; exit 1; }
grep "^{" gpurun_out/r2_bench.log | cut -c1-400
for args in "--force-dist" "--force-dist --grad-wire bf16" "--force-dist --grad-wire bf16 --comm native"; do
  timeout -k 10 200 python bench.py --no-sampler --steps 500 --warmup 20 $args > gpurun_out/r2_dist.log 2>&1 || { tail -5 gpurun_out/r2_dist.log; exit 1; }
  echo "$args $(grep "^{" gpurun_out/r2_dist.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['allreduce'])")"
done
