#!/bin/bash
# training loss on patch rows (EPI_HEADL): GPU tests, then interleaved train A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run headl_tests 300 python -u -m pytest tests/test_sampler_rows_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread
for i in 1 2 3; do
  DDIM_COLD_TARGET_ROWS=1 run tr_rows$i 200 python bench.py --no-sampler --no-gaussian --steps 1000 --warmup 50
  DDIM_COLD_TARGET_ROWS=0 run tr_img$i 200 python bench.py --no-sampler --no-gaussian --steps 1000 --warmup 50
done
grep -ho '"ms_per_step": [0-9.]*' gpurun_out/tr_*.log
