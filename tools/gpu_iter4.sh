#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-900
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run kernels 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q
TAILN=30 run ubench 200 python tools/ubench.py
for sp in 2 3 4; do DDIM_COLD_WGRAD_GROUP_SPLITS=$sp TAILN=1 run ub_sp$sp 200 python tools/ubench.py; done
grep -h "wgrad group" gpurun_out/ub_sp*.log | head -3
run bench 300 python bench.py
