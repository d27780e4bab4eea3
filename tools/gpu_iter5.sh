#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-900
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run kernels 400 python -m pytest tests -m gpu -x -q
TAILN=32 run ubench 200 python tools/ubench.py
DDIM_COLD_LN_GEMM_BM=64 TAILN=1 run ub_bm64 200 python tools/ubench.py
run bench 400 python bench.py --no-eager-baseline
DDIM_COLD_LN_GEMM_BM=64 run bench64 400 python bench.py --no-eager-baseline
