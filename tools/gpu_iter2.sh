#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log
  if [ $rc -gt 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc; }
run kernels 400 python -m pytest tests/test_kernels_gpu.py -x -q || exit 1
run model 300 python -m pytest tests/test_model_gpu.py -x -q || exit 1
run bench 300 python bench.py --steps 200 --warmup 20 --no-sampler
run ubench 200 python tools/ubench.py
for sp in 2 4 8 16; do DDIM_COLD_WGRAD_SPLITS=$sp timeout -k 10 100 python tools/ubench.py 2>&1 | grep wgrad | sed "s/^/splits=$sp /"; done
bash tools/gpu_pmc.sh
