#!/bin/bash
# iterate: kernel tests -> model tests -> bench -> rocprof kernel stats of the fused step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-4} gpurun_out/$name.log
  if [ $rc -gt 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc; }
run kernels 400 python -m pytest tests/test_kernels_gpu.py -x -q || exit 1
run model 300 python -m pytest tests/test_model_gpu.py -x -q || exit 1
run bench 300 python bench.py --steps 200 --warmup 20
export TMPDIR=/tmp
rm -rf gpurun_out/prof_step
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o run -- python3 tools/prof_step.py
