#!/bin/bash
# kernel tests + ubench + bench (graph) ; optional rocprof of eager bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-900
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run kernels 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q
TAILN=40 run ubench 200 python tools/ubench.py
run bench 300 python bench.py
if [ "$PROF" = "1" ]; then
  export TMPDIR=/tmp; rm -rf gpurun_out/prof_bench
  run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph
fi
