#!/bin/bash
# tests + bench (with eager sampler baseline) + rocprof kernel stats of the training step and the sampler
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-1200
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run kernels 400 python -m pytest tests -m gpu -x -q
TAILN=30 run ubench 200 python tools/ubench.py
run bench 400 python bench.py
export TMPDIR=/tmp
rm -rf gpurun_out/prof_step gpurun_out/prof_sampler
run prof_step 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph
run prof_sampler 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sampler -o run -- python3 tools/sampler_prof.py
