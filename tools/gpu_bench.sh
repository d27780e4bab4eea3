#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -4 gpurun_out/$name.log
  if [ $rc -gt 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi }
run bench_graph 300 python bench.py --steps 200 --warmup 20
run bench_eager 300 python bench.py --steps 50 --warmup 5 --no-graph --no-sampler
run bench_forcedist 300 python bench.py --steps 100 --warmup 10 --force-dist --no-sampler
