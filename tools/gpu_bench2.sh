#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "" "--no-graph" "--no-wgrad-stream" "--no-graph --no-wgrad-stream"; do
  echo "=== cfg: $cfg"
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-sampler $cfg > gpurun_out/b2.log 2>&1; rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/b2.log; exit $rc; fi
  tail -1 gpurun_out/b2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
