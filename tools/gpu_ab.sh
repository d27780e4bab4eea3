#!/bin/bash
# A/B of an env switch on the 1-GPU bench:  tools/gpu_ab.sh "VAR=a" "VAR=b" [tests]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
if [ -n "$3" ]; then
  timeout -k 10 600 python -m pytest tests/ -x -q -m gpu $3 > gpurun_out/ab/pytest.log 2>&1 || { tail -40 gpurun_out/ab/pytest.log; exit 1; }
  tail -1 gpurun_out/ab/pytest.log
fi
for round in 1 2; do
  for v in "$1" "$2"; do
    env $v timeout -k 10 300 python bench.py --steps 200 --warmup 30 --no-sampler > gpurun_out/ab/bench.log 2>&1 || { tail -30 gpurun_out/ab/bench.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/bench.log)"
  done
done
