#!/bin/bash
# Multi-rank bench flow rehearsed on a 1-GPU box: 2 ranks share device 0 over gloo
# (probe_allreduce -> fitted cost model -> model-ordered autotune -> event-split
# step graphs with host-issued collectives), then the 1-rank RCCL path.
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
DDIM_COLD_REHEARSE_SHARED_GPU=1 run rehearse2 300 python bench.py --gpus 2 --steps 40 --warmup 5 --no-sampler
run bench_dp1 300 python bench.py --force-dist --no-sampler --steps 300 --warmup 30
