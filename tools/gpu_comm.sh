#!/bin/bash
# native RCCL communicator: 1-rank parity + forced-distributed bench (torch vs native comm), then step/sampler profiles
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run dist_parity 300 python -u tools/dist_parity.py
run bench_fd_torch 200 python bench.py --force-dist --no-sampler --comm torch
run bench_fd_native 200 python bench.py --force-dist --no-sampler --comm native
run bench_fd_native_bf16 200 python bench.py --force-dist --no-sampler --comm native --grad-wire bf16
run bench 300 python bench.py
rm -rf gpurun_out/prof_step gpurun_out/prof_sampler
run prof_step 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph
run prof_sampler 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sampler -o run -- python3 tools/sampler_prof.py
