#!/bin/bash
# graph-mode kernel trace of the data-parallel step on one GPU (1-rank RCCL group, collectives
# captured; DDIM_COLD_FAKE_COMM=1 from the caller swaps each collective for one pass over its range)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_graph_dp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graph_dp -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler --force-dist "$@" > gpurun_out/prof_graph_dp.log 2>&1
rc=$?; tail -2 gpurun_out/prof_graph_dp.log; exit $rc
