#!/bin/bash
# end-of-round pass: smoke, all GPU tests, bench, eager step + sampler kernel stats, graph-mode kernel trace
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PROF=1 TRAIN=0 bash tools/gpu_round.sh || exit $?
bash tools/gpu_graph_trace.sh
