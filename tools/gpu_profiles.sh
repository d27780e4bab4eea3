#!/bin/bash
# refresh the committed profiles: graph-mode kernel traces (single process, data parallel
# 1-rank default path) and per-kernel stats (eager step, sampler)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_graph gpurun_out/prof_graph_dp gpurun_out/prof_step gpurun_out/prof_sampler
run() { local name=$1; shift
  echo "=== $name"; timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$name.log; echo "STOP after $name"; exit $rc; fi; }
run prof_graph rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graph -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler
run prof_graph_dp rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_graph_dp -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler --force-dist
run prof_step rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph
run prof_sampler rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sampler -o run -- python3 tools/sampler_prof.py
run bench python bench.py
grep '^{' gpurun_out/bench.log | cut -c1-300
