#!/bin/bash
# Kernel profiles of the current tree: graph-replayed training step (-> graph_step_table)
# and the sampler's per-kernel stats (no PMC counters)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/profnow
rm -rf $O; mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run graph 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler --no-gaussian
python tools/graph_step_table.py $O/graph/run_kernel_trace.csv 20 > $O/graph_step_table.txt; tail -3 $O/graph_step_table.txt
run sampler 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sampler -o run -- python3 tools/sampler_prof.py
python tools/prof_summary.py $O/sampler/run_kernel_stats.csv 300 "DDIM sampler kernels (ViT-tiny, N=64, k=20; per denoiser step; 3 batches x 100 steps)" > $O/sampler_kernels.md
rm -f $O/graph/run_kernel_trace.csv.gz
