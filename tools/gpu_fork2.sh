#!/bin/bash
# where does the data-parallel fork cost come from? (1 GPU, ms/step, 1000 steps)
#   single          : single-process step (no buckets)
#   fork_tiny       : single-process step + a 1-element kernel on a side stream at every bucket
#                     boundary (graph fork/join topology, no work on the branch)
#   dp_fake_inline  : 1-rank DP step, each bucket's collective replaced by one elementwise pass
#                     over its range ON THE COMPUTE STREAM (no second queue)
#   dp_fake_graph   : same pass on the comm stream, captured as a graph branch
#   dp_rccl         : 1-rank DP step with the real (1-rank) RCCL collectives captured
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 150 env "$@" > gpurun_out/fork2_b.log 2>&1 || { tail -5 gpurun_out/fork2_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/fork2_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
for rep in 1 2; do
run X=single $B
run X=fork_tiny DDIM_COLD_DEBUG_FORK=1 $B
run X=dp_fake_inline DDIM_COLD_FAKE_COMM=1 DDIM_COLD_COMM_INLINE=1 $B --force-dist
run X=dp_fake_graph DDIM_COLD_FAKE_COMM=1 $B --force-dist
run X=dp_rccl $B --force-dist
run X=dp_rccl_inline DDIM_COLD_COMM_INLINE=1 $B --force-dist
done
