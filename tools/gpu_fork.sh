#!/bin/bash
# data-parallel step topology on one GPU: 1-rank group, each bucket's collective replaced
# by one elementwise pass over its range (DDIM_COLD_FAKE_COMM=1) so the step has the
# data-parallel fork / join shape: event-split graphs vs a comm branch in the graph
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 150 env "$@" > gpurun_out/fork_b.log 2>&1 || { tail -5 gpurun_out/fork_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/fork_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
export DDIM_COLD_FAKE_COMM=1
timeout -k 10 300 python tools/dist_parity.py > gpurun_out/dist_parity.log 2>&1 || { tail -20 gpurun_out/dist_parity.log; exit 1; }
tail -2 gpurun_out/dist_parity.log
for rep in 1 2; do
run X=single $B
run X=dp_events $B --force-dist
run X=dp_events $B --force-dist --bucket-blocks 1
run X=dp_events $B --force-dist --bucket-blocks 4
run X=dp_graph DDIM_COLD_COMM_EVENTS=0 $B --force-dist
run X=dp_events_native $B --force-dist --comm native
done
