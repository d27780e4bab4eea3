#!/bin/bash
# data-parallel step graph (1-rank RCCL group): HIP graph queue settings vs the single-process graph
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 1000 --warmup 50 --no-sampler $DPARGS > gpurun_out/dpq.log 2>&1 || { tail -5 gpurun_out/dpq.log; exit 1; }
  echo "$label $(grep '^{' gpurun_out/dpq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['allreduce'])")"
}
for rep in 1 2; do
  DPARGS="" run single X=1
  DPARGS="--force-dist" run dp-default X=1
  DPARGS="--force-dist" run dp-queues1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
  DPARGS="--force-dist" run dp-queues2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
  DPARGS="--force-dist --graph-steps 1" run dp-K1 X=1
  DPARGS="--force-dist --bucket-blocks 4" run dp-bb4 X=1
  DPARGS="--force-dist --bucket-blocks 7" run dp-bb7 X=1
done
