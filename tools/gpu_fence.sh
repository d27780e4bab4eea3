#!/bin/bash
# data-parallel fork cost vs the release scope of the cross-queue synchronisation
# (1 GPU, ms/step over 1000 steps; see tools/gpu_fork2.sh for the variants)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 150 env "$@" > gpurun_out/fence_b.log 2>&1 || { tail -5 gpurun_out/fence_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/fence_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
F="DDIM_COLD_FAKE_COMM=1 DDIM_COLD_COMM_EVENTS=1"
# (ROC_SYSTEM_SCOPE_SIGNAL=0 took fork_tiny 0.995 -> 0.927 ms/step but the process then
#  exited non-zero: not usable)
for rep in 1; do
run X=single $B
run X=fork_tiny DDIM_COLD_DEBUG_FORK=1 $B
run X=fork_tiny_pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DDIM_COLD_DEBUG_FORK=1 $B
run X=fork_tiny_pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DDIM_COLD_DEBUG_FORK=1 $B
run X=ev_default $F $B --force-dist
run X=ev_dev DDIM_COLD_EVENT_FLAGS=0x40000000 $F $B --force-dist
run X=ev_nosys DDIM_COLD_EVENT_FLAGS=0x20000000 $F $B --force-dist
# (0x60000000: hipEventCreateWithFlags rejects the combination)
run X=layout_overlap2_fake DDIM_COLD_FAKE_COMM=1 $B --force-dist --comm-layout overlap-2
run X=layout_inline1_fake DDIM_COLD_FAKE_COMM=1 $B --force-dist --comm-layout inline-1
run X=layout_inline1_rccl $B --force-dist --comm-layout inline-1
run X=layout_auto_fake DDIM_COLD_FAKE_COMM=1 $B --force-dist
grep '^{' gpurun_out/fence_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['comm_layout'], d['config']['comm_layout_ms'])"
done
