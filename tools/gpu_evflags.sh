#!/bin/bash
# per-bucket cost of the event-split data-parallel step vs the boundary events' release scope
# (1 GPU, FAKE comm passes on the comm queue, overlapped 2-block buckets; ms/step, 1000 steps)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  timeout -k 10 150 env "$@" > gpurun_out/evf_b.log 2>&1 || { tail -5 gpurun_out/evf_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/evf_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['ms_per_step'], c['comm_layout'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler --force-dist"
export DDIM_COLD_FAKE_COMM=1
for rep in 1 2; do
run X=flags0 $B --comm-layout overlap-2
run X=release_device DDIM_COLD_EVENT_FLAGS=0x40000000 $B --comm-layout overlap-2
run X=no_system_fence DDIM_COLD_EVENT_FLAGS=0x20000000 $B --comm-layout overlap-2
run X=inline $B --comm-layout inline-1
done
