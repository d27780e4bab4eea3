#!/bin/bash
# comm=auto (verified native RCCL communicator) on one GPU: parity, then 1-rank DP ms/step
# torch vs auto, and the 2-rank gloo one-GPU check (auto falls back to torch on gloo)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dist_parity.py > gpurun_out/dist_parity.log 2>&1 || { tail -20 gpurun_out/dist_parity.log; exit 1; }
tail -2 gpurun_out/dist_parity.log
timeout -k 10 300 python -u tools/dist2_gpu.py > gpurun_out/dist2.log 2>&1 || { tail -20 gpurun_out/dist2.log; exit 1; }
tail -2 gpurun_out/dist2.log
run() {
  timeout -k 10 150 env "$@" > gpurun_out/na_b.log 2>&1 || { tail -5 gpurun_out/na_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/na_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['ms_per_step'], c['comm'], c['comm_layout'], c['comm_layout_ms'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler --force-dist"
for rep in 1 2; do
run X=torch $B --comm torch
run X=auto $B
run X=auto_fake DDIM_COLD_FAKE_COMM=1 $B
done
