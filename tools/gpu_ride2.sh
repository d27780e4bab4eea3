#!/bin/bash
# rider token-split sweep + data-parallel path overhead at 1 rank (captured RCCL / segmented)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
b() { # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 "$@" > gpurun_out/r2_$name.log 2>&1 || { tail -5 gpurun_out/r2_$name.log; exit 1; }
  echo "$name $envs $* $(grep "^{" gpurun_out/r2_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['allreduce'])")"
}
b ride160 "DDIM_COLD_WGRAD_RIDE=1"
b ride64 "DDIM_COLD_RIDE_WG=64"
b ride320 "DDIM_COLD_RIDE_WG=320"
b noride "DDIM_COLD_WGRAD_RIDE=0"
b ride64b "DDIM_COLD_RIDE_WG=64"
b ride160b "DDIM_COLD_WGRAD_RIDE=1"
b dist "X=1" --force-dist
b dist_bf16 "X=1" --force-dist --grad-wire bf16
b dist_native "X=1" --force-dist --comm native
b dist_seg "X=1" --force-dist --segmented-comm
b dist_b7 "X=1" --force-dist --bucket-blocks 7
