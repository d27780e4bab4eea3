#!/bin/bash
# overlap vs inline with a stand-in collective of growing cost (1 GPU, 1-rank group):
# DDIM_COLD_FAKE_COMM_REPS passes over each bucket's gradient range (~4 us each for a 2-block
# bucket) on the comm stream; the autotune's own table shows which layout it keeps
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --steps 500 --warmup 30 --no-sampler --force-dist"
for reps in 1 4 8 16; do
  timeout -k 10 120 env DDIM_COLD_FAKE_COMM=1 DDIM_COLD_FAKE_COMM_REPS=$reps $B > gpurun_out/sim_b.log 2>&1 || { tail -5 gpurun_out/sim_b.log; exit 1; }
  echo "reps=$reps $(grep '^{' gpurun_out/sim_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['ms_per_step'], c['comm_layout'], c['comm_layout_ms'])")"
done
