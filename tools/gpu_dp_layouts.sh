#!/bin/bash
# 1-rank RCCL data-parallel step (pre-issued counter hand-offs) under every bucket size the
# cost model can pick, plus the stand-in collective pass so an early collective would show
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lay in overlap-1 overlap-3 overlap-5 overlap-7; do
  timeout -k 10 200 python bench.py --force-dist --no-sampler --no-gaussian --steps 300 --warmup 30 --comm-layout $lay > gpurun_out/dpl.log 2>&1 || { tail -5 gpurun_out/dpl.log; exit 1; }
  echo "$lay $(grep -h '^{' gpurun_out/dpl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['ms_per_step'], c['comm_layout'], c['handoff'], c['bucket_blocks'], c['final_loss'])")"
done
timeout -k 10 300 python -u tools/dist2_gpu.py > gpurun_out/dist2.log 2>&1; rc=$?; tail -2 gpurun_out/dist2.log; exit $rc
