#!/bin/bash
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for env in "X=1" "DDIM_COLD_FAKE_COMM=1" "DDIM_COLD_FAKE_COMM=1 DDIM_COLD_COMM_SIGNAL=event"; do
  timeout -k 10 120 env $env python -u tools/host_timing.py --layout overlap-2 > gpurun_out/ht.log 2>&1 || { tail -5 gpurun_out/ht.log; exit 1; }
  grep "^layout" gpurun_out/ht.log
done
timeout -k 10 120 python -u tools/host_timing.py --layout inline-1 > gpurun_out/ht.log 2>&1 || { tail -5 gpurun_out/ht.log; exit 1; }
grep "^layout" gpurun_out/ht.log
