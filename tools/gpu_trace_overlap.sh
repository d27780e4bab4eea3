#!/bin/bash
# graph-mode kernel trace of the event-split data-parallel step with overlapped 2-block buckets
# (1 GPU; DDIM_COLD_FAKE_COMM=1: one pass per bucket on the comm stream stands in for the collective)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ov
DDIM_COLD_FAKE_COMM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ov -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler --force-dist --comm-layout overlap-2 > gpurun_out/prof_ov.log 2>&1
rc=$?; tail -2 gpurun_out/prof_ov.log | cut -c1-300; exit $rc
