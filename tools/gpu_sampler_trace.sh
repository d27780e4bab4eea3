#!/bin/bash
# graph-mode kernel trace of the DDIM sampler (k=20, N=64): per-kernel time per denoiser step
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_smp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_smp -o run -- python3 tools/ub_sampler.py PATCH_CHAIN 3 1 > gpurun_out/prof_smp.log 2>&1
rc=$?; tail -2 gpurun_out/prof_smp.log; exit $rc
