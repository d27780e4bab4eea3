#!/bin/bash
# data-parallel bench (1-rank RCCL group, collectives captured in the step graph): clean exit?
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 10 --no-sampler --force-dist > gpurun_out/dpx_$i.log 2>&1
  rc=$?; echo "plain run $i rc=$rc $(grep -c 'watchdog' gpurun_out/dpx_$i.log) watchdog lines"; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/prof_dpx
TORCH_NCCL_CUDA_EVENT_CACHE=0 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dpx -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler --force-dist > gpurun_out/dpx_prof.log 2>&1
rc=$?; echo "profiled, event cache off: rc=$rc $(grep -c 'watchdog' gpurun_out/dpx_prof.log) watchdog lines"; exit $rc
