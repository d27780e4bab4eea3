#!/bin/bash
# A/B of two builds of this tree (DDIM_COLD_LIB=<other .so> vs the in-tree _C.so):
# REPS (default 3) interleaved pairs of training benches (BENCH_ARGS, default
# "--steps 1000 --warmup 50"), then (unless NO_DIST=1) the 2-rank one-GPU DP check
# usage: [BENCH_ARGS=...] [REPS=n] [NO_DIST=1] tools/gpu_lib_ab.sh <other.so>
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OTHER=$1
ARGS=${BENCH_ARGS:---steps 1000 --warmup 50}
run() {
  timeout -k 10 300 env "$@" > gpurun_out/lib_ab.log 2>&1 || { tail -5 gpurun_out/lib_ab.log; exit 1; }
  echo "$1 $(grep '^{' gpurun_out/lib_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
}
for rep in $(seq 1 ${REPS:-3}); do
  run X=other DDIM_COLD_LIB=$OTHER python bench.py $ARGS --no-sampler --no-vendor
  run X=tree python bench.py $ARGS --no-sampler --no-vendor
done
[ "${NO_DIST:-0}" = "1" ] && exit 0
timeout -k 10 300 python -u tools/dist2_gpu.py > gpurun_out/dist2.log 2>&1; rc=$?; tail -4 gpurun_out/dist2.log; exit $rc
