#!/bin/bash
# A/B of two builds of this tree (DDIM_COLD_LIB=<other .so> vs the in-tree _C.so),
# 3 interleaved pairs of 1000-step training benches; then the 2-rank one-GPU DP check
# usage: tools/gpu_lib_ab.sh <other.so>
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OTHER=$1
run() {
  timeout -k 10 150 env "$@" > gpurun_out/lib_ab.log 2>&1 || { tail -5 gpurun_out/lib_ab.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/lib_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
for rep in 1 2 3; do
run X=other DDIM_COLD_LIB=$OTHER $B
run X=tree $B
done
timeout -k 10 300 python -u tools/dist2_gpu.py > gpurun_out/dist2.log 2>&1; rc=$?; tail -4 gpurun_out/dist2.log; exit $rc
