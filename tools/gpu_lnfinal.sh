#!/bin/bash
# LayerNorm replica finalize folded into the embedding backward: full GPU suite, then interleaved A/B
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/lf_tests.log 2>&1
rc=$?; tail -4 gpurun_out/lf_tests.log; [ $rc -eq 0 ] || exit $rc
for env in X=1 DDIM_COLD_FUSE_LNFINAL=0 X=2 DDIM_COLD_FUSE_LNFINAL=0 X=3 DDIM_COLD_FUSE_LNFINAL=0; do
  env $env timeout -k 10 200 python bench.py --no-sampler --steps 1000 --warmup 40 > gpurun_out/lf_bench.log 2>&1 || { tail -5 gpurun_out/lf_bench.log; exit 1; }
  echo "$env $(grep "^{" gpurun_out/lf_bench.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
