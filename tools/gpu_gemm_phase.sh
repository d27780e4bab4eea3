#!/bin/bash
# forward GEMM phases (main loop / epilogue) at sampler + training shapes
cd $GRAFT_REPO_ROOT
for d in 0 1 2; do
  DDIM_COLD_GEMM_DEBUG=$d timeout -k 5 120 python tools/ub_gemm_phase.py 2>/dev/null || exit 1
done
