#!/bin/bash
# GEMM phase study on the forward shapes (tools/ub_gemm_phase.py) under the
# debug / tile switches, plus the lazy-max attention test
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gemm
O=gpurun_out/gemm
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-2} $O/$name.log | cut -c1-700
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run lazy_test 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "lazy_max or spike or attention_fwd_bwd" --timeout 120 --timeout-method thread
TAILN=1 run ph_default 120 python tools/ub_gemm_phase.py
TAILN=1 run ph_dbg1 120 env DDIM_COLD_GEMM_DEBUG=1 python tools/ub_gemm_phase.py
TAILN=1 run ph_dbg2 120 env DDIM_COLD_GEMM_DEBUG=2 python tools/ub_gemm_phase.py
for t in 0 1 2 3; do TAILN=1 run ph_t$t 120 env DDIM_COLD_GEMM_TILE=$t python tools/ub_gemm_phase.py; done
for t in 2 3; do TAILN=1 run ph_t${t}_dbg1 120 env DDIM_COLD_GEMM_TILE=$t DDIM_COLD_GEMM_DEBUG=1 python tools/ub_gemm_phase.py; done
