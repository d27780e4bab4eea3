#!/bin/bash
# long-sequence attention backward dropout hashes (pair-amortized): tests, then
# ub_attn of this tree vs the previous build (ab_old/_C.so), twice interleaved
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run attn_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
  TAILN=0 run ua_new$i 200 python tools/ub_attn.py
  TAILN=0 DDIM_COLD_LIB=ab_old/_C.so run ua_old$i 200 python tools/ub_attn.py
done
grep -H "p0.1" gpurun_out/ua_*.log | grep -v "N65"
