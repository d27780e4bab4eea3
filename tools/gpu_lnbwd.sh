#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ln
for c in 0 4 6 7; do
  DDIM_COLD_LN_BWD_CFG=$c DDIM_COLD_LN_FWD_WAVES=$((c==0?4:c==4?8:c==6?16:2)) timeout -k 10 120 python tools/ub_lnbwd.py > gpurun_out/ln/ub$c.log 2>&1 || { tail -20 gpurun_out/ln/ub$c.log; exit 1; }; grep "cfg\|fwd" gpurun_out/ln/ub$c.log
done
for c in 4 6 7; do
  DDIM_COLD_LN_BWD_CFG=$c timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "layernorm" > gpurun_out/ln/pytest$c.log 2>&1 || { tail -30 gpurun_out/ln/pytest$c.log; exit 1; }
  tail -1 gpurun_out/ln/pytest$c.log
done
for w in 2 8 16; do
  DDIM_COLD_LN_FWD_WAVES=$w timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "layernorm" > gpurun_out/ln/pytestf$w.log 2>&1 || { tail -30 gpurun_out/ln/pytestf$w.log; exit 1; }
  tail -1 gpurun_out/ln/pytestf$w.log
done
