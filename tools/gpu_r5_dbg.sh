#!/bin/bash
# fused dgrad + LayerNorm backward: NaN census per K / mode, then the new-kernel tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5d
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u tools/debug_lnbwd.py > gpurun_out/r5d/debug_lnbwd.txt 2>&1; rc=$?
echo "debug rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_model_gpu.py -k "lnbwd or fused_dgrad or qkv_att or attn" > gpurun_out/r5d/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/r5d/pytest.log; exit $rc
