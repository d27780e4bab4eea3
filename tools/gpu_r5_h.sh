#!/bin/bash
# late epilogue prefetch (residual / DGELU GEMMs): GEMM + model numerics, stamps, both benches
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5h
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_tiles_gpu.py \
  tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/r5h/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r5h/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ub_gemm_stamps.py 20032 > gpurun_out/r5h/stamps_small.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-vendor --no-sampler --no-gaussian > gpurun_out/r5h/bench.json 2> gpurun_out/r5h/bench.err || exit $?
timeout -k 10 300 python bench.py --model vit_small_200 --steps 40 --warmup 8 --no-vendor --no-sampler --no-gaussian > gpurun_out/r5h/bench_small.json 2> gpurun_out/r5h/bench_small.err
