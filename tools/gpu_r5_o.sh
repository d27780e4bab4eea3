#!/bin/bash
# 6-stage GEMM ring: GEMM/model numerics, then a same-box A/B (DDIM_COLD_RING6=0/1) of the ViT-tiny step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5o
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_tiles_gpu.py tests/test_model_gpu.py > gpurun_out/r5o/tests.txt 2>&1 || exit $?
tail -2 gpurun_out/r5o/tests.txt
out=gpurun_out/r5o/ring6_ab.txt
: > $out
for rep in 1 2 3; do
  for r6 in 0 1; do
    timeout -k 10 200 env DDIM_COLD_RING6=$r6 python bench.py --steps 400 --warmup 40 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5o/one.json 2>/dev/null || exit $?
    echo "ring6=$r6 $(python -c 'import json,sys; print(json.loads(open(sys.argv[1]).readline())["ms_per_step"])' gpurun_out/r5o/one.json)" >> $out
    tail -1 $out
  done
done
for r6 in 0 1; do
  timeout -k 10 300 env DDIM_COLD_RING6=$r6 python bench.py --model vit_small_200 --steps 30 --warmup 5 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5o/small_$r6.json 2>/dev/null || exit $?
  echo "small ring6=$r6 $(python -c 'import json,sys; print(json.loads(open(sys.argv[1]).readline())["ms_per_step"])' gpurun_out/r5o/small_$r6.json)" >> $out
  tail -1 $out
done
