#!/bin/bash
# short attention backward (ViT-tiny): stored-flag path as a kernel template parameter:
# numerics, same-box A/B (DDIM_COLD_LIB) of ViT-tiny, per-kernel profiles
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ae
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or attn or program or autograd" > gpurun_out/r5ae/tests.txt 2>&1 || exit $?
tail -2 gpurun_out/r5ae/tests.txt
out=gpurun_out/r5ae/ab.txt
: > $out
for rep in 1 2 3 4; do
  for lib in ablibs/_C_base.so tree; do
    if [ $lib = tree ]; then e=""; else e="DDIM_COLD_LIB=$lib"; fi
    timeout -k 10 200 env $e python bench.py --steps 400 --warmup 40 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5ae/one.json 2>/dev/null || exit $?
    echo "tiny $lib $(python -c 'import json,sys; print(json.loads(open(sys.argv[1]).readline())["ms_per_step"])' gpurun_out/r5ae/one.json)" >> $out
    tail -1 $out
  done
done
export TMPDIR=/tmp
for lib in ablibs/_C_base.so tree; do
  n=$(basename $lib .so)
  if [ $lib = tree ]; then unset DDIM_COLD_LIB; else export DDIM_COLD_LIB=$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ae/proft_$n -o run -- python bench.py --steps 100 --warmup 10 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5ae/proft_$n.log 2>&1 || exit $?
done
