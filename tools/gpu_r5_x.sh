#!/bin/bash
# tail workgroups first (LN-fold loss/counter tail, wgrad grad-norm tail): full GPU suite,
# then same-box A/B (DDIM_COLD_LIB) of ViT-tiny and vit_small_200 with a ViT-tiny profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5x
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5x/pytest_gpu.log 2>&1 || exit $?
tail -2 gpurun_out/r5x/pytest_gpu.log
out=gpurun_out/r5x/ab.txt
: > $out
for rep in 1 2 3; do
  for lib in ablibs/_C_base.so tree; do
    if [ $lib = tree ]; then e=""; else e="DDIM_COLD_LIB=$lib"; fi
    timeout -k 10 200 env $e python bench.py --steps 400 --warmup 40 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5x/one.json 2>/dev/null || exit $?
    echo "tiny $lib $(python -c 'import json,sys; print(json.loads(open(sys.argv[1]).readline())["ms_per_step"])' gpurun_out/r5x/one.json)" >> $out
    tail -1 $out
  done
done
for lib in ablibs/_C_base.so tree; do
  if [ $lib = tree ]; then e=""; else e="DDIM_COLD_LIB=$lib"; fi
  timeout -k 10 300 env $e python bench.py --model vit_small_200 --steps 30 --warmup 5 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5x/one.json 2>/dev/null || exit $?
  echo "small $lib $(python -c 'import json,sys; print(json.loads(open(sys.argv[1]).readline())["ms_per_step"])' gpurun_out/r5x/one.json)" >> $out
  tail -1 $out
done
export TMPDIR=/tmp
for lib in ablibs/_C_base.so tree; do
  n=$(basename $lib .so)
  if [ $lib = tree ]; then unset DDIM_COLD_LIB; else export DDIM_COLD_LIB=$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5x/proft_$n -o run -- python bench.py --steps 100 --warmup 10 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5x/proft_$n.log 2>&1 || exit $?
done
