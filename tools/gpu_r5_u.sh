#!/bin/bash
# dS-materialising attention backward, take 2 (permuted 16-B dS^T stores, coalesced delta,
# dQ staged two tiles ahead): numerics, same-box A/B (DDIM_COLD_ATTN_DS), kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5u
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/r5u/tests.txt 2>&1 || exit $?
tail -2 gpurun_out/r5u/tests.txt
out=gpurun_out/r5u/ds_ab.txt
: > $out
for rep in 1 2; do
  for ds in 0 1; do
    timeout -k 10 300 env DDIM_COLD_ATTN_DS=$ds python bench.py --model vit_small_200 --steps 30 --warmup 5 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5u/one.json 2>/dev/null || exit $?
    echo "small ds=$ds $(python -c 'import json,sys; print(json.loads(open(sys.argv[1]).readline())["ms_per_step"])' gpurun_out/r5u/one.json)" >> $out
    tail -1 $out
  done
done
export TMPDIR=/tmp
DDIM_COLD_ATTN_DS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5u/prof -o run -- python bench.py --model vit_small_200 --steps 10 --warmup 3 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5u/prof.log 2>&1 || exit $?
