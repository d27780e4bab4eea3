#!/bin/bash
# same-box A/B of builds (DDIM_COLD_LIB): round-start hash / vector rng / no stamps / this tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5n
export PYTHONUNBUFFERED=1
out=gpurun_out/r5n/libs_ab.txt
: > $out
for rep in 1 2 3; do
  for lib in ablibs/_C_pre_dropmix.so ablibs/_C_hashonly.so ablibs/_C_nostamps.so ablibs/_C_vecrng.so tree; do
    if [ $lib = tree ]; then e=""; else e="DDIM_COLD_LIB=$lib"; fi
    timeout -k 10 200 env $e python bench.py --steps 400 --warmup 40 --no-sampler --no-vendor --no-gaussian > gpurun_out/r5n/one.json 2>/dev/null || exit $?
    echo "$lib $(head -1 gpurun_out/r5n/one.json | python -c 'import json,sys; print(json.loads(sys.stdin.readline())["ms_per_step"])')" >> $out
    tail -1 $out
  done
done
