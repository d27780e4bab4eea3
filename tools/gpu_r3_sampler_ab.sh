#!/bin/bash
# Sampler A/B (3 interleaved rounds, tools/ub_sampler_lib.py-style: one process per
# build per round) + the high-resolution / OxfordFlower benches of the tree.
# usage: tools/gpu_r3_sampler_ab.sh <other.so>
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
O=gpurun_out/sab; mkdir -p $O
OTHER=$1
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
for r in 1 2 3; do for L in $OTHER ddim_cold_amd/_C.so; do
  n=$(basename $L .so)_$r
  run s_$n 200 env DDIM_COLD_LIB=$L python bench.py --steps 10 --warmup 2 --no-eager-baseline
  grep '^{' $O/s_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n sampler ms', d['ddim_sampler_ms_per_batch'], 'img2img ms', d['draft2drawing_ms'])"
done; done
run hires 400 python bench.py --model vit_small_200 --steps 30 --warmup 10
grep '^{' $O/hires.log | cut -c1-300; grep '^{' $O/hires.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:v for k,v in d.items() if 'sampler' in k})"
run flower 400 python bench.py --model oxford_flower --steps 50 --warmup 10
grep '^{' $O/flower.log | cut -c1-300; grep '^{' $O/flower.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:v for k,v in d.items() if 'sampler' in k})"
