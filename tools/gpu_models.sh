#!/bin/bash
# training (+ sampler) throughput of the other model configs on the current tree
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; grep -h '^{' gpurun_out/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k in ('value','ms_per_step') or 'sampler_img' in k or 'vs_eager' in k or 'gaussian_ddim_train_img' in k})"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run small200 400 python bench.py --model vit_small_200 --steps 30 --warmup 10 --no-gaussian
run flower 300 python bench.py --model oxford_flower --steps 100 --warmup 20 --no-gaussian
