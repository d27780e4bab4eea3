#!/bin/bash
# Round-end style GPU pass: smoke, all GPU tests, trainer on synthetic data (+resume), full bench.
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
if [ "${TRAIN:-1}" = "1" ]; then
  rm -rf /tmp/ddc_train && mkdir -p /tmp/ddc_train
  sed -e 's/epoch : \[0,2\]/epoch : [0,1]/' configs/synthetic_tiny.yaml > /tmp/ddc_train/synth.yaml
  run train 300 python multi_gpu_trainer.py /tmp/ddc_train/synth.yaml --root /tmp/ddc_train
  cp /tmp/ddc_train/Saved_Models/synthvit_tiny_synthetic/train.log gpurun_out/train_synth.log
fi
run bench 300 python bench.py
run bench_dp1 300 python bench.py --force-dist --no-sampler --steps 1000 --warmup 50
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/prof_step gpurun_out/prof_sampler
  run prof_step 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph --no-gaussian
  run prof_sampler 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sampler -o run -- python3 tools/sampler_prof.py
fi
