#!/bin/bash
# rocprof kernel stats of the training step and the sampler, A/B over an env switch: tools/gpu_prof_ab.sh VAR
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=${1:-DDIM_COLD_LN_FOLD}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
for v in 1 0; do
  export $VAR=$v
  rm -rf gpurun_out/prof_step_$v gpurun_out/prof_sampler_$v
  run prof_step_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step_$v -o run -- python3 bench.py --steps 50 --warmup 5 --no-sampler --no-graph
  run prof_sampler_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sampler_$v -o run -- python3 tools/sampler_prof.py
done
