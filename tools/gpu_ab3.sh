#!/bin/bash
# A/B of the in-tree build against other builds of this tree (DDIM_COLD_LIB):
# kernel tests first, forward-GEMM phases (tools/ub_gemm_phase.py), 2 interleaved
# rounds of 1000-step training benches, the sampler/img2img bench, then every GPU test.
# usage: tools/gpu_ab3.sh "<a.so> <b.so>[@VAR=value] ..." [pytest -k expr for the first test pass]
# (an @VAR=value suffix runs that build with one extra environment switch)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3
O=gpurun_out/ab3
LIBS="$1 ddim_cold_amd/_C.so"
K=${2:-gemm or attention or gelu or resid or qkv or embed}
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-2} $O/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
lab() { local b=${1%%@*}; local e=${1#*@}; [ "$e" = "$1" ] && e=""; echo "$(basename $b .so)${e:+_${e//=/}}"; }
lenv() { local b=${1%%@*}; local e=${1#*@}; [ "$e" = "$1" ] && e=""; echo "DDIM_COLD_LIB=$b $e"; }
run ktests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "$K" --timeout 120 --timeout-method thread
for L in $LIBS; do TAILN=1 run phase_$(lab $L) 120 env $(lenv $L) python tools/ub_gemm_phase.py; done
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
for rep in 1 2; do for L in $LIBS; do
  TAILN=0 run bench_$(lab $L)_$rep 200 env $(lenv $L) $B
  grep '^{' $O/bench_$(lab $L)_$rep.log | python -c "import json,sys; print('$(lab $L) ms/step', json.loads(sys.stdin.read())['ms_per_step'])"
done; done
for L in $LIBS; do
  TAILN=0 run sampler_$(lab $L) 300 env $(lenv $L) python bench.py --steps 10 --warmup 2 --no-eager-baseline
  grep '^{' $O/sampler_$(lab $L).log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(lab $L) sampler ms', d['ddim_sampler_ms_per_batch'], 'img2img ms', d['draft2drawing_ms'])"
done
run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
