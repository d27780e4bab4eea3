#!/bin/bash
# Attention VALU diet A/B: smoke + attention GPU tests on this tree, then the
# attention shapes (tools/ub_attn.py) and the 1000-step training bench for three
# builds, interleaved: ab/C_base.so (HEAD), in-tree _C.so, ab/C_all.so (VGPR-form
# MFMA in every unit)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/attn
O=gpurun_out/attn
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -${TAILN:-3} $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run attn_tests 300 python -u -m pytest tests -m gpu -x -q -k "attn or attention or flash or short" --timeout 120 --timeout-method thread
for lib in base tree all; do
  case $lib in base) L=ab/C_base.so;; all) L=ab/C_all.so;; tree) L=ddim_cold_amd/_C.so;; esac
  TAILN=14 run ub_attn_$lib 200 env DDIM_COLD_LIB=$L python tools/ub_attn.py
done
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
for rep in 1 2; do for lib in base tree all; do
  case $lib in base) L=ab/C_base.so;; all) L=ab/C_all.so;; tree) L=ddim_cold_amd/_C.so;; esac
  TAILN=1 run bench_${lib}_$rep 200 env DDIM_COLD_LIB=$L $B
done; done
for lib in base tree all; do
  case $lib in base) L=ab/C_base.so;; all) L=ab/C_all.so;; tree) L=ddim_cold_amd/_C.so;; esac
  TAILN=1 run sampler_$lib 200 env DDIM_COLD_LIB=$L python bench.py --steps 10 --warmup 2
done
run gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
