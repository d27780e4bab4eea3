#!/bin/bash
# A/B of bench.py over an env switch (each value twice, interleaved): tools/gpu_ab_bench.sh VAR v1 v2 [pytest target]
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; T=$4
if [ -n "$T" ]; then
  timeout -k 10 300 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do for v in $A $B; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-eager-baseline > gpurun_out/ab_${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab_${v}_$rep.log; exit 1; }
  python - "$VAR=$v" gpurun_out/ab_${v}_$rep.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], "train ms/step", d["ms_per_step"], "img/s", d["value"], "| sampler ms", d.get("ddim_sampler_ms_per_batch"))
PY
done; done
