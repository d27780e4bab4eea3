#!/bin/bash
# all GPU tests, then bench twice (+ dropout cost diagnostic)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tb_tests.log 2>&1
rc=$?; tail -15 gpurun_out/tb_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-eager-baseline > gpurun_out/tb_bench_$i.log 2>&1 || { tail -5 gpurun_out/tb_bench_$i.log; exit 1; }
  grep "^{" gpurun_out/tb_bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train ms/step', d['ms_per_step'], 'img/s', d['value'], '| sampler ms', d.get('ddim_sampler_ms_per_batch'))"
done
if [ "${DROPCOST:-0}" = "1" ]; then timeout -k 10 300 python tools/drop_cost.py; fi
