#!/bin/bash
# data-parallel default (event-split step graphs, host-issued collectives, autotuned
# layout) on one GPU: parity vs the single process, then ms/step with each bucket's
# collective replaced by one elementwise pass over its range (DDIM_COLD_FAKE_COMM=1:
# real work on the comm queue, as at N > 1) and with the 1-rank RCCL collectives
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dist_parity.py > gpurun_out/dist_parity.log 2>&1 || { tail -20 gpurun_out/dist_parity.log; exit 1; }
tail -2 gpurun_out/dist_parity.log
run() {
  timeout -k 10 150 env "$@" > gpurun_out/ev_b.log 2>&1 || { tail -5 gpurun_out/ev_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/ev_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['ms_per_step'], c['allreduce'], c['comm_layout'], c['comm_layout_ms'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler"
for rep in 1 2; do
run X=single $B
run X=fake_auto DDIM_COLD_FAKE_COMM=1 $B --force-dist
run X=fake_overlap2 DDIM_COLD_FAKE_COMM=1 $B --force-dist --comm-layout overlap-2
run X=fake_inline1 DDIM_COLD_FAKE_COMM=1 $B --force-dist --comm-layout inline-1
run X=fake_captured_overlap2 DDIM_COLD_FAKE_COMM=1 $B --force-dist --captured-comm --comm-layout overlap-2
run X=rccl_auto $B --force-dist
run X=rccl_auto_native $B --force-dist --comm native
done
