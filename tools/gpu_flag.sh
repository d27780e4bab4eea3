#!/bin/bash
# flag hand-off (kernel-node counter + comm-stream wait-value) vs event-record nodes for the
# event-split data-parallel step: parity first, then a graph trace and ms/step (1 GPU)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PARITY:-1}" = "1" ]; then
  timeout -k 10 240 python -u tools/dist_parity.py > gpurun_out/dist_parity.log 2>&1 || { tail -20 gpurun_out/dist_parity.log; exit 1; }
  tail -1 gpurun_out/dist_parity.log
  timeout -k 10 240 python -u tools/dist2_gpu.py > gpurun_out/dist2.log 2>&1 || { tail -20 gpurun_out/dist2.log; exit 1; }
  tail -2 gpurun_out/dist2.log
fi
rm -rf gpurun_out/prof_flag
DDIM_COLD_COMM_PRIO=${PRIO:-0} DDIM_COLD_FAKE_COMM=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_flag -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler --force-dist --comm-layout overlap-2 > gpurun_out/prof_flag.log 2>&1 || { tail -5 gpurun_out/prof_flag.log; exit 1; }
run() {
  timeout -k 10 120 env "$@" > gpurun_out/flag_b.log 2>&1 || { tail -5 gpurun_out/flag_b.log; exit 1; }
  echo "$* $(grep '^{' gpurun_out/flag_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['ms_per_step'], c['comm'], c['comm_layout'], c['comm_layout_ms'])")" | sed 's/python bench.py --steps 1000 --warmup 50 --no-sampler//'
}
B="python bench.py --steps 1000 --warmup 50 --no-sampler --force-dist"
for rep in 1 2; do
run X=fake_flag_overlap2 DDIM_COLD_FAKE_COMM=1 $B --comm-layout overlap-2
run X=fake_flag_overlap2_nopre DDIM_COLD_PREISSUE=0 DDIM_COLD_FAKE_COMM=1 $B --comm-layout overlap-2
run X=fake_flag_overlap4 DDIM_COLD_FAKE_COMM=1 $B --comm-layout overlap-4
run X=fake_flag_inline DDIM_COLD_FAKE_COMM=1 $B --comm-layout inline-1
run X=rccl_auto $B
done
