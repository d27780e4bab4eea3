#!/bin/bash
# Profiles of the current tree: graph-replayed training step kernel trace (-> graph_step_table),
# sampler kernel stats, and two PMC sets over the training-shape hot kernels (tools/pmc_ops.py)
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof3
rm -rf $O; mkdir -p $O
run() { local name=$1 to=$2; shift 2
  echo "=== $name"; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -2 $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi; }
run graph 300 rocprofv3 --kernel-trace --output-format csv -d $O/graph -o run -- python3 bench.py --steps 30 --warmup 10 --no-sampler
python tools/graph_step_table.py $O/graph/run_kernel_trace.csv 20 > $O/graph_step_table.txt; tail -3 $O/graph_step_table.txt
run sampler 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sampler -o run -- python3 tools/sampler_prof.py
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  run pmc$i 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc$i -o run -- python3 tools/pmc_ops.py
done
