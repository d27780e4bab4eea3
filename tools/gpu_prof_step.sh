#!/bin/bash
# Kernel trace of the graph-replayed training step -> per-kernel table in step order.
#   bash tools/gpu_prof_step.sh OUTNAME [bench.py args...]
cd "$(dirname "$0")/.." 2>/dev/null || cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
name=$1; shift
O=gpurun_out/$name
rm -rf "$O"; mkdir -p "$O"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O" -o run -- python3 bench.py --no-sampler --no-gaussian --no-vendor "$@" > "$O/bench.log" 2>&1
rc=$?
tail -2 "$O/bench.log" | cut -c1-300
[ $rc -ne 0 ] && exit $rc
python tools/graph_step_table.py "$O/run_kernel_trace.csv" 10 > "$O/step_table.txt"
rm -f "$O/run_kernel_trace.csv"
tail -3 "$O/step_table.txt"
