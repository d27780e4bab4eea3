#!/bin/bash
# rocprofv3 kernel stats for a target script: tools/prof.sh <name> <script> [args]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/prof_$name
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python3 "$@" > gpurun_out/prof_$name.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 gpurun_out/prof_$name.log
find gpurun_out/prof_$name -name "*kernel_stats.csv" | head -3
exit $rc
