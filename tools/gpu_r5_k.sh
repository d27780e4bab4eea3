#!/bin/bash
# step table with the LayerNorm-prologue GEMMs on (program default in this tree)
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 bash tools/gpu_prof_step.sh r5k/prof_tiny --steps 30 --warmup 10
