#!/bin/bash
# SQ counter passes (per-wave cycles / waits / instruction mix, LDS bank conflicts) and two
# L2-to-memory byte passes over the hot kernels of the targets tools/pmc_<target>.py:
# ops (ViT-tiny training shapes), sampler, hires (vit_small_200).  TARGETS="ops sampler hires"
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcw; rm -rf $O; mkdir -p $O
for tgt in ${TARGETS:-ops sampler}; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES" \
             "FETCH_SIZE SQ_WAVES" "WRITE_SIZE SQ_WAVES"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/$tgt/set$i -o run -- python3 tools/pmc_$tgt.py > $O/${tgt}_set$i.log 2>&1
    rc=$?; echo "$tgt set$i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/${tgt}_set$i.log; exit $rc; fi
  done
  python tools/pmc_waves.py $O/$tgt "$tgt" > $O/$tgt.md
done
