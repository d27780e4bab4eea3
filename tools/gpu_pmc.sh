#!/bin/bash
# rocprofv3 PMC counter sets over tools/pmc_ops.py (kernel-trace only, no sys/runtime trace)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rm -rf gpurun_out/pmc/set*
i=0
for set in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VALU_MFMA_MOPS_BF16" ; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/set$i -o run -- python3 tools/pmc_ops.py > gpurun_out/pmc/set$i.log 2>&1
  rc=$?
  echo "set$i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
