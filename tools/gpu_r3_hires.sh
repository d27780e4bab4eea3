#!/bin/bash
# high-resolution path (vit_small_200, 626 tokens): bench (train + sampler + eager comparator),
# eager-step and sampler kernel stats, long-sequence attention timings + PMC sets
cd "$(dirname "$0")/.." 2>/dev/null || cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hires
export TMPDIR=/tmp
O=gpurun_out/hires
rm -rf $O/*
run() { local name=$1; local lim=$2; shift; shift
  echo "=== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; echo "STOP after $name"; exit $rc; fi; }
run bench 400 python bench.py --model vit_small_200 --steps 30 --warmup 10
grep '^{' $O/bench.log | cut -c1-600
run attn_time 200 python tools/pmc_attn_long.py time
cat $O/attn_time.log
run prof_step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- python3 bench.py --model vit_small_200 --steps 10 --warmup 3 --no-sampler --no-graph
run prof_sampler 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sampler -o run -- python3 tools/sampler_prof_model.py vit_small_200
i=0
for set in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VALU SQ_INSTS_MFMA" ; do
  i=$((i+1))
  run pmc$i 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/pmc$i -o run -- python3 tools/pmc_attn_long.py
done
echo done
