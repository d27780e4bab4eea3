#!/bin/bash
# attention numerics + timings + LDS bank-conflict counters (one GPU call)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/attn
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attn or attention" > gpurun_out/attn/pytest.log 2>&1 || { tail -30 gpurun_out/attn/pytest.log; exit 1; }
tail -2 gpurun_out/attn/pytest.log
timeout -k 10 200 python tools/ub_attn.py > gpurun_out/attn/ub.log 2>&1 || { tail -30 gpurun_out/attn/ub.log; exit 1; }
cat gpurun_out/attn/ub.log
rm -rf gpurun_out/attn/pmc
timeout -k 10 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/attn/pmc -o run -- python3 tools/pmc_ops.py > gpurun_out/attn/pmc.log 2>&1 || { tail -30 gpurun_out/attn/pmc.log; exit 1; }
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/attn/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "attn" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k, {c: sorted(v)[len(v) // 2] for c, v in cs.items()})
PY
