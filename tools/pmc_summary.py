"""rocprofv3 PMC sets (tools/gpu_pmc.sh) -> markdown table with derived ratios.

    python tools/pmc_summary.py gpurun_out/pmc > profiles/pmc.md
"""
import collections
import csv
import glob
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("dc::", "")
    return n.replace("_ZN2dc13ln_fwd_kernelILi3EEEvPKfS2_S2_PDF16bPfS4_if", "ln_fwd_kernel<3>")[:58]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(root + "/set*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("# Hardware counters of the hot kernels (rocprofv3 --pmc, ViT-tiny training shapes)\n")
    print("Target `tools/pmc_ops.py` (20 calls per kernel, eager), collected by `tools/gpu_pmc.sh` in 4 counter sets")
    print("(kernel trace only). Medians per dispatch. Derived: MFMA = bf16 MFMA instructions; VALU/MFMA = vector")
    print("instructions per MFMA; LDS conflict = `SQ_LDS_BANK_CONFLICT` cycles per LDS instruction; L2 hit =")
    print("`TCC_HIT/(TCC_HIT+TCC_MISS)`; HBM rd/wr = `TCC_EA0_RDREQ/WRREQ` (requests, not bytes).\n")
    print("| kernel | µs (profiled) | waves | MFMA | VALU/MFMA | LDS instr | LDS conflict | L2 hit | HBM rd req | HBM wr req |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    rows = []
    for k, cs in agg.items():
        if any(x in k for x in ("copyBuffer", "Fill", "elementwise", "at::")):
            continue
        m = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
        d = sorted(dur[k])[len(dur[k]) // 2]
        mf = m.get("SQ_INSTS_MFMA", 0)
        va = m.get("SQ_INSTS_VALU", 0)
        lds = m.get("SQ_INSTS_LDS", 0)
        cf = m.get("SQ_LDS_BANK_CONFLICT", 0)
        hit, miss = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
        rows.append((d, f"| `{k}` | {d:.1f} | {m.get('SQ_WAVES', 0):.0f} | {mf:.0f} | "
                        f"{(va / mf if mf else float('nan')):.1f} | {lds:.0f} | {(cf / lds if lds else 0):.2f} | "
                        f"{(hit / (hit + miss) if hit + miss else 0):.2f} | {m.get('TCC_EA0_RDREQ_sum', 0):.0f} | "
                        f"{m.get('TCC_EA0_WRREQ_sum', 0):.0f} |"))
    for _, r in sorted(rows, key=lambda x: -x[0]):
        print(r)
    print("\nReading: the GEMMs keep LDS bank conflicts at zero (XOR-swizzled LDS-DMA images) and hit L2 for")
    print("70-85 % of requests; their time is latency (a handful of dependent memory round trips per")
    print("workgroup), not MFMA throughput. The short attention kernels are conflict-free too (P/dS images")
    print("XOR-swizzled per 4-row group); the LayerNorm backward's dgamma/dbeta staging writes (2-float")
    print("stride) cost one conflict cycle per LDS instruction on a small part of its time. The deferred")
    print("weight-gradient launch runs ~1.7 M MFMAs (25.8 GFLOP) at 5 VALU per MFMA, fed from L2 (81 % hit).")
    print("sqnorm and AdamW stream the arenas from HBM by construction (L2 hit 2 % / 65 %).")


if __name__ == "__main__":
    main()
