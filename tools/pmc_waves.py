"""rocprofv3 PMC sets -> per-wave table: cycles per wave, % parked on s_waitcnt /
barriers (SQ_WAIT_ANY), % issue-stalled (SQ_WAIT_INST_ANY), and instructions per
wave by kind.  SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md).

    python tools/pmc_waves.py <dir with set*/run_counter_collection.csv> [title]
"""
import collections
import csv
import glob
import re
import statistics
import sys


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("dc::", "")[:52]


def main():
    root = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else root
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(root + "/*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"# Per-wave hardware counters: {title}\n")
    print("Medians per dispatch; cycles = 4 x SQ_WAVE_CYCLES / SQ_WAVES; wait = SQ_WAIT_ANY (parked on "
          "s_waitcnt / barrier), stall = SQ_WAIT_INST_ANY (issue-stalled), both as % of wave cycles.\n")
    print("| kernel | waves | cycles/wave | wait % | stall % | VALU/wave | MFMA/wave | VALU/MFMA | SALU/wave | "
          "LDS/wave | LDS bank conflict cycles/wave | VMEM rd/wave | VMEM wr/wave | L2->HBM fetch MB | write MB |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, cs in sorted(agg.items()):
        if any(x in k for x in ("elementwise", "Fill", "copy", "at::")):
            continue
        m = {c: statistics.median(v) for c, v in cs.items()}
        w = max(m.get("SQ_WAVES", 1), 1)
        wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
        print(f"| `{k}` | {w:.0f} | {4 * wc / w:.0f} | {100 * m.get('SQ_WAIT_ANY', 0) / wc:.0f} | "
              f"{100 * m.get('SQ_WAIT_INST_ANY', 0) / wc:.0f} | {m.get('SQ_INSTS_VALU', 0) / w:.0f} | "
              f"{m.get('SQ_INSTS_MFMA', 0) / w:.0f} | "
              f"{(m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']) if m.get('SQ_INSTS_MFMA') else float('nan'):.1f} | "
              f"{m.get('SQ_INSTS_SALU', 0) / w:.0f} | "
              f"{m.get('SQ_INSTS_LDS', 0) / w:.0f} | {m.get('SQ_LDS_BANK_CONFLICT', 0) / w:.1f} | "
              f"{m.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | "
              f"{m.get('SQ_INSTS_VMEM_WR', 0) / w:.0f} | {m.get('FETCH_SIZE', 0) / 1024:.1f} | "
              f"{m.get('WRITE_SIZE', 0) / 1024:.1f} |")


if __name__ == "__main__":
    main()
