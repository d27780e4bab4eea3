"""Per-kernel durations + gaps of the graph-replayed DDIM sampler (one denoiser step =
the kernels between two head-GEMM launches), median over the replayed steps of a
rocprofv3 kernel trace of tools/sampler_graph_prof.py.
usage: python tools/sampler_graph_table.py <run_kernel_trace.csv>"""
import csv, re, statistics, sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
heads = [i for i, x in enumerate(k) if re.search(r"gemm_dma_kernel<[^>]*, 10, ", x[2])]
segs = [k[a + 1:b + 1] for a, b in zip(heads, heads[1:])]
n = statistics.mode(len(s) for s in segs)
segs = [s for s in segs if len(s) == n and (s[-1][1] - s[0][0]) < 2e6]
def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "").replace("dc::", "")[:70]
tot = gaps = 0.0
print(f"{len(segs)} denoiser steps, {n} kernels/step")
print("  #   dur_us  gap_us  kernel")
for i in range(n):
    d = statistics.median((s[i][1] - s[i][0]) / 1e3 for s in segs)
    gp = statistics.median(((s[i][0] - s[i - 1][1]) if i else 0) / 1e3 for s in segs)
    tot += d
    gaps += gp
    print(f"{i:3d} {d:8.2f} {gp:7.2f}  {short(segs[0][i][2])}")
wall = statistics.median((s[-1][1] - s[0][0]) / 1e3 for s in segs)
print(f"sum of kernel durations {tot:.1f} us, gaps {gaps:.1f} us, first-start to last-end {wall:.1f} us")
