"""Per-kernel durations of the graph-replayed training step, in step order (median
over the last `steps` steps of a rocprofv3 kernel trace of `bench.py`).
usage: python tools/graph_step_table.py gpurun_out/prof_graph/run_kernel_trace.csv [steps]"""
import csv, sys, statistics, re

rows = list(csv.DictReader(open(sys.argv[1])))
k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ends = [i for i, x in enumerate(k) if "adamw_kernel" in x[2]]  # a step ends with its optimizer
sel = ends[-steps - 1:]
segs = [k[a + 1:b + 1] for a, b in zip(sel, sel[1:])]
n = min(len(s) for s in segs)
segs = [s for s in segs if len(s) == n]
def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("dc::", "")
    return name[:70]
tot = 0.0
print(f"{len(segs)} steps, {n} kernels/step")
print("  #   dur_us  gap_us  kernel")
for i in range(n):
    d = statistics.median((s[i][1] - s[i][0]) / 1e3 for s in segs)
    gp = statistics.median(((s[i][0] - s[i - 1][1]) if i else 0) / 1e3 for s in segs)
    tot += d
    print(f"{i:3d} {d:8.2f} {gp:7.2f}  {short(segs[0][i][2])}")
wall = statistics.median((s[-1][1] - s[0][0]) / 1e3 for s in segs)
print(f"sum of kernel durations {tot:.1f} us, first-start to last-end {wall:.1f} us")
