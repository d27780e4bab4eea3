"""Idle gaps between kernels of the graph-replayed training step (rocprofv3 kernel
trace of `bench.py` in graph mode): per-step kernel busy time vs wall time.
usage: python tools/graph_gaps.py gpurun_out/prof_graph/run_kernel_trace.csv [steps]"""
import csv, sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
k.sort()
# take the last `steps` steps: split at adamw_kernel
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ends = [i for i, x in enumerate(k) if "adamw_kernel" in x[2]]
sel = ends[-steps - 1:]
tot_wall = tot_busy = 0
gaps = defaultdict(float)
n = 0
for a, b in zip(sel, sel[1:]):
    seg = k[a + 1:b + 1]
    wall = seg[-1][1] - k[a][1]
    busy = 0
    last_end = k[a][1]
    for s, e, name in seg:
        busy += e - max(s, last_end) if e > last_end else 0
        g = s - last_end
        if g > 0:
            gaps[name.split("(")[0][:60]] += g
        last_end = max(last_end, e)
    tot_wall += wall
    tot_busy += busy
    n += 1
print(f"steps {n}: wall {tot_wall / n / 1e3:.1f} us/step, kernels busy {tot_busy / n / 1e3:.1f} us/step, "
      f"idle {(tot_wall - tot_busy) / n / 1e3:.1f} us/step, kernels/step {len(k[sel[-2] + 1:sel[-1] + 1])}")
for name, g in sorted(gaps.items(), key=lambda x: -x[1])[:12]:
    print(f"  gap before {name}: {g / n / 1e3:.2f} us/step")
