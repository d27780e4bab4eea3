"""rocprofv3 --stats kernel table -> markdown (per-step microseconds).

    python tools/prof_summary.py <run_kernel_stats.csv> <steps> <title> > profiles/<name>.md
"""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("dc::", "")
    return name[:90]


def main():
    path, steps, title = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Source: `rocprofv3 --kernel-trace --stats` ({path.split('/')[-1]}), {steps:g} steps; "
          f"kernel time summed per step = **{tot / 1e3 / steps:.1f} us**.\n")
    print("| us/step | calls/step | avg us | share | kernel |")
    print("|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        if t / tot < 0.002:
            continue
        print(f"| {t / 1e3 / steps:.1f} | {int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.2f} | "
              f"{100 * t / tot:.1f}% | `{short(r['Name'])}` |")


if __name__ == "__main__":
    main()
