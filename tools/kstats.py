import csv, sys
f = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_step/run_kernel_stats.csv'
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e3/steps:8.1f} us/step  n={int(r['Calls'])/steps:5.1f} avg={float(r['AverageNs'])/1e3:6.2f}us  {r['Name'][:100]}")
print(f'total {tot/1e3/steps:.1f} us/step')
