import csv, sys, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + '/set*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:90]
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
        dur[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, cs in agg.items():
    if 'copyBuffer' in k or 'Fill' in k: continue
    print(k, f" dur~{sorted(dur[k])[len(dur[k])//2]:.1f}us")
    print('   ' + '  '.join(f"{c}={sorted(v)[len(v)//2]:.3g}" for c, v in sorted(cs.items())))
