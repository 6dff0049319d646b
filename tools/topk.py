import csv, sys
f = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof/bench_kernel_stats.csv'
k = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:k]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}% calls {r['Calls']:>6} avg {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
print('total ms', tot/1e6)
