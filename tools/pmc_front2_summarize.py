"""Per-kernel means of tools/pmc_front2.sh's counters."""
import collections
import csv
import glob
import sys

for d in sorted(glob.glob(f"gpurun_out/pmc_front2{sys.argv[1] if len(sys.argv) > 1 else ''}_p*")):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "k_front" not in r["Kernel_Name"]:
            continue
        acc[(r["Kernel_Name"][:20], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(d)
    for (k, c), v in sorted(acc.items()):
        print(f"  {k:20s} {c:24s} {sum(v) / len(v):16.0f}  (n={len(v)})")
