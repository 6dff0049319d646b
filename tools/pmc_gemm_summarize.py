"""Per-kernel means of the counters of tools/pmc_gemm.sh (one line per counter)."""
import collections
import csv
import glob
import sys

for d in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_gemm_b*_p*")):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"]
        if "k_bres" not in name and "k_x3nt" not in name:
            continue
        acc[(name[:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(d)
    for (k, c), v in sorted(acc.items()):
        print(f"  {k:40s} {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
