"""Per-kernel sums of the SQ counters of tools/pmc_front.sh (per launch)."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    disp = collections.defaultdict(dict)
    for r in rows:
        d = disp[r["Dispatch_Id"]]
        d["name"] = r["Kernel_Name"][:40]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in disp.values():
        a = agg[d["name"]]
        a["n"] += 1
        for k, v in d.items():
            if k != "name":
                a[k] += v
    print(path)
    for name, a in agg.items():
        if "bwd" not in name and "fwd" not in name:
            continue
        n = a.pop("n")
        print(f"  {name}: " + ", ".join(f"{k} {v / n:.3g}" for k, v in sorted(a.items())))
