"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

python tools/pmc_traffic_summarize.py KERNEL_SUBSTR fetch.csv write.csv out.json [ALG_BYTES] [NOTE]

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half of the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is taken as is.  Medians over the launches.
"""
import csv
import json
import statistics
import sys

kern, fetch_csv, write_csv, out = sys.argv[1:5]
alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
note = sys.argv[6] if len(sys.argv) > 6 else ""


def per_launch(path, counter):
    vals, name = [], None
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
    return vals, name


f, name = per_launch(fetch_csv, "FETCH_SIZE")
w, _ = per_launch(write_csv, "WRITE_SIZE")
fetch_b = statistics.median(f) * 1024 * 2
write_b = statistics.median(w) * 1024
res = {"kernel": name, "launches": [len(f), len(w)], "fetch_bytes_per_launch": fetch_b,
       "write_bytes_per_launch": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
       "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of wide reads); WRITE_SIZE KiB x 1024",
       "note": note}
if alg:
    res["algorithmic_bytes_per_launch"] = alg
    res["ratio_to_algorithmic"] = (fetch_b + write_b) / alg
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
