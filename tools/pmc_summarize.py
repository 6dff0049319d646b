"""Per-launch HBM bytes of k_step from two rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half of the
bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is taken as is.  Writes {"hbm_bytes_per_launch": ...}.
"""
import csv
import json
import statistics
import sys

fetch_csv, write_csv, out = sys.argv[1:4]


def per_launch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if "k_step" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return vals


f = per_launch(fetch_csv, "FETCH_SIZE")
w = per_launch(write_csv, "WRITE_SIZE")
fetch_b = statistics.median(f) * 1024 * 2
write_b = statistics.median(w) * 1024
res = {"kernel": "k_step", "launches": [len(f), len(w)], "fetch_bytes_per_launch": fetch_b,
       "write_bytes_per_launch": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
       "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of wide reads); WRITE_SIZE KiB x 1024",
       "command": "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
