"""Per-kernel MFMA utilisation from one rocprofv3 --pmc pass.

util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128): GRBM_GUI_ACTIVE is
summed over the 8 XCDs, so GRBM / 8 x 256 CUs x 4 SIMDs = GRBM x 128 SIMD-cycles
of capacity; SQ_VALU_MFMA_BUSY_CYCLES is summed over all SIMDs
(MI355X_MICROARCH.md, cycle constants / DVFS sections).  clock_ghz =
GRBM / 8 / kernel duration.
"""
import collections
import csv
import json
import sys

src, out = sys.argv[1:3]
rows = list(csv.DictReader(open(src)))
disp = collections.defaultdict(dict)
for r in rows:
    d = disp[r["Dispatch_Id"]]
    d["name"] = r["Kernel_Name"]
    d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in disp.values():
    if d.get("SQ_INSTS_MFMA", 0) <= 0:
        continue
    a = agg[d["name"][:120]]
    a["launches"] += 1
    for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "GRBM_GUI_ACTIVE", "ns"):
        a[k] += d.get(k, 0.0)
res = {}
for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
    res[name] = {"launches": int(a["launches"]), "avg_us": a["ns"] / a["launches"] / 1e3,
                 "mfma_util": a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] * 128),
                 "clock_ghz": a["GRBM_GUI_ACTIVE"] / 8 / a["ns"]}
json.dump(res, open(out, "w"), indent=1)
for k, v in list(res.items())[:12]:
    print(f"{v['mfma_util']:.3f} util {v['clock_ghz']:.2f} GHz {v['avg_us']:8.1f} us x{v['launches']}  {k[:90]}")
