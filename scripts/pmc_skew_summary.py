"""Per-launch averages of the K1w PMC passes (scripts/pmc_skew.sh) -> <dir>/pmc_skew.json.

Per case W x R (a board, or a one-rank-ring strip with suffix r): every
counter averaged over the gol_skew_kernel dispatches, the kernel duration,
SQ_INSTS_VALU against the minimum (11 instructions per word-turn with two
words per lane: 9 LUTs + 1 DPP + 1 alignbit; 10 with four), the VALU-busy
fraction SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES... and HBM bytes (2 x FETCH_SIZE
+ WRITE_SIZE, gfx950 correction, MI355X_MICROARCH.md).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

src = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(src, "pmc_*_1"))):
    case = re.match(r"pmc_(.+)_1$", os.path.basename(d)).group(1)
    vals, durs, depth, wpl = {}, [], None, None
    for path in glob.glob(os.path.join(src, f"pmc_{case}_*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if "gol_skew_kernel" not in row["Kernel_Name"]:
                continue
            m = re.search(r"gol_skew_kernel<(\d+), (\d+)>", row["Kernel_Name"])
            if m:
                depth, wpl = int(m.group(1)), int(m.group(2))
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
            durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    if not vals:
        continue
    avg = {k: statistics.mean(v) for k, v in vals.items()}
    W, R = (int(x) for x in case.rstrip("r").split("x"))
    rec = {"case": case, "kernel": f"gol_skew_kernel<{depth}, {wpl}>", "dispatch_records": len(durs),
           "duration_us_median": statistics.median(durs) * 1e6, "counters": avg}
    if "SQ_INSTS_VALU" in avg and depth:
        words = R * ((W + 31) // 32)
        minimum = words * depth / 64 * (9 + (2 if wpl <= 2 else 1) * (1 if wpl >= 2 else 2))
        rec["insts_valu_vs_min"] = avg["SQ_INSTS_VALU"] / minimum
        rec["valu_active_frac"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"] if avg.get("SQ_WAVE_CYCLES") else None
    if "SQ_WAIT_INST_ANY" in avg:
        rec["wait_inst_frac"] = avg["SQ_WAIT_INST_ANY"] / max(1.0, avg.get("SQ_WAIT_INST_ANY", 0) + avg.get("SQ_WAIT_ANY", 0) + avg.get("SQ_ACTIVE_INST_ANY", 0))
        rec["wait_any_frac"] = avg["SQ_WAIT_ANY"] / max(1.0, avg["SQ_WAIT_INST_ANY"] + avg["SQ_WAIT_ANY"] + avg["SQ_ACTIVE_INST_ANY"])
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rec["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        rec["board_bytes"] = W * R / 8
    res[case] = rec
json.dump(res, open(os.path.join(src, "pmc_skew.json"), "w"), indent=1)
for k, r in res.items():
    print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in r.items() if x != "counters"})
