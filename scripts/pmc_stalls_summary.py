"""Summary of scripts/pmc_stalls.sh passes: per-dispatch averages of every
counter for the kernels matching a name, and the wave-cycle breakdown.

    python scripts/pmc_stalls_summary.py <dir> [kernel-substring] > <dir>/stalls_summary.json

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave
(MI355X_MICROARCH.md, constants table); WAIT_ANY (parked at s_waitcnt /
barrier / sleep) + WAIT_INST_ANY (ready but not issued: dependency, pipe or
instruction-fetch stall) + ACTIVE_INST_ANY (issuing) ~= WAVE_CYCLES.
GRBM_GUI_ACTIVE (summed over 8 XCDs) / 8 / dispatch time = effective clock.

Only the timed dispatches count: a pass keeps the dispatches at least half
as long as its longest one (probes run a short warmup launch before the
timed one, e.g. 200 then 1000 turns; round 5), and the
summary records how many it kept and dropped.
"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

src = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "gol_skew_kernel"
res = {}
for path in sorted(glob.glob(os.path.join(src, "stall_*", "**", "*counter_collection.csv"), recursive=True)):
    tag = re.sub(r"_\d+$", "", os.path.basename(os.path.dirname(path)) if "stall_" in os.path.dirname(path)
                 else path.split(os.sep)[-3])
    rows = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        if want not in r["Kernel_Name"]:
            continue
        d = rows[r["Dispatch_Id"]]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    if not rows:
        continue
    longest = max(d["_dur"] for d in rows.values())
    dropped = [k for k, d in rows.items() if d["_dur"] < 0.5 * longest]
    for k in dropped:
        del rows[k]
    rec = res.setdefault(tag, {"kernel": sorted(set(names.values())), "counters": {}, "dispatches": 0,
                               "dropped_short_dispatches": 0})
    rec["dropped_short_dispatches"] = max(rec["dropped_short_dispatches"], len(dropped))
    keys = set().union(*[set(d) for d in rows.values()])
    for k in sorted(keys):
        vals = [d[k] for d in rows.values() if k in d]
        if k == "_dur":
            rec.setdefault("dur_us_median", []).append(statistics.median(vals) * 1e6)
        else:
            rec["counters"][k] = statistics.mean(vals)
    rec["dispatches"] = max(rec["dispatches"], len(rows))
for tag, rec in res.items():
    c = rec["counters"]
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        rec["wave_cycle_split"] = {k: round(c[k] / wc, 4) for k in
                                   ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                    "SQ_ACTIVE_INST_SCA", "SQ_BUSY_CYCLES") if k in c}
    if "SQ_INSTS_VALU" in c:
        tot = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                          "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"))
        rec["instruction_mix"] = {k: round(c[k] / tot, 4) for k in c if k.startswith("SQ_INSTS_")}
    if "GRBM_GUI_ACTIVE" in c and rec.get("dur_us_median"):
        rec["clock_ghz_est"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (statistics.median(rec["dur_us_median"]) * 1e-6) / 1e9, 3)
print(json.dumps(res, indent=1))
