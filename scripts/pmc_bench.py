"""Summarise rocprofv3 --pmc passes of bench.py into profiles/pmc_bench.json.

    python scripts/pmc_bench.py <dir with pmc_<workload>_<pass>/ outputs> <out.json>

Per workload and step-kernel family (gol_skew_kernel, gol_tb_pair_kernel, gol_persist_kernel, ...),
averaged over every dispatch of that family in the bench run:
  HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  On
  gfx950 FETCH_SIZE counts half the bytes of a coalesced streaming read
  (MI355X_MICROARCH.md, HBM section; the step kernels read 8 B (two words per
  lane) or 16 B (four) per lane, whole rows); WRITE_SIZE is exact.  Both count
  Infinity-Cache hits, so a board <= 256 MiB reads low.
  SQ_INSTS_VALU per launch, VALU-active fraction, clock from GRBM_GUI_ACTIVE.
turns_per_launch comes from the bench's own JSON line in the pass's log.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

src, dst = sys.argv[1], sys.argv[2]
out = json.load(open(dst)) if os.path.exists(dst) else {}
FAMILIES = ("gol_persist_kernel", "gol_tb_pair_kernel", "gol_split_pair_kernel", "gol_split_tri_kernel", "gol_skew_kernel",
            "gol_flip_turn_kernel")

for d in sorted(glob.glob(os.path.join(src, "pmc_*_*"))):
    if not os.path.isdir(d):
        continue
    m = re.match(r"pmc_(\d+)_", os.path.basename(d))
    if not m:
        continue
    wl = int(m.group(1))
    bench = None
    log = d + ".log"
    if os.path.exists(log):
        for line in open(log):
            if line.startswith('{"metric"'):
                bench = json.loads(line)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            fam = next((f for f in FAMILIES if f + "<" in row["Kernel_Name"] or f + "(" in row["Kernel_Name"]), None)
            if fam is None:
                continue
            rec = out.setdefault(f"{wl}:{fam}", {"_vals": {}, "_durs": []})
            rec.setdefault("_vals", {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
            rec.setdefault("_durs", []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
            if bench and fam in bench["roofline"]["kernel"]:
                rec["turns_per_launch"] = bench["roofline"].get("turns_per_launch", 1)
                rec["bench_kernel"] = bench["roofline"]["kernel"]

for key, rec in list(out.items()):
    vals = rec.pop("_vals", None)
    durs = rec.pop("_durs", None)
    if not vals:
        continue
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        f = statistics.mean(vals["FETCH_SIZE"]) * 1024
        w = statistics.mean(vals["WRITE_SIZE"]) * 1024
        rec.update({"fetch_size_bytes_raw": f, "fetch_bytes_corrected": 2 * f, "write_bytes": w,
                    "hbm_bytes_per_launch": 2 * f + w, "dispatches": len(vals["FETCH_SIZE"])})
    if "SQ_INSTS_VALU" in vals:
        dur = statistics.median(durs)
        rec.update({"sq_insts_valu": statistics.mean(vals["SQ_INSTS_VALU"]),
                    "sq_insts_salu": statistics.mean(vals.get("SQ_INSTS_SALU", [0.0])),
                    "sq_waves": statistics.mean(vals.get("SQ_WAVES", [0.0])),
                    "valu_active_frac": statistics.mean(vals["SQ_ACTIVE_INST_VALU"]) /
                    max(1.0, statistics.mean(vals["SQ_WAVE_CYCLES"])),
                    "pmc_median_dispatch_s": dur})
        if "GRBM_GUI_ACTIVE" in vals and dur > 0:
            rec["clock_ghz_est"] = statistics.mean(vals["GRBM_GUI_ACTIVE"]) / 8 / dur / 1e9
    rec["note"] = ("rocprofv3 --pmc passes of bench.py (scripts/pmc_bench.sh), one counter group per pass; "
                   "FETCH_SIZE x2 per the gfx950 correction; Infinity-Cache hits are counted")
# split tiling: one step launch is kernel A + kernel B (one dispatch of each)
for key in [k for k in out if k.endswith(":gol_split_pair_kernel")]:
    wl = key.split(":")[0]
    a, b = out[key], out.get(f"{wl}:gol_split_tri_kernel")
    if not b:
        continue
    rec = {"parts": ["gol_split_pair_kernel", "gol_split_tri_kernel"], "note": a.get("note"),
           "turns_per_launch": a.get("turns_per_launch"), "bench_kernel": a.get("bench_kernel")}
    for f in ("hbm_bytes_per_launch", "fetch_bytes_corrected", "write_bytes", "sq_insts_valu", "sq_insts_salu"):
        if f in a and f in b:
            rec[f] = a[f] + b[f]
    if "valu_active_frac" in a:
        rec["valu_active_frac"] = a["valu_active_frac"]
        rec["clock_ghz_est"] = a.get("clock_ghz_est")
    out[f"{wl}:gol_split"] = rec
json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1))
