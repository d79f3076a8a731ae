"""Summarise rocprofv3 --pmc passes of the step kernel into profiles/pmc_traffic.json.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a
coalesced streaming read (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact.
"""
import csv
import glob
import json
import os
import statistics
import sys

src = sys.argv[1]
dst = sys.argv[2]
out = json.load(open(dst)) if os.path.exists(dst) else {}
KERNELS = ("gol_persist_kernel", "gol_tb_kernel", "gol_tb_pair_kernel")
for size, kname in [(s, k) for s in (16384, 65536, 262144) for k in KERNELS]:
    vals = {}
    durs = []
    for path in glob.glob(os.path.join(src, f"pmc_{size}_*", "*counter_collection.csv")):
        for row in csv.DictReader(open(path)):
            if kname + "<" not in row["Kernel_Name"]:
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
            durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        continue
    tpl = 64 if kname == "gol_persist_kernel" else 16
    for log in glob.glob(os.path.join(src, f"pmc_{size}_*.log")):  # prof_step.py's own line
        for line in open(log):
            if line.startswith('{"turns_per_launch"'):
                tpl = json.loads(line)["turns_per_launch"]
    f = statistics.mean(vals["FETCH_SIZE"]) * 1024
    w = statistics.mean(vals["WRITE_SIZE"]) * 1024
    rec = {"fetch_size_bytes_raw": f, "fetch_bytes_corrected": 2 * f, "write_bytes": w,
           "hbm_bytes_per_launch": 2 * f + w, "board_bytes": size * size / 8, "launches": len(vals["FETCH_SIZE"]),
           "kernel": kname,
           # prof_step.py: a persistent launch runs 4 super-steps, a per-launch one the
           # board's launch depth (16, or 8 with four words per lane)
           "turns_per_launch": tpl,
           "note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes, scripts/prof_step.py; "
                   "Infinity-Cache hits are counted (a board <= 256 MiB is cache-resident)"}
    if "SQ_INSTS_VALU" in vals:
        dur = statistics.median(durs)
        g = statistics.mean(vals["GRBM_GUI_ACTIVE"])
        rec.update({
            "sq_insts_valu": statistics.mean(vals["SQ_INSTS_VALU"]),
            "sq_insts_salu": statistics.mean(vals["SQ_INSTS_SALU"]),
            "sq_waves": statistics.mean(vals["SQ_WAVES"]),
            "valu_active_frac": statistics.mean(vals["SQ_ACTIVE_INST_VALU"]) / max(1.0, statistics.mean(vals["SQ_WAVE_CYCLES"])),
            "clock_ghz_est": g / 8 / dur / 1e9 if dur > 0 else None,
        })
    out[f"{size}:{kname}"] = rec
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
