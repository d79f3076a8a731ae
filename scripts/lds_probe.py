"""K1r (resident LDS bands) probe: GCUPS and, from the kernel's own
s_memrealtime stamps (option "trace"), the average time a workgroup spends
per super-step in compute, publish (edge stores + flag), neighbour wait and
halo load.

    python scripts/lds_probe.py --cases 8192x8192,5120x5120 --sets "lds_depth=8;lds_depth=12,lds_waves=16" [--turns 2000]
"""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cases", default="8192x8192,5120x5120")
ap.add_argument("--sets", default="lds_depth=8")
ap.add_argument("--turns", type=int, default=2000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--traces", default="0,1", help="trace settings to run (0: untraced only, e.g. under rocprofv3 --pmc)")
a = ap.parse_args()
sets = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv) for s in a.sets.split(";")]
for rep in range(a.reps):
    for case in a.cases.split(","):
        W, H = (int(x) for x in case.split("x"))
        for opts in sets:
            for trace in (int(t) for t in a.traces.split(",")):
                with golhip.Board(W, H) as b:
                    b.set_option("persistent", 1)
                    b.set_option("lds_band", 1)
                    if trace:
                        b.set_option("trace", 1)
                    for k, v in opts.items():
                        b.set_option(k, v)
                    b.fill_random(0x5EED0002)
                    b.step(200)
                    b.sync()
                    if trace:
                        b.persist_trace()
                    b.perf_reset()
                    t0 = time.perf_counter()
                    b.step(a.turns)
                    b.sync()
                    dt = time.perf_counter() - t0
                    p = b.perf()
                    rec = {"case": case, "opts": opts, "trace": trace, "rep": rep, "gcups": round(W * H * a.turns / dt / 1e9, 1),
                           "lds_launches": p["lds_launches"]}
                    if trace:
                        t = b.persist_trace()
                        wgs = max(1, t["workgroups"])
                        D = opts.get("lds_depth", 12)
                        ss = (a.turns + D - 1) // D
                        # ticks are 10 ns: per workgroup, per super-step, in us
                        names = ["compute", "publish", "wait", "halo"]
                        vals = [t["band_ticks"], t["max_band_ticks"], t["wait_ticks"], t["kernel_ticks"]]
                        rec["us_per_superstep"] = {n: round(v / wgs / ss / 100, 3) for n, v in zip(names, vals)}
                        # per wave: ticks in the turn barriers (slots 8.. of the trace)
                        tw = b.persist_trace_waves(min(wgs, 1024)).astype(np.int64)
                        bt, bn = tw[:, :, 0], tw[:, :, 1]
                        live = bn > 0
                        if live.any():
                            rec["barrier"] = {
                                "us_per_turn_per_wave": round(float((bt[live] / bn[live]).mean()) / 100, 3),
                                "share_of_compute": round(float(bt[live].mean()) / max(1.0, vals[0] / wgs), 3)}
                    print(json.dumps(rec), flush=True)
