"""Per-wave timing of one K1w launch (option "trace"): where the launch time goes.

    python scripts/trace_skew.py [--case 65536x65536] [--opt k=v ...]

Prints, per stack position (wave w = position for stacks of 8 bands), the
mean band time and mean end time relative to the launch's first wave start,
and the spread of the workgroups' last-wave end (the launch tail).
Times in us (s_memrealtime, 100 MHz).
"""
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "game-of-life-distributed_amd")]
import golhip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--case", default="65536x65536")
ap.add_argument("--opt", action="append", default=[])
ap.add_argument("--depth", type=int, default=20)
a = ap.parse_args()
ring = a.case.endswith("r")
W, R = (int(x) for x in a.case.rstrip("r").split("x"))
with golhip.Board(W, R, timing=True) as b:
    if ring:
        b.comm_init(golhip.unique_id(), 1, 0)
        b.set_option("force_halo", 1)
    b.set_tb_depth(a.depth)
    for kv in a.opt:
        k, v = kv.split("=")
        b.set_option(k, int(v))
    b.set_option("trace", 1)
    b.fill_random(0x5EED0002)
    b.step(200)
    b.sync()
    b.perf_reset()
    b.step(a.depth)  # one launch (torus only: a ring step would run its exchange group)
    b.sync()
    p = b.perf()
    t = b.persist_trace_waves(256).astype(np.int64)  # (blocks, 64, 2)
st, en = t[:, :16, 0], t[:, :16, 1]
live = (st > 0) & (en > 0)
blocks = np.nonzero(live.any(axis=1))[0]
st, en, live = st[blocks], en[blocks], live[blocks]
t0 = st[live].min()
dur = (en - st) / 100.0
endr = (en - t0) / 100.0
res = {"case": a.case, "opts": a.opt, "launch_ms_event": p["step_kernel_ms"] / max(1, p["step_launches"]),
       "blocks": int(len(blocks)), "span_us": float(endr[live].max()),
       "start_spread_us": float((st[live].max() - t0) / 100.0)}
pos = []
for w in range(16):
    m = live[:, w]
    if m.any():
        pos.append({"w": w, "dur_mean": round(float(dur[m, w].mean()), 2), "dur_min": round(float(dur[m, w].min()), 2),
                    "dur_max": round(float(dur[m, w].max()), 2), "end_mean": round(float(endr[m, w].mean()), 2)})
# phase stamps (fill done, main loop done) of the same waves: slots 16..31
fe, me = t[blocks, 16:32, 0], t[blocks, 16:32, 1]
ok = live & (fe > 0) & (me > 0)
if ok.any():
    for q in pos:
        m = ok[:, q["w"]]
        if m.any():
            w = q["w"]
            q["fill_us"] = round(float(((fe[m, w] - st[m, w]) / 100.0).mean()), 2)
            q["main_us"] = round(float(((me[m, w] - fe[m, w]) / 100.0).mean()), 2)
            q["drain_us"] = round(float(((en[m, w] - me[m, w]) / 100.0).mean()), 2)
# diagnostic builds (GOL_SKEW_WAIT_TRACE): load-wait ticks and groups, main loop (slots 32..47) and fill (48..63)
wm, nm, wf, nf = t[blocks, 32:48, 0], t[blocks, 32:48, 1], t[blocks, 48:64, 0], t[blocks, 48:64, 1]
if (nm > 0).any():
    for q in pos:
        w = q["w"]
        m = live[:, w] & (nm[:, w] > 0)
        if m.any():
            q["main_wait_us"] = round(float((wm[m, w] / 100.0).mean()), 2)
            q["main_groups"] = round(float(nm[m, w].mean()), 1)
        m = live[:, w] & (nf[:, w] > 0)
        if m.any():
            q["fill_wait_us"] = round(float((wf[m, w] / 100.0).mean()), 2)
            q["fill_groups"] = round(float(nf[m, w].mean()), 1)
res["positions"] = pos
wg_end = np.where(live, endr, 0).max(axis=1)
wg_mean = np.where(live, endr, 0).sum(axis=1) / np.maximum(1, live.sum(axis=1))
res["wg_end_us"] = {"min": float(wg_end.min()), "mean": float(wg_end.mean()), "max": float(wg_end.max())}
res["wg_idle_frac"] = float(((wg_end[:, None] - np.where(live, endr, wg_end[:, None])).sum()) / (wg_end.sum() * np.maximum(1, live.sum(axis=1)).mean()))
print(json.dumps(res))
