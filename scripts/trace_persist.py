"""Persistent-kernel time split (band compute vs neighbour wait) per variant.
usage: python scripts/trace_persist.py --size 16384 --variants "persist_waves=8;persist_waves=16" """
import argparse
import json
import os

os.environ.setdefault("GOLHIP_TUNING", "1")  # A/B knobs of the kernel plans (golhip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "game-of-life-distributed_amd"))
import golhip  # noqa: E402
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=16384)
ap.add_argument("--depths", default="16")
ap.add_argument("--turns", type=int, default=1024)
ap.add_argument("--variants", default="")
a = ap.parse_args()
with golhip.Board(a.size, a.size, timing=True) as b:
    b.set_option("trace", 1)
    b.fill_random(0x5EED0001)
    for d in map(int, a.depths.split(",")):
        for v in [x for x in a.variants.split(";") if x] or [""]:
            opts = {"wpl": 0, "persistent": 1, "persist_waves": 0}
            opts.update({k: int(x) for k, x in (kv.split("=") for kv in v.split(",") if kv)})
            for k, x in opts.items():
                b.set_option(k, x)
            b.set_tb_depth(d)
            b.step(2 * d)
            b.sync()
            b.persist_trace()
            b.perf_reset()
            b.step(a.turns)
            b.sync()
            p = b.perf()
            t = b.persist_trace()
            n_sup = a.turns // d
            wgs = max(1, t["workgroups"])
            rec = dict(N=a.size, depth=d, variant=v, gcups=a.size * a.size * p["persist_turns"] / max(1e-9, p["persist_kernel_ms"] * 1e-3) / 1e9,
                       kernel_us=p["persist_kernel_ms"] * 1e3, supersteps=n_sup, workgroups=wgs,
                       wg_kernel_us=t["kernel_ticks"] / 100 / wgs,
                       wait_us_per_superstep=t["wait_ticks"] / 100 / wgs / n_sup,
                       max_band_us=t["max_band_ticks"] / 100,
                       mean_band_us=t["band_ticks"] / 100 / max(1, wgs) / n_sup)
            print(json.dumps(rec), flush=True)
            tw = b.persist_trace_waves(wgs).astype(np.int64)
            act = tw[:, :, 1] > 0
            st = np.where(act, tw[:, :, 0], np.iinfo(np.int64).max).min(axis=1)
            dur = np.where(act, tw[:, :, 1] - tw[:, :, 0], 0)
            end = np.where(act, tw[:, :, 1], 0).max(axis=1)
            spread = (end - st) / 100.0
            mean_d = dur.sum(axis=1) / np.maximum(act.sum(axis=1), 1) / 100.0
            t0 = st.min()
            print(json.dumps(dict(wg_span_us_mean=float(spread.mean()), wave_mean_us=float(mean_d.mean()),
                                  wave_max_us=float(dur.max() / 100), wg_start_spread_us=float((st.max() - t0) / 100),
                                  per_wave_slot_mean_us=[round(float(x), 1) for x in
                                                         (np.where(act, dur, 0).sum(axis=0) / np.maximum(act.sum(axis=0), 1) / 100)[:16]])),
                  flush=True)
