"""bench.py's multi-rank plumbing on CPU: `--gpus N`
without a launcher spawns its own N ranks (torchrun-style environment, before
any GPU call), fails fast with a JSON error line when there are fewer devices
than ranks, ends every rank when one fails, and a stage that hangs (a lost
RCCL peer) ends its rank through the watchdog with a JSON error line."""
import argparse
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

bench = pytest.importorskip("bench")


def _args(**kw):
    a = argparse.Namespace(gpus=2, steps=3, warmup=1, workload=65536, launch_timeout=60.0, stage_timeout=300.0)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _json_lines(text):
    return [json.loads(l) for l in text.splitlines() if l.startswith("{")]


def test_gpus_gt_devices_fails_fast_with_json_line():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""  # no device, even on a GPU box
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, p.stderr
    (line,) = _json_lines(p.stdout)
    assert line["value"] is None and line["n_gpus"] == 2
    assert "devices < 2 ranks" in line["error"]


def test_launcher_gives_every_rank_its_environment(tmp_path, capsys):
    child = textwrap.dedent(f"""
        import json, os
        r = os.environ["RANK"]
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GOL_BENCH_SELF_LAUNCH"]
        json.dump({{k: os.environ.get(k) for k in keys}}, open(os.path.join({str(tmp_path)!r}, r + ".json"), "w"))
        if r == "0":
            print(json.dumps({{"metric": "m", "value": 1.0}}))
    """)
    rc = bench.launch_ranks(_args(gpus=4), cmd=[sys.executable, "-c", child], n_devices=4)
    assert rc == 0
    out = capsys.readouterr().out
    assert _json_lines(out) == [{"metric": "m", "value": 1.0}]  # rank 0's line, relayed once
    envs = [json.load(open(tmp_path / f"{r}.json")) for r in range(4)]
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["GOL_BENCH_SELF_LAUNCH"] == "1"


def test_launcher_ends_the_others_when_one_rank_fails(capsys):
    child = "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(5)\ntime.sleep(600)\n"
    import time
    t0 = time.monotonic()
    rc = bench.launch_ranks(_args(gpus=3), cmd=[sys.executable, "-c", child], n_devices=3)
    assert time.monotonic() - t0 < 30
    assert rc != 0
    (line,) = _json_lines(capsys.readouterr().out)
    assert line["value"] is None and "rank 1 exited with status 5" in line["error"]


def test_launcher_timeout_ends_hung_ranks(capsys):
    rc = bench.launch_ranks(_args(gpus=2, launch_timeout=2.0), cmd=[sys.executable, "-c", "import time; time.sleep(600)"],
                            n_devices=2)
    assert rc != 0
    (line,) = _json_lines(capsys.readouterr().out)
    assert "launch-timeout" in line["error"]


def test_watchdog_ends_a_hung_stage_with_a_json_line():
    code = textwrap.dedent(f"""
        import argparse, sys, time
        sys.path.insert(0, {ROOT!r})
        import bench
        a = argparse.Namespace(gpus=2, steps=1, warmup=1, workload=65536)
        wd = bench.Watchdog(a, 0)
        wd.arm("golhip_comm_init", 1.0)
        time.sleep(60)
    """)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3
    (line,) = _json_lines(p.stdout)
    assert line["stage"] == "golhip_comm_init" and line["value"] is None and "watchdog" in line["error"]
