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


# ---------------------------------------------------------------- configs[3] block
FULLSIZE = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))


class _FakeBoard:
    """Stands in for golhip.Board: turns advance, the digest / alive count are
    the fixture's at the checkpoint (rank 0's share; the others add 0), or a
    wrong digest for the configs named in `bad`."""

    def __init__(self, W, H, row0, rows, rank, bad):
        self.W, self.rows, self.rank, self.bad = W, rows, rank, bad
        self.key = {65536: "c2", 262144: "c3"}[W]
        self.turn = 0
        self.closed = False

    def set_tb_depth(self, d): pass
    def set_rows_per_wave(self, r): pass
    def set_option(self, k, v): pass
    def comm_init(self, uid, n, r): self.comm = (n, r)
    def comm_info(self): return {"nranks": self.comm[0], "rank": self.comm[1], "ring_rows": self.rows}
    def fill_random(self, seed): self.turn = 0
    def step(self, n): self.turn += n
    def sync(self): pass
    def stream(self): return 0
    def perf_reset(self): pass
    def close(self): self.closed = True

    def _cp(self):
        return FULLSIZE[self.key]["checkpoints"].get(str(self.turn))

    def board_hash(self):
        cp = self._cp()
        if self.rank or cp is None:
            return 0
        return int(cp["hash"], 16) ^ (1 if self.key in self.bad else 0)

    def alive_count(self, global_sum=False):
        cp = self._cp()
        return (cp["alive"] if cp and self.rank == 0 else 0), self.turn

    def perf(self):
        wpl = 4 if self.W == 262144 else 2
        return {"persist_turns": 0, "step_turns": 100, "step_launches": 10, "skew_launches": 10,
                "tb_depth": 9 if wpl == 4 else 20, "words_per_lane": wpl,
                "persist_launches": 0, "persist_depth": 0, "rows_per_wave": 0, "halo_bytes": 0,
                "halo_exchanges": 0}


def _fake_env(world=1, bad=()):
    boards = []

    class FakeEnv:
        def __init__(self, a, world_, rank, local):
            self.a, self.world, self.rank, self.local, self.dist = a, world, 0, 0, None

        def stage(self, name): pass

        def board(self, W, H, row0, rows):
            b = _FakeBoard(W, H, row0, rows, self.rank, bad)
            boards.append(b)
            return b

        def unique_id(self): return b"x"
        def ring_init(self, board, tag=""): board.comm_init(self.unique_id(), self.world, self.rank)
        def barrier(self, board): pass
        def gsum(self, x): return x % (1 << 64)
        def gmax(self, x): return x
        def bcast(self, x): return x

        def gather(self, obj):  # every rank's row, as rank r would report it
            return [dict(obj, rank=r, row0=r * obj["rows"]) for r in range(self.world)]

        def region_timer(self, board):
            class T:
                def start(self): pass
                def stop(self): return 1.0
            return T()

        def close(self): pass

    return FakeEnv, boards


def _run_main(monkeypatch, capsys, argv, env):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    code = 0
    try:
        bench.main(env_factory=env)
    except SystemExit as e:
        code = e.code
    return code, _json_lines(capsys.readouterr().out)


@pytest.mark.parametrize("world", [1, 2, 8])
def test_default_line_carries_a_configs3_block(monkeypatch, capsys, world):
    env, boards = _fake_env(world)
    if world > 1:
        monkeypatch.setenv("WORLD_SIZE", str(world))
        monkeypatch.setenv("RANK", "0")
    code, (line,) = _run_main(monkeypatch, capsys, ["--gpus", str(world), "--steps", "3", "--no-cpu-baseline",
                                                    "--warmup-seconds", "0", "--configs3-warmup-seconds", "0"], env)
    assert code == 0 and line["parity"] is True
    assert line["config"]["board"] == [65536, 65536] and line["value"] > 0  # the primary value stays configs[2]
    c3 = line["configs3"]
    assert c3["config"]["board"] == [262144, 262144] and c3["config"]["turns_per_step"] == 100
    assert c3["config"]["rows_per_rank"] == 262144 // world and c3["n_gpus"] == world and c3["steps"] == 3
    assert c3["parity"] is True and c3["parity_check"]["fixture"] == "tests/golden/fullsize.json c3 turn 100"
    assert c3["parity_check"]["alive"] == FULLSIZE["c3"]["checkpoints"]["100"]["alive"]
    assert c3["value"] > 0 and c3["unit"] == "GCUPS" and c3["scaling"] == "strong"
    assert c3["roofline"]["frac"] > 0 and c3["config"]["words_per_lane"] == 4
    if world > 1:
        assert [r["rank"] for r in c3["config"]["ranks"]] == list(range(world))
        assert {r["rows"] for r in c3["config"]["ranks"]} == {262144 // world}
    assert [b.W for b in boards] == [65536, 262144] and all(b.closed for b in boards)  # one board at a time


def test_configs3_parity_failure_fails_the_line(monkeypatch, capsys):
    env, _ = _fake_env(1, bad=("c3",))
    code, (line,) = _run_main(monkeypatch, capsys, ["--steps", "1", "--no-cpu-baseline", "--warmup-seconds", "0",
                                                    "--configs3-warmup-seconds", "0"], env)
    assert code == 1 and line["parity"] is False and line["configs3"]["parity"] is False
    assert line["parity_check"]["ok"] is True  # configs[2] itself was right


def test_no_configs3_flag_and_other_workloads_skip_the_block(monkeypatch, capsys):
    env, boards = _fake_env(1)
    code, (line,) = _run_main(monkeypatch, capsys, ["--steps", "1", "--no-cpu-baseline", "--warmup-seconds", "0",
                                                    "--no-configs3"], env)
    assert code == 0 and "configs3" not in line and [b.W for b in boards] == [65536]


def test_cpu_share_is_measured():
    s = bench.cpu_share()
    assert s["affinity"] == len(os.sched_getaffinity(0)) and 1 <= s["threads"] <= s["affinity"]
    assert s["gomaxprocs_equiv"] == s["threads"]


def test_count_gpus_honours_visible_devices(monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.count_gpus()[0] == 0
