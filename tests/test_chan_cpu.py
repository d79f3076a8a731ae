"""gol::Chan (the host mirror's Go channel, csrc/gol_host.h) under contention:
values delivered exactly once and in per-sender order for capacities 0, 1, 7
and 1000 with 1 and 3 senders, single sends mixed with send_batch runs, close ends the range loop, send after close
fails (tests/cpp/chan_stress.cpp, built with g++ here; no GPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chan_stress(tmp_path):
    exe = tmp_path / "chan_stress"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "game-of-life-distributed_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "chan_stress.cpp"), "-o", str(exe)], check=True, timeout=120)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "chan stress ok" in p.stdout, p.stdout + p.stderr
