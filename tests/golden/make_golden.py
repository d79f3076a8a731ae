"""Generate tests/golden/ fixtures from the reference's own data files.

Run once in the build container (the only place /root/reference exists):

    python tests/golden/make_golden.py

It reads the reference's input boards (images/*.pgm), its golden boards
(check/images/*.pgm, used by gol_test.go:15-47 / pgm_test.go:10-42) and its
alive-count tables (check/alive/*.csv, used by count_test.go:17-69 and
sdl_test.go:93-128), and stores them as DATA:

* fixtures.npz   — boards bit-packed (uint32 words, cell (r, c) = bit c%32 of
                   word c//32 of row r, alive <=> byte == 255) and the alive
                   counts as int32 arrays indexed by completed turns (index 0
                   = the initial board, taken from the input image);
* manifest.json  — for every source file: size, SHA-256 and the exact PGM
                   header bytes, so tests can rebuild byte-identical PGM files.

No reference source is copied; the GPU box only ever sees these fixtures.
Provenance: reference data files are CC BY-NC-ND 4.0 (reference LICENSE:1).
"""
from __future__ import annotations

import csv
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.oracle import pack_bits, parse_pgm  # noqa: E402

REF = "/root/reference"
INPUTS = [16, 64, 128, 256, 512]
CHECKS = [(16, 0), (16, 1), (16, 100), (64, 0), (64, 1), (64, 100), (512, 0), (512, 1), (512, 100)]
ALIVE_CSV = [16, 64, 512]


def sha(data: bytes) -> str:
    return hashlib.sha256(data).hexdigest()


def header_of(data: bytes, W: int, H: int) -> bytes:
    return data[: len(data) - W * H]


def main() -> None:
    arrays: dict[str, np.ndarray] = {}
    manifest: dict[str, dict] = {}

    def add_board(key: str, rel: str, n: int) -> np.ndarray:
        with open(os.path.join(REF, rel), "rb") as f:
            data = f.read()
        board = parse_pgm(data, n, n)
        vals = sorted(set(np.unique(board).tolist()))
        assert set(vals) <= {0, 255}, (rel, vals)
        arrays[key] = pack_bits(board)
        manifest[key] = {
            "source": rel, "width": n, "height": n, "bytes": len(data),
            "sha256": sha(data), "header": header_of(data, n, n).decode("ascii"),
            "alive": int((board == 255).sum()),
        }
        return board

    for n in INPUTS:
        add_board(f"image_{n}", f"images/{n}x{n}.pgm", n)
    for n, t in CHECKS:
        add_board(f"check_{n}x{t}", f"check/images/{n}x{n}x{t}.pgm", n)

    for n in ALIVE_CSV:
        rel = f"check/alive/{n}x{n}.csv"
        with open(os.path.join(REF, rel), "rb") as f:
            data = f.read()
        rows = list(csv.reader(data.decode().splitlines()))
        assert rows[0] == ["completed_turns", "alive_cells"], rows[0]
        turns = [int(r[0]) for r in rows[1:]]
        assert turns == list(range(1, len(turns) + 1)), rel
        counts = np.zeros(len(turns) + 1, dtype=np.int32)
        counts[0] = manifest[f"image_{n}"]["alive"]
        counts[1:] = [int(r[1]) for r in rows[1:]]
        arrays[f"alive_{n}"] = counts
        manifest[f"alive_{n}"] = {"source": rel, "bytes": len(data), "sha256": sha(data),
                                  "turns": len(turns)}

    np.savez_compressed(os.path.join(HERE, "fixtures.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(f"wrote {len(arrays)} arrays")


if __name__ == "__main__":
    main()
