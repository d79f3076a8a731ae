"""Parity of the 8-byte instructions in every hot loop of a libgolhip build.

On gfx950 the step kernels' 8-byte VALU instructions issue ~20 % faster at
addresses = 4 (mod 8) than at 0 (mod 8) (profiles/r2la: one 4-byte shift of
the same code costs 65536^2 120 -> 97 TCUPS); gol_kernels.hip's parity_fix
re-anchors every 3-row group.  This prints, per loop (a backward branch over
more than `--min` dwords) of the named kernels, how many 8-byte instructions
sit at each parity.  No GPU needed.

    python scripts/loop_parity.py game-of-life-distributed_amd/golhip/libgolhip.so [kernel-substring ...]
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT = ["gol_split_pair_kernelILi20ELi2E", "gol_tb_pair_kernelILi20ELi2ELb0", "gol_tb_pair_kernelILi8ELi4ELb0",
           "gol_persist_kernelILi16ELi2ELi8E"]


def disassemble(lib):
    with tempfile.TemporaryDirectory() as d:
        fb, dev = os.path.join(d, "fb.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={dev}", "--unbundle"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", dev], check=True,
                              capture_output=True, text=True).stdout.splitlines()


def kernels(lines):
    name, body = None, []
    for l in lines:
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", l)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name and l.strip():
            body.append(l)
    if name:
        yield name, body


def loops(body):
    """(start, end, Counter) of every loop (backward branch) in a kernel's disassembly."""
    ins = []
    for l in body:
        m = re.search(r"// ([0-9A-F]+): [0-9A-F]+( [0-9A-F]+)?", l)
        if m:
            ins.append((int(m.group(1), 16), 8 if m.group(2) else 4, l.split("//")[0].strip()))
    out = []
    for addr, size, txt in ins:
        m = re.match(r"(s_cbranch_\w+|s_branch)\s+(\d+)", txt)
        if not m:
            continue
        off = int(m.group(2))
        off = off - 65536 if off >= 32768 else off
        if off >= 0:
            continue
        tgt = addr + 4 + 4 * off
        out.append((tgt, addr, collections.Counter(f"b8@{x % 8}" if s == 8 else "b4"
                                                   for x, s, _ in ins if tgt <= x <= addr)))
    return ins, out


def main_loop_parity(lines, kernel):
    """Good-parity fraction of the kernel's main loop: the last innermost loop
    (no loop of >= 100 dwords inside it) with >= 500 8-byte instructions (the
    stream loops' main loop follows their fill loops)."""
    for name, body in kernels(lines):
        if kernel not in name:
            continue
        ins, lps = loops(body)
        inner = [l for l in lps if not any(o is not l and l[0] <= o[0] and o[1] <= l[1] and (o[1] - o[0]) >= 400
                                           for o in lps)]
        big = [l for l in inner if l[2]["b8@4"] + l[2]["b8@0"] >= 500]
        best = max(big, key=lambda l: l[0])
        c = best[2]
        return c["b8@4"] / max(1, c["b8@4"] + c["b8@0"]), c["b8@4"] + c["b8@0"]
    raise KeyError(kernel)


def inner_loops(lines, kernel, min_b8=300):
    """(start, good fraction, 8-byte count) of every innermost loop of the
    kernel with at least min_b8 8-byte instructions, in address order."""
    for name, body in kernels(lines):
        if kernel not in name:
            continue
        ins, lps = loops(body)
        inner = [l for l in lps if not any(o is not l and l[0] <= o[0] and o[1] <= l[1] and (o[1] - o[0]) >= 400
                                           for o in lps)]
        out = []
        for l in sorted(inner, key=lambda l: l[0]):
            n = l[2]["b8@4"] + l[2]["b8@0"]
            if n >= min_b8:
                out.append((l[0], l[2]["b8@4"] / max(1, n), n))
        return out
    raise KeyError(kernel)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("kernels", nargs="*", default=DEFAULT)
    ap.add_argument("--min", type=int, default=300, help="smallest loop (dwords) reported")
    a = ap.parse_args()
    for name, body in kernels(disassemble(a.lib)):
        if not any(k in name for k in a.kernels):
            continue
        ins = []
        for l in body:
            m = re.search(r"// ([0-9A-F]+): [0-9A-F]+( [0-9A-F]+)?", l)
            if m:
                ins.append((int(m.group(1), 16), 8 if m.group(2) else 4, l.split("//")[0].strip()))
        for addr, size, txt in ins:
            m = re.match(r"(s_cbranch_\w+|s_branch)\s+(\d+)", txt)
            if not m:
                continue
            off = int(m.group(2))
            off = off - 65536 if off >= 32768 else off
            tgt = addr + 4 + 4 * off
            if off >= 0 or -off < a.min:
                continue
            c = collections.Counter(f"b8@{x % 8}" if s == 8 else "b4" for x, s, _ in ins if tgt <= x <= addr)
            good = c["b8@4"] / max(1, c["b8@4"] + c["b8@0"])
            print(f"{name[:60]:60s} loop {tgt - ins[0][0]:#7x} +{(addr - tgt) // 4:5d} dw  "
                  f"b8@4 {c['b8@4']:5d}  b8@0 {c['b8@0']:5d}  b4 {c['b4']:4d}  good {good:.2f}")


if __name__ == "__main__":
    main()
