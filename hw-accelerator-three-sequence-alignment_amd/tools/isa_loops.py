#!/usr/bin/env python3
"""Per-loop instruction counts of one kernel in a built object (static ISA census).

    python tools/isa_loops.py build/lap_kernel.o 'lap_kernelILi1ELi4ELb1ELb1ELb0ELb0ELb0ELb0E' [--min 150]

Extracts the gfx950 code object from the object's .hip_fatbin, disassembles
the first kernel whose symbol contains the given fragment, and for every loop
(a backward branch) of at least --min instructions prints:
  * `body`: every instruction between the header and the back-edge, by class
    (VALU / SALU / DS / VMEM / SMEM / branch+waitcnt+nop), slow paths included;
  * `fast`: the shortest header -> back-edge path through the loop's CFG, with
    `s_cbranch_execz` taken as not taken (a lane-masked store runs) and every
    inner loop (a spin on a progress word) entered zero times -- the
    instructions one pass of the loop issues when no wait spins. Blocks under
    a uniform run-time condition (e.g. `if (zout)`) count only when the
    shortest path needs them, so `fast` is a lower bound for the waves that
    execute them; `body` bounds it above.
A step-unrolled loop's counts divide by its steps per pass (the caller knows).
"""
import argparse
import collections
import heapq
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
LINE = re.compile(r"^\s+([a-z_0-9]+)\b(.*?)//\s*([0-9A-F]{12}):")
BR = re.compile(r"^s_(cbranch_\w+|branch)$")


def disassemble(obj: str) -> list:
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat"), os.path.join(td, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout.split("\n")


def kernel_insts(lines: list, frag: str) -> list:
    """[(addr, mnemonic, operands)] of the first symbol containing frag."""
    out, on = [], False
    for ln in lines:
        if ln.endswith(">:") and "<" in ln:
            if on:
                break
            on = frag in ln
            continue
        if on:
            m = LINE.match(ln)
            if m:
                out.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return out


def klass(mn: str) -> str:
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("ds_"):
        return "ds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith(("s_load", "s_buffer_load", "s_store", "s_memtime", "s_memrealtime", "s_dcache")):
        return "smem"
    if BR.match(mn) or mn in ("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_setprio", "s_endpgm"):
        return "ctl"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def target(ops: str, addr: int):
    """Branch target: llvm-objdump prints the word offset; target = addr + 4 + 4 * simm16."""
    m = re.match(r"(-?\d+)", ops)
    if not m:
        return None
    off = int(m.group(1))
    if off >= 32768:
        off -= 65536
    return addr + 4 + 4 * off


def census(ins: list, lo: int, hi: int) -> collections.Counter:
    c = collections.Counter()
    for a, mn, _ in ins:
        if lo <= a <= hi:
            c[klass(mn)] += 1
    return c


def fast_path(ins: list, head: int, tail: int, inner: list) -> collections.Counter:
    """Shortest (instruction count) path from head to the back-edge at tail."""
    idx = {a: i for i, (a, _, _) in enumerate(ins)}
    i0, i1 = idx[head], idx[tail]
    in_inner = lambda a: any(lo <= a <= hi for lo, hi in inner)
    dist = {i0: 0}
    prev = {}
    pq = [(0, i0)]
    while pq:
        d, i = heapq.heappop(pq)
        if d > dist.get(i, 1 << 30):
            continue
        if i == i1:
            break
        a, mn, ops = ins[i]
        nxt = []
        if BR.match(mn):
            t = target(ops, a)
            if mn != "s_branch":
                nxt.append(i + 1)
            if t is not None and t in idx and mn != "s_cbranch_execz" and head <= t <= tail and t > a:
                nxt.append(idx[t])
        else:
            nxt.append(i + 1)
        for j in nxt:
            if j > i1 or in_inner(ins[j][0]):
                continue
            nd = d + 1
            if nd < dist.get(j, 1 << 30):
                dist[j] = nd
                prev[j] = i
                heapq.heappush(pq, (nd, j))
    if i1 not in dist:
        return collections.Counter()
    c = collections.Counter()
    j = i1
    while True:
        c[klass(ins[j][1])] += 1
        if j == i0:
            break
        j = prev[j]
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=150)
    args = ap.parse_args()
    ins = kernel_insts(disassemble(args.obj), args.kernel)
    if not ins:
        sys.exit(f"no kernel matching {args.kernel}")
    loops = []
    for a, mn, ops in ins:
        if BR.match(mn):
            t = target(ops, a)
            if t is not None and t < a:
                loops.append((t, a))
    fmt = lambda c: " ".join(f"{k}={c[k]}" for k in ("valu", "salu", "ds", "vmem", "smem", "ctl") if c[k])
    for head, tail in sorted(loops):
        n = sum(1 for a, _, _ in ins if head <= a <= tail)
        if n < args.min:
            continue
        inner = [(h, t) for h, t in loops if head < h and t < tail]
        print(f"loop {head:#x}..{tail:#x}: body {fmt(census(ins, head, tail))} | "
              f"fast {fmt(fast_path(ins, head, tail, inner))}")


if __name__ == "__main__":
    main()
