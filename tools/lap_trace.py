#!/usr/bin/env python3
"""Single-cube lap-kernel timeline (TSA_LAP_TRACE): per (lap, tile) workgroup
start / loop-begin / loop-end in microseconds from the first workgroup start,
and the per-lap hand-off delay (loop begin of lap L+1 minus lap L). Run on the
GPU box: python tools/lap_trace.py [L] [score_bits]."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    bits = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    import torch  # noqa: F401
    import bench
    tsa = bench.load_pkg()
    import tsa_amd.synth as synth
    path = os.path.join(ROOT, "gpurun_out", f"lap_trace_{L}.csv")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    a, b, c = synth.triple(0, L)
    p = tsa.TsaParams.default(score_bits=bits)
    tsa.score(a, b, c, p, kernel="pencil")  # warm-up
    os.environ["TSA_LAP_TRACE"] = path
    s = tsa.score(a, b, c, p, kernel="pencil")
    del os.environ["TSA_LAP_TRACE"]
    rows = list(csv.DictReader(open(path)))
    t0 = min(int(r["start"]) for r in rows)
    us = lambda v: (int(v) - t0) / 100.0  # s_memrealtime: 100 MHz
    laps = {}
    for r in rows:
        laps.setdefault(int(r["lap"]), []).append(r)
    out = []
    for lp in sorted(laps):
        rs = laps[lp]
        out.append({"lap": lp, "start": round(min(us(r["start"]) for r in rs), 2),
                    "loop_begin": round(min(us(r["loop_begin"]) for r in rs), 2),
                    "loop_end": round(max(us(r["loop_end"]) for r in rs), 2),
                    "polls": sum(int(r["polls"]) for r in rs), "spins": sum(int(r["spins"]) for r in rs)})
    ends = [o["loop_end"] for o in out]
    print(json.dumps({"L": L, "score": s, "wgs": len(rows), "total_us": max(ends),
                      "plan": tsa.describe_plan(1, L, L, L, p)}))
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
