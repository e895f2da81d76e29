#!/usr/bin/env python3
"""Single-cube lap-kernel diagnostics on the GPU box (TSA_LAP_TRACE).

    python tools/lap_trace.py [--bits 12] [--reps 5] SPEC [SPEC ...]

SPEC = LA[xLBxLC][:KEY=VAL,KEY=VAL...], e.g. 64, 256, 64x16x64:TSA_LAP_NW=8.
Knobs are libtrialign environment knobs (TSA_PENCIL_MODE=lap is always set).
Per spec one JSON line: the median event-timed latency of `reps` calls, then
from one traced call the lap-to-lap lag of the loop ends (the hand-off
chain), each
workgroup's loop time per step (us and shader-clock cycles; the clock in MHz),
loader stalls (tag re-fetches), wave 0's missed progress polls and
the producers' back-pressure waits. Traces land in
gpurun_out/lap_trace_<spec>.csv."""
import argparse
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_spec(spec):
    shape, _, knobs = spec.partition(":")
    dims = [int(v) for v in shape.split("x")]
    la, lb, lc = (dims * 3)[:3] if len(dims) == 1 else dims
    env = dict(kv.split("=", 1) for kv in knobs.split(",") if kv)
    return la, lb, lc, env


def lap_steps(la, lb, lc, lap, tile, M, NW, SK=1):
    """Steps of workgroup (lap, tile): lap_kernel.hip's T."""
    RW, ZT, WO = 2 * NW, 64 * M, SK + 1
    tau = lambda r: WO * (r >> 1) + (r & 1)
    rows = min(RW, lb - lap * RW)
    zt = min(ZT, lc - tile * ZT)
    return la + tau(rows - 1) + zt - 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--bits", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kernel", default="pencil", help="pencil, or checked (the lap kernel with the range monitor)")
    args = ap.parse_args()
    import torch
    import bench
    tsa = bench.load_pkg()
    import tsa_amd.synth as synth
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    p = tsa.TsaParams.default(score_bits=args.bits)
    for spec in args.specs:
        la, lb, lc, env = parse_spec(spec)
        env.setdefault("TSA_PENCIL_MODE", "lap")
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            a, b, c = synth.triple(0, la, lb, lc)
            seqs, offs = tsa.pack_batch([(a, b, c)])
            d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
            d_sc = torch.zeros(1, dtype=torch.int32, device="cuda")
            ws = tsa.workspace_size(1, la, lb, lc, p, args.kernel)
            d_ws = torch.empty(max(ws, 16), dtype=torch.uint8, device="cuda")
            st = torch.cuda.current_stream()

            def call():
                tsa.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), 1, la, lb, lc,
                                      d_sc.data_ptr(), d_ws.data_ptr(), ws, st.cuda_stream, p, args.kernel)
            call()
            torch.cuda.synchronize()
            times = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                call()
                e1.record(st)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3)
            score = int(d_sc.item())
            plan = tsa.describe_plan(1, la, lb, lc, p, kernel=args.kernel, sync=False)
            path = os.path.join(out_dir, "lap_trace_" + re.sub(r"[^0-9A-Za-z_=.-]", "_", spec) + ".csv")
            os.environ["TSA_LAP_TRACE"] = path
            call()
            torch.cuda.synchronize()
            del os.environ["TSA_LAP_TRACE"]
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        rec = {"spec": spec, "plan": plan, "score": score, "us_median": round(statistics.median(times), 2),
               "us_min": round(min(times), 2)}
        m = re.search(r"M=(\d+) NW=(\d+)", plan)
        if m and os.path.exists(path):
            M, NW = int(m.group(1)), int(m.group(2))
            rows = list(csv.DictReader(open(path)))
            t0 = min(int(r["start"]) for r in rows)
            us = lambda v: (int(v) - t0) / 100.0  # s_memrealtime: 100 MHz
            laps = {}
            per_step_us, per_step_clk, mhz = [], [], []
            for r in rows:
                lp, tl = int(r["lap"]), int(r["tile"])
                laps.setdefault(lp, []).append(us(r["loop_begin"]))
                T = lap_steps(la, lb, lc, lp, tl, M, NW)
                dt = us(r["loop_end"]) - us(r["loop_begin"])
                clk = int(r.get("loop_clk") or 0)
                per_step_us.append(dt / T)
                if clk and dt > 0:
                    per_step_clk.append(clk / T)
                    mhz.append(clk / dt)
            ends = {}
            for r in rows:
                lp = int(r["lap"])
                ends[lp] = max(ends.get(lp, 0.0), us(r["loop_end"]))
            # every workgroup starts at once (its prologue waits for nothing), so
            # the chain shows in the loop ends: lap L+1 ends one hand-off after lap L
            e = [ends[k] for k in sorted(ends)]
            lags = [round(b1 - b0, 2) for b0, b1 in zip(e, e[1:])]
            rec.update({
                "wgs": len(rows), "trace_total_us": round(max(us(r["loop_end"]) for r in rows), 2),
                "lap_end_lag_us": {"median": round(statistics.median(lags), 2) if lags else None,
                               "max": max(lags) if lags else None, "first": lags[:4]},
                "step_us": {"median": round(statistics.median(per_step_us), 4),
                            "max": round(max(per_step_us), 4)},
                "step_clk": round(statistics.median(per_step_clk), 1) if per_step_clk else None,
                "clock_mhz": round(statistics.median(mhz)) if mhz else None,
                "stalls": sum(int(r["stalls"]) for r in rows),
                "w0_waits": sum(int(r.get("w0_waits") or 0) for r in rows),
                "bp_waits": sum(int(r["bp_waits"]) for r in rows),
            })
            prof_cols = [k for k in rows[0] if k.startswith("prof")]
            if prof_cols:  # TSA_DIAG build: per-wave cycles per step (medians over workgroups)
                prof = {}
                for wv in range(NW):
                    parts = []
                    for ph in range(4):
                        vals = [int(r[f"prof{wv}_{ph}"]) / lap_steps(la, lb, lc, int(r["lap"]), int(r["tile"]), M, NW)
                                for r in rows]
                        parts.append(round(statistics.median(vals), 1))
                    prof[f"w{wv}"] = parts
                rec["prof_clk_per_step"] = {"phases": "reads+pre, check, post+stores, gap", **prof}
            if "lag_y" in rows[0]:  # TSA_DIAG: the ring slots each workgroup needed
                for key in ("lag_y", "lag_z"):
                    vals = sorted(int(r[key]) for r in rows)
                    by_tile, by_lap = {}, {}
                    for r in rows:
                        v, tl, lp = int(r[key]), int(r["tile"]), int(r["lap"])
                        by_tile[tl] = max(by_tile.get(tl, 0), v)
                        by_lap[lp] = max(by_lap.get(lp, 0), v)
                    q = lambda f: vals[min(len(vals) - 1, int(f * len(vals)))]
                    rec[key] = {"max": vals[-1], "p50": q(0.5), "p90": q(0.9), "p99": q(0.99),
                                "by_tile": [by_tile[k] for k in sorted(by_tile)],
                                "by_lap_q": [by_lap[k] for k in sorted(by_lap)][:: max(1, len(by_lap) // 16)]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
