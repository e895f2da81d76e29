#!/usr/bin/env python3
"""A/B timing of kernel variants in ONE process, interleaved rounds (guide
rule 24). Variants are environment knobs read by libtrialign at launch.
  python tools/bench_variants.py --variants "TSA_PENCIL_NW=16" "TSA_PENCIL_NW=8,TSA_PENCIL_STAGGER=14"
A variant is a comma-separated list of KEY=VALUE; every key named by any
variant is unset before each run, so variants never inherit each other's knobs.
Prints one JSON line per variant (median/min ms, GCUPS) to stdout."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--L", type=int, default=256)
    ap.add_argument("--kernel", default="pencil")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--score-bits", type=int, default=12)
    ap.add_argument("--preload", action="store_true",
                    help="queue a ~1 ms matmul before each timed call, so the events time the "
                         "device work and not the host's submission (small cubes)")
    args = ap.parse_args()
    import torch
    import bench
    tsa = bench.load_pkg()
    import tsa_amd.synth as synth
    L, n = args.L, args.n
    seqs, offs = synth.batch(0, n, L)
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_scores = torch.zeros(n, dtype=torch.int32, device="cuda")
    p = tsa.TsaParams.default(score_bits=args.score_bits)
    ws = 0
    keys = sorted({kv.split("=", 1)[0] for v in args.variants for kv in v.split(",") if kv})

    def apply(v):
        for k in keys:
            os.environ.pop(k, None)
        for kv in v.split(","):
            if kv:
                k, val = kv.split("=", 1)
                os.environ[k] = val

    for v in args.variants:  # workspace depends on the knobs: take the max
        apply(v)
        ws = max(ws, tsa.workspace_size(n, L, L, L, p, args.kernel))
    d_ws = torch.empty(ws, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    times = {v: [] for v in args.variants}
    scores = {}

    def run(v):
        apply(v)
        tsa.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), n, L, L, L, d_scores.data_ptr(),
                              d_ws.data_ptr(), ws, st.cuda_stream, p, args.kernel)

    for v in args.variants:  # warm-up
        run(v)
    torch.cuda.synchronize()
    pre = torch.randn(4096, 4096, device="cuda") if args.preload else None
    for _ in range(args.rounds):
        for v in args.variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if pre is not None:  # a spin (no memory traffic), else a matmul
                if hasattr(torch.cuda, "_sleep"):
                    torch.cuda._sleep(2_000_000)
                else:
                    torch.mm(pre, pre)
            e0.record(st)
            run(v)
            e1.record(st)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
            scores[v] = d_scores.cpu().numpy().copy()
    ref = None
    if args.check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        idx = list(range(0, n, max(1, n // 8)))
        trip = [synth.triple(i, L) for i in idx]
        cs, co = tsa.pack_batch(trip)
        ref = oracle.score_batch(cs, co, oracle.default_params(score_bits=args.score_bits), nthreads=8)
    plans = {}
    for v in args.variants:
        apply(v)
        try:
            plans[v] = tsa.describe_plan(n, L, L, L, p, args.kernel, sync=False)
        except Exception as e:  # noqa: BLE001 -- a label only
            plans[v] = f"? ({e})"
    for v in args.variants:
        med = statistics.median(times[v])
        rec = {"variant": v, "n": n, "L": L, "median_ms": round(med, 4), "min_ms": round(min(times[v]), 4),
               "gcups": round(n * L ** 3 / (med * 1e-3) / 1e9, 2), "plan": plans[v]}
        if ref is not None:
            rec["parity_ok"] = bool((scores[v][idx] == ref).all())
        # every variant must score the batch identically (and never the
        # TSA_SCORE_INVALID of a timed-out hand-off)
        rec["agree"] = bool((scores[v] == scores[args.variants[0]]).all()) and int(scores[v].min()) > -(1 << 30)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
