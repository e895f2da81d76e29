#!/usr/bin/env python3
"""bench.py -- TriAlign 3-D DP throughput on MI355X (GCUPS), driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload batch|single]
                    [--kernel auto|plane|pencil] [--per-gpu B] [--length L]

Workload (BASELINE.json metric "GCUPS + achieved HBM GB/s, 256^3 cube"):
  batch  (default) -- configs[4]'s per-GPU shard: B (default 512) independent
         256^3 synthetic triples per GPU, weak scaling: N GPUs score N*B
         triples, sharded contiguously, one process per GPU; the only
         collective is the RCCL all-gather of the int32 scores.
  single -- configs[2]: one 256^3 triple per GPU (replicas at N>1).
A "step" is one pass of the hot path over the GPU's batch, inputs already
resident in HBM. value = cells scored by all ranks / max-over-ranks time.
The single-cube latency (configs[2]) is always measured on rank 0 and
reported under "single_cube". Rank 0 checks a sample of the gathered scores
against the CPU oracle ("parity") and, at N=1, times the oracle on a bounded
sample of the same workload ("cpu_baseline").

Prints exactly one JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.environ.get("TSA_PKG_DIR", os.path.join(ROOT, "hw-accelerator-three-sequence-alignment_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
BYTES_PER_CELL = 28            # 7 int16 states written + read once
# VALU issue ceiling: 256 CU x 4 SIMD, one wave64 VALU instruction per 4 cycles
# per SIMD (MI355X_MICROARCH.md "vector-instruction ISSUE cost"), 2.4 GHz
VALU_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_pkg():
    spec = importlib.util.spec_from_file_location(
        "tsa_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["tsa_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_pmc(kernel_name: str, workload: str) -> dict:
    """Per-launch PMC figures from the committed profile (profiles/pmc_*.json,
    written by tools/pmc_traffic.py per the MI355X_MICROARCH.md HBM recipe):
    hbm_bytes_per_launch (FETCH_SIZE x2 + WRITE_SIZE) and valu_insts_per_launch."""
    path = os.path.join(ROOT, "profiles", f"pmc_{kernel_name}_{workload}.json")
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:  # noqa: BLE001
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["batch", "single"], default="batch")
    ap.add_argument("--kernel", choices=["auto", "plane", "pencil"], default="auto")
    ap.add_argument("--per-gpu", type=int, default=512)
    ap.add_argument("--length", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the configs[1]/configs[3] single-cube timings")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target wall time of the CPU-baseline sample")
    ap.add_argument("--check", type=int, default=4, help="triples checked vs the oracle")
    ap.add_argument("--score-bits", type=int, default=12,
                    help="12 = RTL wrap (default); 16/0 for cubes beyond the RTL envelope (1024^3)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    tsa = load_pkg()
    import tsa_amd.synth as synth  # noqa: E402
    import tsa_amd.shard as shard  # noqa: E402

    L = args.length
    per_gpu = args.per_gpu if args.workload == "batch" else 1
    n_total = per_gpu * world
    i0, i1 = shard.shard_range(n_total, rank, world)
    n = i1 - i0
    params = tsa.TsaParams.default(score_bits=args.score_bits)

    # ---- inputs resident in HBM before timing --------------------------------
    seqs, offs = synth.batch(i0, n, L)
    offs = offs - offs[0]
    d_seqs = torch.from_numpy(seqs).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    d_scores = torch.zeros(n, dtype=torch.int32, device=dev)
    ws_bytes = tsa.workspace_size(n, L, L, L, params, args.kernel)
    d_ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        tsa.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), n, L, L, L,
                              d_scores.data_ptr(), d_ws.data_ptr(), ws_bytes, stream.cuda_stream,
                              params, args.kernel)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms_per_step = ev0.elapsed_time(ev1) / args.steps
    elapsed_max = shard.max_over_ranks(elapsed, dev)

    cells_per_triple = L * L * L
    total_cells = n_total * cells_per_triple * args.steps
    gcups = total_cells / elapsed_max / 1e9
    ms_per_step = elapsed_max / args.steps * 1e3

    # ---- score gather (the one collective) + parity sample --------------------
    all_scores = shard.gather_scores(d_scores, n_total, world).cpu().numpy()

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    kind = args.kernel
    if kind == "auto":  # AUTO = pencil whenever its factored arithmetic is exact
        kind = "pencil" if _pencil_ok(tsa, L, params) else "plane"
    kernel_name = {"plane": "plane_step_kernel", "pencil": "pencil_kernel"}[kind]
    launches_per_step = (3 * L - 1) if kind == "plane" else 1
    # kernel, arithmetic and schedule the library picks (host-only query)
    plan = tsa.describe_plan(per_gpu, L, L, L, params, kernel=kind, sync=False)
    # exact integer values in f16 / int16 lanes; plane: int32 math on int16 planes
    arith = "f16" if " f16 " in plan else ("i32" if plan == "plane" else "i16")

    # per-rank kernel time of THIS rank's stream (HIP events on the launch stream)
    per_gpu_cells = n * cells_per_triple
    achieved_gbs = per_gpu_cells * BYTES_PER_CELL / (kernel_ms_per_step * 1e-3) / 1e9
    pmc = load_pmc(kernel_name, args.workload) if (L == 256 and per_gpu == 512) else {}
    traffic = pmc.get("hbm_bytes_per_launch")
    valu = None
    if pmc.get("valu_insts_per_launch") and kind == "pencil":
        # the binding resource of the pencil kernel: VALU issue (states never
        # leave the chip, so the 28 B/cell streaming roofline is exceeded)
        insts = pmc["valu_insts_per_launch"]
        ach = insts / (kernel_ms_per_step * 1e-3)
        valu = {"bound": "valu", "achieved": round(ach / 1e9, 2), "peak": VALU_WAVE_INSTR_PER_S / 1e9,
                "unit": "G wave-instr/s", "frac": round(ach / VALU_WAVE_INSTR_PER_S, 4),
                "insts_per_launch": insts,
                "lane_insts_per_cell": round(insts * 64 / per_gpu_cells, 3),
                "source": f"SQ_INSTS_VALU, profiles/pmc_{kernel_name}_{args.workload}.json"}

    # single-cube latency: configs[2] (L^3, params as the batch), plus configs[1]
    # (64^3) and configs[3] (1024^3, 16-bit words: beyond the RTL envelope)
    def time_single(Ls, prm, reps=5):
        sa = synth.batch(0, 1, Ls)
        s_seqs = torch.from_numpy(sa[0]).to(dev)
        s_offs = torch.from_numpy(sa[1]).to(dev)
        s_score = torch.zeros(1, dtype=torch.int32, device=dev)
        s_ws = tsa.workspace_size(1, Ls, Ls, Ls, prm, args.kernel)
        s_wsb = torch.empty(max(s_ws, 16), dtype=torch.uint8, device=dev)

        def sstep():
            tsa.score_batch_async(s_seqs.data_ptr(), s_offs.data_ptr(), 1, Ls, Ls, Ls,
                                  s_score.data_ptr(), s_wsb.data_ptr(), s_ws, stream.cuda_stream,
                                  prm, args.kernel)
        sstep()
        torch.cuda.synchronize()
        times = []  # median of individually timed calls (a latency, not a throughput)
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            sstep()
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        sms = float(np.median(times))
        return {"ms": round(sms, 4), "gcups": round(Ls ** 3 / (sms * 1e-3) / 1e9, 3),
                "score": int(s_score.item()), "score_bits": prm.score_bits}

    single = None
    other_configs = {}
    try:
        single = {"config": f"configs[2]: one {L}^3 triple", **time_single(L, params)}
        if not args.no_extra_configs:
            other_configs["configs[1]: one 64^3 triple"] = time_single(64, params, reps=10)
            other_configs["configs[3]: one 1024^3 triple"] = time_single(
                1024, tsa.TsaParams.default(score_bits=16), reps=7)
    except Exception as e:  # noqa: BLE001
        log("single-cube measurement failed:", e)

    # parity sample vs the CPU oracle (checker only)
    parity = None
    cpu_baseline = None
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # noqa: E402
        nthreads = max(1, min(16, os.cpu_count() or 1))
        idx = sorted(set([0, n_total - 1] + [int(v) for v in np.linspace(0, n_total - 1, args.check)]))
        trip = [synth.triple(i, L) for i in idx]
        cs, co = tsa.pack_batch(trip)
        oparams = oracle.default_params(score_bits=args.score_bits)
        ref = oracle.score_batch(cs, co, oparams, nthreads=nthreads)
        got = all_scores[idx]
        parity = {"checked": len(idx), "mismatches": int((ref != got).sum()),
                  "against": "oracle/tsa_oracle.c"}
        if single is not None:
            parity["single_cube_ok"] = bool(single["score"] == int(ref[0]))
        if world == 1 and not args.no_cpu_baseline:
            # bounded sample of the same workload: one 256^3 triple per thread per round
            t_one = oracle.now()
            oracle.score_batch(cs[: 3 * L], co[:4], oparams, nthreads=1)
            t_one = oracle.now() - t_one
            rounds = max(1, int(args.cpu_seconds / max(t_one, 1e-3)))
            ns = nthreads * rounds
            bs, bo = synth.batch(0, ns, L)
            t = oracle.now()
            oracle.score_batch(bs, bo, oparams, nthreads=nthreads)
            t = oracle.now() - t
            cpu_baseline = {
                "value": round(ns * cells_per_triple / t / 1e9, 5), "unit": "GCUPS",
                "cores": nthreads, "kind": "port",
                "sample": f"{ns} synthetic {L}^3 triples (same generator) on {nthreads} threads, "
                          f"{t:.1f} s wall; 1-thread rate {cells_per_triple / t_one / 1e9:.4f} GCUPS; "
                          f"oracle/tsa_oracle.c literal RTL form, gcc -O2",
            }
    except Exception as e:  # noqa: BLE001
        log("oracle leg failed:", e)

    out = {
        "metric": "GCUPS (10^9 3D-DP cell updates/s), 256^3 cubes",
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": arith,
        "data": "synthetic (splitmix64 uniform DNA, SURVEY.md 8d seeds)",
        "config": {
            "workload": (f"batch: {per_gpu} independent {L}^3 triples per GPU (configs[4] per-GPU shard)"
                         if args.workload == "batch" else f"single: one {L}^3 triple per GPU (configs[2])"),
            "length": L, "triples_per_gpu": per_gpu, "triples_total": n_total,
            "kernel": kind, "plan": plan, "launches_per_step": launches_per_step,
            "parallelism": f"shard{world}", "score_bits": params.score_bits,
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": kernel_name, "bytes_per_cell": BYTES_PER_CELL,
            "kernel_ms_per_step": round(kernel_ms_per_step, 4),
            "traffic_bytes_per_cell": (round(traffic / per_gpu_cells, 3) if traffic else None),
            "valu": valu,
        },
        "cpu_baseline": cpu_baseline,
        "single_cube": single,
        "other_configs": other_configs,
        "parity": parity,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _pencil_ok(tsa, L, params):
    try:
        tsa.workspace_size(1, L, L, L, params, "pencil")
        return True
    except tsa.TsaError:
        return False


if __name__ == "__main__":
    main()
