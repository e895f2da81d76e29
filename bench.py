#!/usr/bin/env python3
"""bench.py -- TriAlign 3-D DP throughput on MI355X (GCUPS), driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload batch|single]
                    [--kernel auto|plane|pencil] [--per-gpu B] [--length L]

Workload (BASELINE.json metric "GCUPS + achieved HBM GB/s, 256^3 cube"):
  batch  (default) -- configs[4]: "4096 independent 256^3 triples sharded across
         8 GPUs", i.e. B = 512 triples per GPU; weak scaling: N GPUs score N*B
         triples, sharded contiguously, one process per GPU; the only
         collective is the RCCL all-gather of the int32 scores.
  single -- configs[2]: one 256^3 triple per GPU (replicas at N>1).
A "step" is one pass of the hot path over the GPU's batch, inputs already
resident in HBM. value = cells scored by all ranks / max-over-ranks time.

Ranks: under torch.distributed.run (WORLD_SIZE set) this process is one rank
and --gpus must equal WORLD_SIZE. Started directly with --gpus N > 1, this
process starts the N rank processes itself (RANK/LOCAL_RANK/WORLD_SIZE set
before any of them touches the GPU; this parent never does) and exits with
their status.

Rank 0 also times single cubes (configs[1..3] and the paper's Table III sizes
128^3 / 512^3, "single_cube"), checks a sample of the gathered scores against
the CPU oracle ("parity") and, at N=1, times the oracle on a bounded sample of
the same workload on every host core the job may use ("cpu_baseline").

Prints exactly one JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import hashlib
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.environ.get("TSA_PKG_DIR", os.path.join(ROOT, "hw-accelerator-three-sequence-alignment_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
BYTES_PER_CELL = 28            # 7 int16 states written + read once
# VALU issue ceiling of the packed-16-bit wave64 instructions the pencil kernel
# issues: 256 CU x 4 SIMD x 2.4 GHz / 4 cycles per instruction per SIMD. The
# 4 cycles are measured (tools/valu_peak.hip -> profiles/r3_valu_peak.jsonl):
# v_pk_maximum3_f16, v_pk_add_f16, v_pk_fma_f32, v_pk_max_i16, v_bfi_b32,
# v_perm_b32, DPP movs and v_max_i32 / v_max3_f32 top out at 0.23-0.24
# instructions per cycle per SIMD at 4-8 waves; the same harness does see the
# guide's faster issue (MI355X_MICROARCH.md:54,473) on v_add_u32 (0.40-0.43,
# 2 cycles) and partly on v_fma_f32 (0.28), so 4 cycles is the packed ops'
# own cost, not a limit of the harness.
VALU_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 4
VALU_PEAK_SOURCE = ("profiles/r3_valu_peak.jsonl (tools/valu_peak.hip: packed-16 ops 0.24 "
                    "instr/cycle/SIMD; 2-cycle control v_add_u32 0.43; MI355X_MICROARCH.md:54,473)")
# Cubes the split-over-devices leg times (tools/split_cube.py --lengths)
SPLIT_LENGTHS = "256,1024,1024r"  # 1024r: the RTL's 12-bit words, literal split
# Paper Table III (pic/Result.png): ASIC runtime per N^3 cube, ms
ASIC_MS = {64: 0.03, 128: 0.19, 256: 1.39, 512: 10.82}

# Kernel sources whose instruction stream a committed PMC profile describes
# (bench refuses a profile whose stamp differs: the counters would be stale).
KERNEL_SOURCES = {
    "pencil_kernel": ["pencil_kernel.hip", "pencil_kernel.h", "pencil_common.h", "tsa_internal.h"],
    "plane_step_kernel": ["plane_kernel.hip", "tsa_internal.h"],
    "lap_kernel": ["lap_kernel.hip", "lap_kernel.h", "pencil_common.h", "pencil_kernel.h", "tsa_internal.h"],
}
# Lane-operations per cell of the V-space pair core (cell_messages_vs: 24
# packed instructions per pair of cells = 12 per cell), the algorithmic VALU
# work of one cell; DESIGN.md 4.2
CORE_LANE_OPS_PER_CELL = 12


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_source_hash(kernel_name: str) -> str:
    h = hashlib.sha256()
    for fn in KERNEL_SOURCES.get(kernel_name, []):
        p = os.path.join(PKG_DIR, "csrc", fn)
        if os.path.exists(p):
            with open(p, "rb") as f:
                h.update(fn.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def load_pkg():
    if "tsa_amd" in sys.modules:
        return sys.modules["tsa_amd"]
    spec = importlib.util.spec_from_file_location(
        "tsa_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["tsa_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_pmc(kernel_name: str, workload: str) -> dict:
    """Per-launch PMC figures from the committed profile (profiles/pmc_*.json,
    written by tools/pmc_traffic.py per the MI355X_MICROARCH.md HBM recipe):
    hbm_bytes_per_launch (2 x FETCH_SIZE + WRITE_SIZE) and
    valu_insts_per_launch (SQ_INSTS_VALU). Refused ({"stale": ...}) when its
    source stamp is not the hash of the kernel sources in this tree."""
    path = os.path.join(ROOT, "profiles", f"pmc_{kernel_name}_{workload}.json")
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as f:
            pmc = json.load(f)
    except Exception:  # noqa: BLE001
        return {}
    want = kernel_source_hash(kernel_name)
    if pmc.get("kernel_source_sha256") != want:
        return {"stale": f"{os.path.relpath(path, ROOT)} stamped "
                         f"{pmc.get('kernel_source_sha256')}, sources {want}"}
    return pmc


def host_cores() -> int:
    """Host cores this job may use: the affinity mask, capped by a cgroup CPU
    quota (the GPU box gives each job a share of a larger machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                n = min(n, max(1, int(int(quota) // int(period))))
        except (OSError, ValueError):
            pass
    return max(1, n)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list[str], script: str = __file__) -> int:
    """Start n rank processes of `script argv` (one per GPU) with the
    torch.distributed env set before any of them touches a device; wait for
    all; return the worst exit status. This process never initialises the
    GPU (no exec either: the ranks are children)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return (abs(bad[0]) or 1) if bad else 0


# The profiled child runs the parent's --steps after at least PROFILE_WARMUP
# warm-up launches (the first launches on a cold box run ~20 % long while the
# clocks ramp: profiles/r4s per-dispatch trace 5.88 -> 4.77 ms over 9 launches);
# roofline.frac comes from its per-dispatch trace of the timed launches only.
PROFILE_WARMUP, PROFILE_SINGLE_REPS = 10, 9
# profiled kernel time allowed above the live kernel time before the line flags it
PROFILE_TOLERANCE = 1.03


def run_profile_child(args) -> dict:
    """rocprofv3 --kernel-trace --stats over this same bench (the program
    directly after --): a child process that runs max(--warmup, PROFILE_WARMUP)
    + --steps batch launches and the configs[2] single cube (1 + 2 x
    PROFILE_SINGLE_REPS calls) on the same box, before this process touches the
    GPU. Returns, per kernel, the per-dispatch durations of the timed window
    only (timed_dispatches: the batch's warm-up launches dropped), the stats
    summary of every launch under "stats" ({} with an "error" when the profiler
    is absent or fails) and both csv paths, so the line's roofline.frac comes
    from the profiled launches that correspond to the timed ones."""
    import csv
    import shutil
    import signal
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return {"error": "rocprofv3 not found"}
    out = os.path.abspath(args.profile_dir or os.path.join(ROOT, "gpurun_out", "bench_profile"))
    os.makedirs(out, exist_ok=True)
    warm = max(args.warmup, PROFILE_WARMUP)
    cmd = [prof, "--kernel-trace", "--stats", "-d", out, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--profile-child", "--steps", str(args.steps),
           "--warmup", str(warm), "--per-gpu", str(args.per_gpu), "--length", str(args.length),
           "--score-bits", str(args.score_bits), "--kernel", args.kernel, "--workload", args.workload]
    env = dict(os.environ, TMPDIR="/tmp")
    t0 = time.perf_counter()
    try:
        p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True, start_new_session=True)
        try:
            _, err = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.communicate()
            return {"error": "rocprofv3 child timed out (300 s)"}
        if p.returncode != 0:
            return {"error": f"rocprofv3 child rc={p.returncode}: {err.strip()[-300:]}"}
        stats = os.path.join(out, "run_kernel_stats.csv")
        with open(stats) as f:
            rows = list(csv.DictReader(f))
        trace = os.path.join(out, "run_kernel_trace.csv")
        with open(trace) as f:
            disp = list(csv.DictReader(f))
    except Exception as e:  # noqa: BLE001  (recorded: the line falls back to the live time)
        return {"error": str(e)[-300:]}
    rel = (lambda p: os.path.relpath(p, ROOT) if p.startswith(ROOT) else p)
    res = {"csv": rel(stats), "trace_csv": rel(trace),
           "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --profile-child "
                      f"--steps {args.steps} --warmup {warm}",
           "child_s": round(time.perf_counter() - t0, 1)}
    res.update(timed_dispatches(disp, warm, args.steps))
    for r in rows:  # the stats summary (every launch, warm-ups included)
        name = r["Name"]
        for key in ("pencil_kernel", "lap_kernel", "plane_step_kernel", "literal_kernel"):
            if f"tsa::{key}<" in name and key not in res.get("stats", {}):
                res.setdefault("stats", {})[key] = {
                    "name": name.split("(")[0], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                    "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    return res


def timed_dispatches(rows, warmup: int, steps: int) -> dict:
    """Per-dispatch durations (rocprofv3 --kernel-trace csv rows) of the
    profiled child's launches, by kernel, in dispatch order: the batch kernel's
    first `warmup` launches are dropped and the next `steps` kept -- exactly
    the window the parent times -- and the single-cube lap kernel's first
    launch (the untimed warm-up call) is dropped. Each kept kernel gets
    {name, calls, avg_ns, median_ns, min_ns, max_ns, dispatch_ids, window}."""
    import statistics
    out = {}
    by = {}
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = r["Kernel_Name"]
        for key in ("pencil_kernel", "lap_kernel", "plane_step_kernel", "literal_kernel"):
            if f"tsa::{key}<" in name:
                by.setdefault(key, []).append(
                    (int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), name))
    for i, (key, ds) in enumerate(by.items()):
        # the first kernel family in dispatch order is the batch's
        keep = ds[warmup:warmup + steps] if i == 0 else ds[1:]
        window = (f"launches {warmup + 1}..{warmup + len(keep)} of {len(ds)} (warm-ups dropped)" if i == 0
                  else f"launches 2..{len(ds)} (the untimed first call dropped)")
        if not keep:
            continue
        ns = [d for _, d, _ in keep]
        out[key] = {"name": keep[0][2].split("(")[0], "calls": len(ns), "avg_ns": float(statistics.mean(ns)),
                    "median_ns": float(statistics.median(ns)), "min_ns": float(min(ns)),
                    "max_ns": float(max(ns)), "dispatch_ids": [keep[0][0], keep[-1][0]], "window": window}
    return out


def profile_child_main(args) -> int:
    """The program rocprofv3 traces (run_profile_child): the batch hot path,
    warmup + steps launches, then the configs[2] single cube; no output line."""
    import torch
    torch.cuda.set_device(0)
    tsa = load_pkg()
    import tsa_amd.synth as synth  # noqa: E402
    L = args.length
    n = args.per_gpu if args.workload == "batch" else 1
    params = tsa.TsaParams.default(score_bits=args.score_bits)
    seqs, offs = synth.batch(0, n, L)
    hot = GpuBatch(tsa, torch.device("cuda", 0), seqs, offs - offs[0], n, L, params, args.kernel)
    for _ in range(args.warmup + args.steps):
        hot.step()
    hot.sync()
    args.no_extra_configs = True
    time_singles(args, tsa, synth, hot, torch.device("cuda", 0), L, params, reps=PROFILE_SINGLE_REPS)
    hot.sync()
    return 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 20 timed steps after 10 warm-ups (~0.15 s of GPU): the first
    # launches of a fresh process run 5-25 % slow while the clocks settle
    # (per-dispatch trace: 5.84, 5.26, 5.05, 4.85, 4.78 ms, then 4.6-4.7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["batch", "single"], default="batch")
    ap.add_argument("--kernel", choices=["auto", "plane", "pencil"], default="auto")
    ap.add_argument("--per-gpu", type=int, default=512)
    ap.add_argument("--length", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the single-cube timings other than configs[2]")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target wall time of the CPU-baseline sample")
    ap.add_argument("--check", type=int, default=16,
                    help="batch triples checked vs the oracle (both ends included); 0 = no parity leg")
    ap.add_argument("--score-bits", type=int, default=12,
                    help="12 = RTL wrap (default); 16/0 for cubes beyond the RTL envelope (1024^3)")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the rocprofv3 kernel-trace child (roofline.frac from the live time only)")
    ap.add_argument("--profile-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--profile-dir", default=None,
                    help="where the rocprofv3 child writes (default gpurun_out/bench_profile)")
    return ap.parse_args(argv)


class GpuBatch:
    """The hot path on this rank's GPU: tsa_score_batch_async over a batch
    resident in HBM, launched on torch's current stream."""

    def __init__(self, tsa, dev, seqs, offs, n, L, params, kernel):
        import torch
        self.torch, self.tsa = torch, tsa
        self.n, self.L, self.params, self.kernel = n, L, params, kernel
        self.d_seqs = torch.from_numpy(seqs).to(dev)
        self.d_offs = torch.from_numpy(offs).to(dev)
        self.d_scores = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        self.ws = tsa.workspace_size(max(n, 1), L, L, L, params, kernel)
        self.d_ws = torch.empty(max(self.ws, 16), dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.current_stream()
        self.ev = None

    def step(self):
        if self.n:
            self.tsa.score_batch_async(self.d_seqs.data_ptr(), self.d_offs.data_ptr(), self.n,
                                       self.L, self.L, self.L, self.d_scores.data_ptr(),
                                       self.d_ws.data_ptr(), self.ws, self.stream.cuda_stream,
                                       self.params, self.kernel)

    def sync(self):
        self.torch.cuda.synchronize()

    def mark(self):  # HIP events on the launch stream (torch events see only torch's stream)
        e = self.torch.cuda.Event(enable_timing=True)
        e.record(self.stream)
        return e

    @staticmethod
    def elapsed_ms(e0, e1):
        return e0.elapsed_time(e1)

    def scores(self):
        return self.d_scores[: self.n]


def fallback_counters(tsa) -> dict:
    """The library's fallback counters (tsa_fallback_count: lap hand-offs that
    timed out and were rescored without the lap schedule; tsa_check_fallback_count:
    triples the checked kernel could not certify, rescored in the literal
    arithmetic). Both count on the synchronous entry points; on the async path
    the same events read as TSA_SCORE_INVALID / _UNCERTIFIED scores, which the
    bench counts per timed call (invalid_reps)."""
    return {"lap_timeouts": tsa.fallback_count(), "uncertified": tsa.check_fallback_count()}


def counter_delta(c0: dict, c1: dict) -> dict:
    return {k: c1[k] - c0[k] for k in c0}


def run_rank(args, world: int, rank: int, local_rank: int, backend: str, make_batch,
             device=None, extras: bool = True, on_scores=None, prof=None):
    """One rank of the bench: shard, stage, warm up, time K steps between
    barriers, take the max over ranks, gather the scores (the one collective)
    and, on rank 0, return the JSON record. make_batch(tsa, dev, seqs, offs, n,
    L, params, kernel) builds the rank's scorer (GpuBatch on the box)."""
    import torch
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    elif backend == "nccl":
        torch.cuda.set_device(0)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())

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
    hot = make_batch(tsa, dev, seqs, offs, n, L, params, args.kernel)

    for _ in range(args.warmup):
        hot.step()
    hot.sync()
    warm_scores = hot.scores().clone() if args.warmup > 0 else None
    fb0 = fallback_counters(tsa)
    if world > 1:
        dist.barrier()
    hot.sync()
    t0 = time.perf_counter()
    ev0 = hot.mark()
    for _ in range(args.steps):
        hot.step()
    ev1 = hot.mark()
    hot.sync()
    if world > 1:
        dist.barrier()
    hot.sync()
    elapsed = time.perf_counter() - t0
    kernel_ms_per_step = hot.elapsed_ms(ev0, ev1) / args.steps
    # the timed launches ran the planned kernel: no fallback counted, and the
    # last step's scores equal the warm-up's (a timed-out hand-off would read
    # TSA_SCORE_INVALID on this async path)
    batch_fb = counter_delta(fb0, fallback_counters(tsa))
    sc = hot.scores()
    batch_fb["invalid_scores"] = int((sc <= tsa.SCORE_UNCERTIFIED).sum().item()) if sc.numel() else 0
    batch_fb["stable_vs_warmup"] = bool((sc == warm_scores).all().item()) if warm_scores is not None else None
    elapsed_max = shard.max_over_ranks(elapsed, dev)

    # what this rank saw: the collective's world (RCCL under "nccl") and the
    # devices visible to it, so an N-GPU line shows RCCL ran N ranks
    devices = {"backend": (backend if world > 1 else "none (single process)"),
               "dist_world_size": dist.get_world_size() if world > 1 else 1,
               "visible_devices": torch.cuda.device_count() if backend == "nccl" else 0,
               "device": str(dev)}
    if backend == "nccl":
        devices["device_name"] = torch.cuda.get_device_name(dev)

    cells_per_triple = L * L * L
    total_cells = n_total * cells_per_triple * args.steps
    gcups = total_cells / elapsed_max / 1e9
    ms_per_step = elapsed_max / args.steps * 1e3

    # ---- score gather (the one collective) ------------------------------------
    all_scores = shard.gather_scores(hot.scores(), n_total, world).cpu().numpy()

    rec = None
    if rank == 0:
        rec = report(args, tsa, synth, hot, dev, world, n_total, per_gpu, n, L, params, gcups,
                     ms_per_step, kernel_ms_per_step, all_scores, extras, prof)
        rec["config"]["devices"] = devices
        rec["config"]["split_devices"] = split_devices(args.gpus)
        rec["fallbacks"] = fallback_summary(batch_fb, rec.get("single_cube") or {})
        if on_scores is not None:  # test hook: the gathered scores, global order
            on_scores(rec, all_scores)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return rec


def report(args, tsa, synth, hot, dev, world, n_total, per_gpu, n, L, params, gcups, ms_per_step,
           kernel_ms_per_step, all_scores, extras, prof=None):
    prof = prof or {}
    kind = args.kernel
    if kind == "auto":  # AUTO = pencil whenever its factored arithmetic is exact
        kind = "pencil" if _pencil_ok(tsa, L, params) else "plane"
    kernel_name = {"plane": "plane_step_kernel", "pencil": "pencil_kernel"}[kind]
    launches_per_step = (3 * L - 1) if kind == "plane" else 1
    # kernel, arithmetic and schedule the library picks (host-only query)
    plan = tsa.describe_plan(max(per_gpu, 1), L, L, L, params, kernel=kind, sync=False)
    # exact integer values in f16 / int16 lanes; plane: int32 math on int16 planes
    arith = "f16" if " f16" in plan else ("i32" if plan.split()[:2] == ["plane", "est"] else "i16")

    per_gpu_cells = n * L * L * L
    kernel_s = kernel_ms_per_step * 1e-3
    algo_gbs = per_gpu_cells * BYTES_PER_CELL / kernel_s / 1e9
    pmc = load_pmc(kernel_name, args.workload) if (L == 256 and per_gpu == 512) else {}
    if pmc.get("stale"):
        log("PMC profile refused:", pmc["stale"])
    traffic = pmc.get("hbm_bytes_per_launch")
    insts = pmc.get("valu_insts_per_launch")
    hbm = {"bound": "hbm", "achieved": round(traffic / kernel_s / 1e9, 2) if traffic else None,
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(traffic / kernel_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
           "bytes_per_launch": traffic,
           "bytes_per_cell": round(traffic / per_gpu_cells, 3) if traffic else None,
           "source": "2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 --pmc, separate passes; gfx950 "
                     f"FETCH_SIZE correction), profiles/pmc_{kernel_name}_{args.workload}.json"}
    hbm_model = {"bound": "hbm", "bytes_per_cell": BYTES_PER_CELL, "achieved": round(algo_gbs, 2),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(algo_gbs / HBM_PEAK_GBS, 4),
                 "note": "SURVEY.md 8d: 7 int16 states written + read once per cell; the pencil "
                         "kernel keeps states in registers/LDS, so this model is not its ceiling"}
    kprof = prof.get(kernel_name)
    if insts and kind == "pencil":
        # the binding resource of the pencil kernel: VALU issue. frac: the
        # rocprofv3 average of this run's own profiled child (same box, same
        # command); frac_live: the live HIP-event time of the timed steps
        live = insts / kernel_s
        prof_s = kprof["avg_ns"] * 1e-9 if kprof else None
        ach = insts / prof_s if prof_s else live
        # the profiled launches must describe the timed ones: flag a profiled
        # mean more than PROFILE_TOLERANCE above the live kernel time
        prof_ratio = round(prof_s / kernel_s, 4) if prof_s else None
        roofline = {"bound": "valu", "achieved": round(ach / 1e9, 2),
                    "peak": VALU_WAVE_INSTR_PER_S / 1e9, "unit": "G wave-instr/s",
                    "frac": round(ach / VALU_WAVE_INSTR_PER_S, 4),
                    "frac_live": round(live / VALU_WAVE_INSTR_PER_S, 4),
                    "achieved_live": round(live / 1e9, 2), "traffic": traffic,
                    "peak_source": VALU_PEAK_SOURCE, "insts_per_launch": insts,
                    "lane_insts_per_cell": round(insts * 64 / per_gpu_cells, 3),
                    # the V-space pair core's 12 lane-ops per cell at the line's rate:
                    # how far the cells/s are from what the issue ceiling allows
                    "algorithmic": round(gcups / world * 1e9 * CORE_LANE_OPS_PER_CELL / 64
                                         / VALU_WAVE_INSTR_PER_S, 4),
                    "algorithmic_note": f"value/n_gpus x {CORE_LANE_OPS_PER_CELL} lane-ops per cell "
                                        "(cell_messages_vs pair core) / (64 x peak)",
                    "profiled_ms": round(prof_s * 1e3, 4) if prof_s else None,
                    "profiled_median_ms": round(kprof["median_ns"] * 1e-6, 4) if kprof else None,
                    "profiled_window": kprof.get("window") if kprof else None,
                    "profiled_over_live": prof_ratio,
                    "profile_consistent": (prof_ratio <= PROFILE_TOLERANCE) if prof_ratio else None,
                    "source": (f"SQ_INSTS_VALU per launch (profiles/pmc_{kernel_name}_{args.workload}.json)"
                               " / " + ("mean per-dispatch duration of the profiled child's timed window "
                                        "(rocprofv3 --kernel-trace, warm-ups dropped; profile.trace_csv)"
                                        if prof_s else "live kernel time (HIP events; no profile: "
                                        + str(prof.get("error", "skipped")) + ")"))}
        if prof_ratio and prof_ratio > PROFILE_TOLERANCE:
            log(f"roofline: profiled kernel {prof_s * 1e3:.4f} ms is {prof_ratio:.3f} x the live "
                f"{kernel_ms_per_step:.4f} ms (> {PROFILE_TOLERANCE}): flagged (profile_consistent false)")
    else:  # no current profile: the contract's HBM form on algorithmic bytes
        roofline = dict(hbm_model, traffic=traffic)
    roofline.update({"kernel": kernel_name, "kernel_ms_per_step": round(kernel_ms_per_step, 4),
                     "hbm": hbm, "hbm_model": hbm_model, "pmc_stale": pmc.get("stale"),
                     "profile": prof or None})

    # the single cubes' oracle scores (two 1024^3 among them, ~30 s each on
    # one core) run in threads while the GPU times the cubes
    pending = start_single_oracles(args, synth, L) if extras and args.check > 0 else None
    single = {}
    if extras:
        single = time_singles(args, tsa, synth, hot, dev, L, params)
        roofline["single_cube_lap"] = lap_roofline(args, L, single, prof)
    parity, cpu_baseline = None, None
    if extras and args.check > 0:
        parity, cpu_baseline = oracle_leg(args, tsa, synth, world, n_total, L, all_scores, single,
                                          pending)

    return {
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
            "workload": (f"batch: {per_gpu} independent {L}^3 triples per GPU -- the per-GPU shard "
                         f"of configs[4] (4096 x 256^3 over 8 GPUs); value = all ranks' cells / "
                         f"max-over-ranks time" if args.workload == "batch"
                         else f"single: one {L}^3 triple per GPU (configs[2])"),
            "config_index": 4 if args.workload == "batch" else 2,
            "length": L, "triples_per_gpu": per_gpu, "triples_total": n_total,
            "kernel": kind, "plan": plan, "launches_per_step": launches_per_step,
            "parallelism": f"shard{world}", "world_size": world, "score_bits": params.score_bits,
        },
        "roofline": roofline,
        "cpu_baseline": cpu_baseline,
        "single_cube": single,
        "parity": parity,
        "build": tsa.build_info(),
    }


def fallback_summary(batch_fb: dict, single: dict) -> dict:
    """Every fallback the timed work could have taken, in one place: the batch
    step's counter deltas and score checks, each single cube's, and all_zero
    (true when no counter moved and no timed call read an invalid score)."""
    singles = {k: v["fallbacks"] for k, v in single.items() if isinstance(v, dict) and "fallbacks" in v}
    vals = [batch_fb] + list(singles.values())
    zero = all(d.get("lap_timeouts", 0) == 0 and d.get("uncertified", 0) == 0
               and d.get("invalid_scores", d.get("invalid_reps", 0)) == 0 for d in vals)
    zero = zero and batch_fb.get("stable_vs_warmup") is not False
    return {"batch": batch_fb, "single_cube": singles, "all_zero": zero}


def lap_roofline(args, L, single, prof) -> dict | None:
    """VALU roofline of the single-cube lap kernel on configs[2] (one L^3
    cube): SQ_INSTS_VALU per launch from the stamped committed PMC profile
    (profiles/pmc_lap_kernel_single.json) over the profiled child's average
    (frac) and the live median (frac_live). The lap kernel is latency-bound
    (DESIGN.md 4.4): this says how much of the chip's issue it uses."""
    r = single.get(f"configs[2]: {L}^3", {})
    if "ms" not in r:
        return None
    pmc = load_pmc("lap_kernel", "single")
    insts = pmc.get("valu_insts_per_launch") if L == 256 else None
    kp = (prof or {}).get("lap_kernel")
    out = {"bound": "valu", "kernel": "lap_kernel", "cube": f"{L}^3", "plan": r.get("plan"),
           "peak": VALU_WAVE_INSTR_PER_S / 1e9, "unit": "G wave-instr/s", "ms_live": r["ms"],
           "insts_per_launch": insts, "pmc_stale": pmc.get("stale")}
    if insts:
        out["frac_live"] = round(insts / (r["ms"] * 1e-3) / VALU_WAVE_INSTR_PER_S, 4)
        if kp:
            out["profiled_avg_ms"] = round(kp["avg_ns"] * 1e-6, 4)
            out["frac"] = round(insts / (kp["avg_ns"] * 1e-9) / VALU_WAVE_INSTR_PER_S, 4)
    return out


def single_specs(args, L):
    """(key, length, score_bits, reps, kernel) of every single cube rank 0
    times: configs[2] (L^3, the batch's words), configs[1] (64^3), the
    paper's 128^3 and 512^3 (Table III, RTL 12-bit words) and configs[3]
    (1024^3 with 16-bit words, and with the RTL's 12-bit words on the checked
    kernel), and 512^3 / 1024^3 in the literal arithmetic (kernel=plane: the
    literal lap kernel)."""
    specs = [(f"configs[2]: {L}^3", L, args.score_bits, 7, None)]
    if not args.no_extra_configs:
        specs += [("configs[1]: 64^3", 64, args.score_bits, 15, None),
                  ("paper N=128: 128^3", 128, args.score_bits, 9, None),
                  ("paper N=512: 512^3", 512, args.score_bits, 5, None),
                  ("configs[3]: 1024^3 (16-bit words)", 1024, 16, 5, None),
                  # the score is exact, or TSA_SCORE_UNCERTIFIED (then rescored by PLANE)
                  ("configs[3]: 1024^3 (12-bit RTL words, checked)", 1024, 12, 5, "checked"),
                  # the RTL's literal wrapped arithmetic (TSA_KERNEL_PLANE: the literal lap)
                  ("paper N=512: 512^3 (literal arithmetic)", 512, 12, 5, "plane"),
                  ("configs[3]: 1024^3 (12-bit RTL words, literal arithmetic)", 1024, 12, 5, "plane")]
    return specs


DAT_KEY = "configs[0]: dat/{A,B,C}_seq.dat"
SPIN_OK = [True]  # torch.cuda._sleep usable as the single cubes' preload


def dat_triple():
    """The reference's dat/{A,B,C}_seq.dat triple, as committed numbers
    (tests/golden/golden.json case "dat", golden score 1)."""
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return next(c for c in json.load(f)["cases"] if c["name"] == "dat")


def time_singles(args, tsa, synth, hot, dev, L, params, reps=None):
    """Single-cube latency (single_specs, plus the dat triple): median of
    individually timed calls on the launch stream. Each cube is
    synth.triple(0, length)."""
    import torch
    stream = hot.stream

    def one(Ls, prm, nrep, kernel=None, trip=None):
        kernel = kernel or args.kernel
        sa = synth.batch(0, 1, Ls) if trip is None else tsa.pack_batch([trip])
        la, lb, lc = (int(sa[1][i + 1] - sa[1][i]) for i in range(3))
        s_seqs = torch.from_numpy(sa[0]).to(dev)
        s_offs = torch.from_numpy(sa[1]).to(dev)
        s_score = torch.zeros(1, dtype=torch.int32, device=dev)
        s_ws = tsa.workspace_size(1, la, lb, lc, prm, kernel)
        s_wsb = torch.empty(max(s_ws, 16), dtype=torch.uint8, device=dev)

        def sstep():
            tsa.score_batch_async(s_seqs.data_ptr(), s_offs.data_ptr(), 1, la, lb, lc,
                                  s_score.data_ptr(), s_wsb.data_ptr(), s_ws, stream.cuda_stream,
                                  prm, kernel)
        sstep()
        torch.cuda.synchronize()

        def spin():
            if SPIN_OK[0]:
                try:
                    torch.cuda._sleep(2_000_000)  # ~1 ms of clock spinning, no memory traffic
                    return
                except Exception:  # noqa: BLE001  (no such op on this build: the batch instead)
                    SPIN_OK[0] = False
            hot.step()

        rep_scores = []

        def timed(preload):
            # preload: a spin kernel queued first keeps the GPU busy while the
            # host submits e0, the cube's launch(es) and e1, so e0 -> e1 is the
            # device time of the call; without it the span also holds the
            # host's submission latency (the round-3 figure). The spin touches
            # no memory (a batch launch as the preload left dirty L2 lines that
            # slowed the cube after it)
            times = []
            for _ in range(reps or nrep):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if preload:
                    spin()
                e0.record(stream)
                sstep()
                e1.record(stream)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
                rep_scores.append(int(s_score.item()))  # every timed call's own score
            return float(np.median(times))
        fb0 = fallback_counters(tsa)
        sms = timed(preload=hot.n > 0)
        r = {"ms": round(sms, 4), "gcups": round(la * lb * lc / (sms * 1e-3) / 1e9, 3),
             "score": int(s_score.item()), "score_bits": prm.score_bits,
             "plan": tsa.describe_plan(1, la, lb, lc, prm, kernel=kernel, sync=False),
             "timing": "device: median of HIP events around the call's launches, queued behind a "
                       "spin kernel so host submission is hidden" if hot.n > 0 else "events, host submit included"}
        if hot.n > 0:
            r["ms_incl_submit"] = round(timed(preload=False), 4)
        # the timed calls ran the planned kernel: counters unmoved, no call
        # read TSA_SCORE_INVALID (a timed-out hand-off on this async path), and
        # every call scored the same
        fb = counter_delta(fb0, fallback_counters(tsa))
        bad = sum(1 for v in rep_scores if v == tsa.SCORE_INVALID or
                  (v == tsa.SCORE_UNCERTIFIED and kernel != "checked"))
        fb.update({"timed_calls": len(rep_scores), "invalid_reps": bad,
                   "uncertified_reps": sum(1 for v in rep_scores if v == tsa.SCORE_UNCERTIFIED),
                   "scores_agree": len(set(rep_scores)) <= 1})
        r["fallbacks"] = fb
        if Ls in ASIC_MS and prm.score_bits == 12 and trip is None:
            r["asic_ms"] = ASIC_MS[Ls]
            r["vs_asic"] = round(ASIC_MS[Ls] / sms, 3)
        if kernel == "checked":
            r["certified"] = r["score"] != tsa.SCORE_UNCERTIFIED
        return r

    out = {}
    for key, Ls, bits, nrep, kernel in single_specs(args, L):
        try:
            out[key] = one(Ls, tsa.TsaParams.default(score_bits=bits), nrep, kernel)
        except Exception as e:  # noqa: BLE001  (recorded; the parity leg counts it)
            log(f"single-cube {key} failed:", e)
            out[key] = {"error": str(e)[-300:], "score_bits": bits}
    if not args.no_extra_configs:
        dat = dat_triple()
        try:  # the testbench's own input on the device-resident path (AUTO kernel)
            out[DAT_KEY] = one(64, tsa.TsaParams.default(), 15, "auto", (dat["a"], dat["b"], dat["c"]))
        except Exception as e:  # noqa: BLE001
            log("dat triple failed:", e)
            out[DAT_KEY] = {"error": str(e)[-300:], "score_bits": 12}
        out["split over devices"] = time_split(world_devices=args.gpus)
    return out


def split_devices(world_devices: int) -> str:
    """Devices the split-over-devices leg lays one cube over: 2 parts sharing
    device 0 at N = 1, devices 0..N-1 on an N-GPU run."""
    return ",".join(str(d) for d in range(world_devices)) if world_devices > 1 else "0,0"


def time_split(world_devices: int) -> dict:
    """One cube split over devices by laps, in a child
    process with its own time limit: 2 parts sharing device 0 at N = 1,
    devices 0..N-1 on an N-GPU run (rank 0, while the other ranks wait)."""
    devs = split_devices(world_devices)
    cmd = [sys.executable, os.path.join(ROOT, "tools", "split_cube.py"), "--devices", devs,
           "--lengths", SPLIT_LENGTHS]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
        if r.returncode == 0 and r.stdout.strip():
            return json.loads(r.stdout.strip().splitlines()[-1])
        return {"devices": devs, "error": f"rc={r.returncode}: {r.stderr.strip()[-300:]}"}
    except Exception as e:  # noqa: BLE001
        return {"devices": devs, "error": str(e)[-300:]}


def _import_oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402
    return oracle


CPU_REPS_SMALL, CPU_REPS_LARGE = 5, 1  # oracle repetitions per single cube: <= 512^3 / 1024^3


def start_single_oracles(args, synth, L):
    """Oracle scores of every single cube bench times (and splits) and of the
    dat triple, keyed by (length, score_bits) / "dat", started in threads (the
    C oracle releases the GIL) that overlap the GPU timings. Each is also the
    software baseline of its config, as the reference's Table III "software"
    row (pic/Result.png): one core, the median of CPU_REPS_SMALL runs up to
    512^3 and one run at 1024^3. The threads are pinned one per core to the
    LAST cores of the job's affinity set and capped below the core count, so
    the launching thread keeps a core of its own (timed launches of small
    cubes are not inflated by them). Future -> (score, [seconds per run])."""
    from concurrent.futures import ThreadPoolExecutor
    import itertools
    import threading
    try:
        oracle = _import_oracle()
    except Exception as e:  # noqa: BLE001
        log("oracle unavailable:", e)
        return None
    want = sorted({(Ls, bits) for _, Ls, bits, _, _ in single_specs(args, L)}, key=lambda t: -t[0])
    if not args.no_extra_configs:  # the split child process times 256^3 (12-bit), 1024^3 (16- and 12-bit)
        want = sorted(set(want) | {(256, 12), (1024, 16), (1024, 12)}, key=lambda t: -t[0])
    try:
        allowed = sorted(os.sched_getaffinity(0))[: host_cores()]
    except AttributeError:
        allowed = list(range(host_cores()))
    nthr = max(1, min(len(want) + 1, len(allowed) - 2))
    cores = allowed[-nthr:]
    counter = itertools.count()

    def pin():
        try:
            os.sched_setaffinity(0, {cores[next(counter) % len(cores)]})  # this thread only (Linux)
        except (AttributeError, OSError):
            pass

    def run(a, b, c, prm, reps):
        times, score = [], None
        for _ in range(reps):
            t = oracle.now()
            score = oracle.score(a, b, c, prm)
            times.append(oracle.now() - t)
        return score, times

    pool = ThreadPoolExecutor(max_workers=nthr, initializer=pin)
    futs = {(Ls, bits): pool.submit(run, *synth.triple(0, Ls), oracle.default_params(score_bits=bits),
                                    CPU_REPS_LARGE if Ls > 512 else CPU_REPS_SMALL)
            for Ls, bits in want}
    if not args.no_extra_configs:
        dat = dat_triple()
        futs["dat"] = pool.submit(run, dat["a"], dat["b"], dat["c"], oracle.default_params(), CPU_REPS_SMALL)
    futs["_pinning"] = {"threads": nthr, "cores": cores, "of": len(allowed),
                        "main_thread": threading.current_thread().name}
    pool.shutdown(wait=False)
    return futs


def oracle_leg(args, tsa, synth, world, n_total, L, all_scores, single, pending):
    """Checker + CPU baseline (the only use of oracle/ here).

    parity: >= args.check gathered batch scores (both ends included), every
    single cube rank 0 timed and both split-cube scores against the C oracle
    on the same inputs, plus the reference's dat triple through tsa_score_gpu
    (golden score 1, tests/golden/golden.json). Each config is listed as
    {gpu, oracle, ok}; parity["mismatches"] counts every failure (an error or
    a missing score counts too) and main() exits non-zero when it is not 0.
    cpu_baseline: at N=1 the oracle timed on a bounded sample of the same
    workload on every host core the job may use."""
    parity, cpu_baseline = {"mismatches": 1, "error": "oracle leg did not run"}, None
    try:
        oracle = _import_oracle()
        cores = host_cores()
        configs = {}

        def put(name, gpu, ref):
            configs[name] = {"gpu": gpu, "oracle": ref, "ok": gpu is not None and gpu == ref}

        # batch: both ends + an even spread
        idx = sorted(set([0, n_total - 1] + [int(v) for v in np.linspace(0, n_total - 1, args.check)]))
        trip = [synth.triple(i, L) for i in idx]
        cs, co = tsa.pack_batch(trip)
        oparams = oracle.default_params(score_bits=args.score_bits)
        ref = oracle.score_batch(cs, co, oparams, nthreads=cores)
        got = all_scores[idx]
        bad = [int(i) for i, g, r in zip(idx, got, ref) if g != r]
        batch = {"checked": len(idx), "indices": [int(i) for i in idx], "mismatches": len(bad),
                 "mismatched_indices": bad, "score_bits": args.score_bits}
        # single cubes and the split (oracle scores started before the GPU timings);
        # each one's 1-core oracle time is the config's software baseline
        pin_info = pending.pop("_pinning", None) if pending else None
        done = {k: f.result() for k, f in pending.items()} if pending else {}
        refs = {k: v[0] for k, v in done.items()}
        cpu_ms = {k: round(float(np.median(v[1])) * 1e3, 3) for k, v in done.items()}

        def baseline(r, key):
            if key in cpu_ms and isinstance(r, dict):
                r["cpu_ms"] = cpu_ms[key]
                r["cpu_runs"] = len(done[key][1])
                if r.get("ms"):
                    r["speedup"] = round(cpu_ms[key] / r["ms"], 2)

        for key, Ls, bits, _, _ in single_specs(args, L):
            r = single.get(key, {})
            put(key, r.get("score"), refs.get((Ls, bits)))
            baseline(r, (Ls, bits))
        if DAT_KEY in single:
            put(DAT_KEY + " (device-resident path)", single[DAT_KEY].get("score"), refs.get("dat"))
            baseline(single[DAT_KEY], "dat")
        sp = single.get("split over devices")
        errors = {}
        if isinstance(sp, dict):
            lens = [k for k in sp if "^3" in k and isinstance(sp[k], dict)]
            devs = sp.get("devices")
            if isinstance(devs, str):  # the child failed before printing ("0,1")
                devs = [int(d) for d in devs.split(",") if d.strip().isdigit()]
            # across distinct GPUs (the driver's N-GPU run) the split is the one
            # path no 1-GPU box can exercise: an error there (no score) is
            # recorded under parity["errors"]; a wrong score still fails
            cross = isinstance(devs, list) and len(set(devs)) > 1
            if not lens:
                if cross:
                    errors["split over devices"] = sp.get("error", "no result")
                else:
                    put("split over devices", None, None)
            for k in lens:
                Ls = int(k.split("^3")[0])
                okey = (Ls, sp[k]["score_bits"])
                if okey in cpu_ms:
                    sp[k]["cpu_ms"] = cpu_ms[okey]
                for part in ("one_part", "split"):
                    r = sp[k].get(part, {})
                    name = f"split over devices {devs}: {k} {part}"
                    # only a setup failure of the cross-device split (no peer
                    # access, no such device: TSA_EDEVICE / TSA_ENODEV) is
                    # non-failing; repetitions that disagree, a timed-out hand-off
                    # or a wrong score fail the parity leg
                    if (cross and part == "split" and r.get("score") is None and not r.get("disagree")
                            and r.get("rc") in (-3, -4)):
                        errors[name] = r.get("error", "no score")
                        continue
                    put(name, r.get("score"), refs.get(okey))
                    if r.get("disagree"):
                        configs[name]["ok"] = False
                        configs[name]["disagree"] = r.get("scores")
        # the reference's own parity input: dat/{A,B,C}_seq.dat through tsa_score_gpu
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            dat = next(c for c in json.load(f)["cases"] if c["name"] == "dat")
        try:
            g_dat = tsa.score(dat["a"], dat["b"], dat["c"], device=0)
        except Exception as e:  # noqa: BLE001
            log("dat triple failed:", e)
            g_dat = None
        put("configs[0]: dat/{A,B,C}_seq.dat (tsa_score_gpu)", g_dat,
            oracle.score(dat["a"], dat["b"], dat["c"]))
        configs["configs[0]: dat/{A,B,C}_seq.dat (tsa_score_gpu)"]["golden"] = dat["score"]
        if dat["score"] != configs["configs[0]: dat/{A,B,C}_seq.dat (tsa_score_gpu)"]["oracle"]:
            configs["configs[0]: dat/{A,B,C}_seq.dat (tsa_score_gpu)"]["ok"] = False
        n_bad = len(bad) + sum(not c["ok"] for c in configs.values())
        parity = {"mismatches": n_bad, "batch": batch, "configs": configs,
                  "against": "oracle/tsa_oracle.c (literal RTL form, same inputs)"}
        if pin_info:
            parity["oracle_threads"] = dict(pin_info, overlapped="the single-cube GPU timings")
        if errors:
            parity["errors"] = errors
        if world == 1 and not args.no_cpu_baseline:
            # bounded sample of the same workload: one L^3 triple per thread per round
            t_one = oracle.now()
            oracle.score_batch(cs[: 3 * L], co[:4], oparams, nthreads=1)
            t_one = oracle.now() - t_one
            rounds = max(1, int(args.cpu_seconds / max(t_one, 1e-3)))
            ns = cores * rounds
            bs, bo = synth.batch(0, ns, L)
            t = oracle.now()
            oracle.score_batch(bs, bo, oparams, nthreads=cores)
            t = oracle.now() - t
            cpu_baseline = {
                "value": round(ns * L ** 3 / t / 1e9, 5), "unit": "GCUPS",
                "cores": cores, "kind": "port",
                "sample": f"{ns} synthetic {L}^3 triples (same generator) on {cores} threads "
                          f"(all host cores this job may use: affinity mask / cgroup quota; "
                          f"os.cpu_count()={os.cpu_count()}), {t:.1f} s wall; 1-thread rate "
                          f"{L ** 3 / t_one / 1e9:.4f} GCUPS; oracle/tsa_oracle.c literal RTL "
                          f"form, gcc -O2",
            }
    except Exception as e:  # noqa: BLE001
        log("oracle leg failed:", e)
        parity = {"mismatches": 1, "error": str(e)[-300:]}
    return parity, cpu_baseline


def _pencil_ok(tsa, L, params):
    try:
        tsa.workspace_size(1, L, L, L, params, "pencil")
        return True
    except tsa.TsaError:
        return False


def main(argv=None):
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # started directly: become the launcher of args.gpus rank processes
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv)))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.profile_child:
        sys.exit(profile_child_main(args))
    prof = None
    if world == 1 and not args.no_profile:
        # before this process touches the GPU: the same workload under
        # rocprofv3 on this box, for the line's profiled roofline
        prof = run_profile_child(args)
        if prof.get("error"):
            log("profile child:", prof["error"])
    rec = run_rank(args, world, rank, local_rank, "nccl", GpuBatch, prof=prof)
    if rec is not None:
        print(json.dumps(rec), flush=True)
        par = rec.get("parity")
        if par is not None and par.get("mismatches", 0) != 0:
            log(f"bench.py: {par['mismatches']} parity failure(s) against the oracle")
            sys.exit(3)


if __name__ == "__main__":
    main()
