#!/usr/bin/env python3
"""Summarise a scripts/gpu_profile.sh run into profiles/ (tracked).

For each kernel directory under gpurun_out/prof_<tag>/<kernel>/ this reads the
rocprofv3 kernel trace (per-dispatch durations, grouped by grid size so the
batch launch and the single-cube launch are separated) and the two PMC passes
(FETCH_SIZE, WRITE_SIZE; separate runs as MI355X_MICROARCH.md prescribes), the
SQ_INSTS_VALU pass (wave-level VALU instructions per dispatch), and
writes
  profiles/<tag>_<kernel>_kernel_stats.csv   (rocprofv3 --stats summary, copied)
  profiles/pmc_<kernel_name>_batch.json      (read by bench.py: traffic field)
HBM bytes per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE counts
half the bytes of wide (16 B/lane) coalesced reads on gfx950 (the pencil ring
DMA is such a read); for the plane kernel's 2-byte gathers the x2 is an upper
bound (uncalibrated access width), so both raw and corrected values are kept.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_source_hash  # noqa: E402  (the stamp bench.py checks)


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(tag="r1"):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    outdir = os.path.join(ROOT, "profiles")
    os.makedirs(outdir, exist_ok=True)
    summary = {}
    for kdir in sorted(os.listdir(base)):
        d = os.path.join(base, kdir)
        stats = os.path.join(d, "trace", "run_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(outdir, f"{tag}_{kdir}_kernel_stats.csv"))
        trace = os.path.join(d, "trace", "run_kernel_trace.csv")
        per = defaultdict(list)
        names = {}
        for r in rows(trace):
            name = r["Kernel_Name"]
            if not name.startswith(("tsa::", "void tsa::")):
                continue
            grid = int(r["Grid_Size"]) if "Grid_Size" in r else \
                int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            key = (name.split("(")[0], grid)
            per[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            names[key] = name
        pmc = defaultdict(lambda: defaultdict(list))
        for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU"):
            p = os.path.join(d, f"pmc_{c}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            for r in rows(p):
                name = r["Kernel_Name"]
                if not name.startswith(("tsa::", "void tsa::")):
                    continue
                key = (name.split("(")[0], int(r["Grid_Size"]))
                pmc[key][c].append(float(r["Counter_Value"]))
        ks = {}
        for key, durs in per.items():
            kname, grid = key
            ent = {"kernel": kname, "grid_size": grid, "dispatches": len(durs),
                   "avg_ns": statistics.mean(durs), "median_ns": statistics.median(durs)}
            if key in pmc:
                fk = statistics.mean(pmc[key]["FETCH_SIZE"]) if pmc[key]["FETCH_SIZE"] else None
                wk = statistics.mean(pmc[key]["WRITE_SIZE"]) if pmc[key]["WRITE_SIZE"] else None
                ent["FETCH_SIZE_kB"] = fk
                ent["WRITE_SIZE_kB"] = wk
                if fk is not None and wk is not None:
                    ent["hbm_bytes_raw"] = (fk + wk) * 1024
                    ent["hbm_bytes_corrected"] = (2 * fk + wk) * 1024
                if pmc[key]["SQ_INSTS_VALU"]:
                    ent["valu_insts"] = statistics.mean(pmc[key]["SQ_INSTS_VALU"])
            ks[f"{kname}@{grid}"] = ent
        summary[kdir] = ks
        # bench.py's single-cube lap roofline: the lap launch of the profiled
        # child's configs[2] cube (one lap instantiation runs there)
        laps = [v for v in ks.values() if "lap_kernel" in v["kernel"] and v.get("valu_insts")]
        if laps:
            lp = max(laps, key=lambda v: v["dispatches"])
            with open(os.path.join(outdir, "pmc_lap_kernel_single.json"), "w") as f:
                json.dump({"tag": tag, "kernel": lp["kernel"], "grid_size": lp["grid_size"],
                           "avg_ns": lp["avg_ns"], "hbm_bytes_per_launch": lp.get("hbm_bytes_corrected"),
                           "valu_insts_per_launch": lp["valu_insts"],
                           "kernel_source_sha256": kernel_source_hash("lap_kernel"),
                           "workload": "bench.py --profile-child: configs[2], one 256^3 cube"}, f, indent=1)
        # bench.py traffic: the batch launch = the largest grid of the main kernel
        main_k = [v for v in ks.values() if ("pencil_kernel" in v["kernel"] or "plane_step_kernel" in v["kernel"])]
        if main_k:
            big = max(main_k, key=lambda v: v["grid_size"])
            if "hbm_bytes_corrected" in big:
                kn = "pencil_kernel" if "pencil" in big["kernel"] else "plane_step_kernel"
                # plane: one step = 3L-1 launches of varying size; report per-step total
                with open(os.path.join(outdir, f"pmc_{kn}_batch.json"), "w") as f:
                    json.dump({"tag": tag, "kernel": big["kernel"], "grid_size": big["grid_size"],
                               "avg_ns": big["avg_ns"], "hbm_bytes_per_launch": big["hbm_bytes_corrected"],
                               "hbm_bytes_raw": big["hbm_bytes_raw"],
                               "valu_insts_per_launch": big.get("valu_insts"),
                               "kernel_source_sha256": kernel_source_hash(kn),
                               "note": "(2*FETCH_SIZE+WRITE_SIZE)*1024, gfx950 FETCH_SIZE correction"},
                              f, indent=1)
    with open(os.path.join(outdir, f"{tag}_profile_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main(*sys.argv[1:])
