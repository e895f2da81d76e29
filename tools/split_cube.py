"""Time one cube split over devices by laps (tsa_score_gpu_multi, SURVEY.md
8(f)2) against the same cube as one part, and print one JSON object.

bench.py runs this as a child process (a fault here cannot take the bench
line down): on one GPU the parts share device 0 (concurrently, on streams of
their own, when all their workgroups fit at once -- the 256^3 case; else one
after another on one stream, as 1024^3: the hand-off protocol without the
xGMI hop); under the driver's
N-GPU run rank 0 passes devices 0..N-1 (the real multi-GPU split). A case
that fails records {"error": ...} in place of its score.

    python tools/split_cube.py --devices 0,1 --lengths 256,1024 --reps 5
"""
import argparse
import importlib.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "hw-accelerator-three-sequence-alignment_amd")


def load_pkg():
    spec = importlib.util.spec_from_file_location(
        "tsa_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["tsa_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0,0")
    # "1024r": 1024^3 with the RTL's 12-bit words -- beyond the factored form's
    # a-priori bound, so the split runs the literal arithmetic
    ap.add_argument("--lengths", default="256,1024,1024r")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args(argv)
    tsa = load_pkg()
    import tsa_amd.synth as synth  # noqa: E402
    devs = [int(d) for d in args.devices.split(",")]
    out = {"devices": devs, "timing": "host wall: first launch .. last part synchronised, median"}
    for spec in args.lengths.split(","):
        L, rtl = int(spec.rstrip("r")), spec.endswith("r")
        # 16-bit words beyond the RTL's envelope (as bench's configs[3] line)
        prm = tsa.TsaParams.default(score_bits=12 if (L <= 512 or rtl) else 16)
        a, b, c = synth.triple(0, L)
        rec = {"score_bits": prm.score_bits}
        for label, dl in (("one_part", devs[:1]), ("split", devs)):
            walls, scores = [], set()
            try:
                for _ in range(args.reps + 1):
                    s, w = tsa.score_multi(a, b, c, dl, prm)
                    scores.add(s)
                    walls.append(w)
            except Exception as e:  # noqa: BLE001  (recorded: no score, bench counts it)
                # rc: TSA_EDEVICE / TSA_ENODEV are setup failures (peer access, no
                # such device); anything else is a failure of the split itself
                rec[label] = {"parts": len(dl), "error": str(e)[-300:], "rc": getattr(e, "rc", None)}
                continue
            # every repetition must agree: a differing one is flagged "disagree",
            # which bench.py's parity leg always counts as a failure
            rec[label] = {"parts": len(dl), "us": round(float(np.median(walls[1:])), 1),
                          "score": scores.pop() if len(scores) == 1 else None}
            if rec[label]["score"] is None:
                rec[label]["disagree"] = True
                rec[label]["scores"] = sorted(scores)
                rec[label]["error"] = f"repetitions disagree: {sorted(scores)}"
        rec["same_score"] = rec["one_part"].get("score") == rec["split"].get("score") is not None
        out[f"{L}^3" + (" (12-bit RTL words, literal)" if rtl else "")] = rec
    print(json.dumps(out))


if __name__ == "__main__":
    main()
