"""bench.py's parity leg (oracle_leg) on the CPU: the per-config {gpu, oracle,
ok} records, and how the split-over-devices leg counts. GPU scores are stood in
by the oracle's own (this checks the bookkeeping, not a kernel)."""
import os
import sys
from argparse import Namespace
from concurrent.futures import Future

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _done(v):
    f = Future()
    f.set_result(v)
    return f


def _leg(tsa, orc, synth, split):
    import bench
    L, n = 16, 6
    ref = {i: orc.score(*synth.triple(i, L), orc.default_params(score_bits=12)) for i in range(n)}

    class GpuStandIn:
        pack_batch = staticmethod(tsa.pack_batch)

        @staticmethod
        def score(a, b, c, device=0):
            return orc.score(a, b, c)

    args = Namespace(check=3, score_bits=12, no_extra_configs=True, no_cpu_baseline=True, cpu_seconds=1)
    single = {f"configs[2]: {L}^3": {"score": ref[0]}, "split over devices": split}
    scores = np.array([ref[i] for i in range(n)], dtype=np.int32)
    pending = {(L, 12): _done((ref[0], [0.002, 0.001, 0.003])), "_pinning": {"threads": 1, "cores": [0]}}
    parity, _ = bench.oracle_leg(args, GpuStandIn, synth, 1, n, L, scores, single, pending)
    return parity, ref[0]


def test_parity_leg_counts_configs_and_split(tsa, orc, synth):
    ok = lambda s: {"parts": 1, "us": 1.0, "score": s}  # noqa: E731
    # one GPU: both split scores checked; an error there is a mismatch
    parity, s0 = _leg(tsa, orc, synth, {"devices": [0, 0], "16^3": {"score_bits": 12, "one_part": ok(None), "split": ok(None)}})
    assert parity["mismatches"] == 2 and "errors" not in parity
    parity, s0 = _leg(tsa, orc, synth, {"devices": [0, 0], "16^3": {"score_bits": 12, "one_part": ok(s0), "split": ok(s0)}})
    assert parity["mismatches"] == 0 and parity["batch"]["checked"] >= 3
    assert parity["configs"]["configs[0]: dat/{A,B,C}_seq.dat (tsa_score_gpu)"]["ok"]
    # distinct GPUs: a wrong split score fails, an error (no score) is recorded
    # under errors without failing the line
    parity, _ = _leg(tsa, orc, synth, {"devices": [0, 1], "16^3": {"score_bits": 12, "one_part": ok(s0), "split": ok(s0 + 1)}})
    assert parity["mismatches"] == 1
    parity, _ = _leg(tsa, orc, synth, {"devices": [0, 1], "16^3": {"score_bits": 12, "one_part": ok(s0),
                                                                  "split": {"parts": 2, "error": "peer access",
                                                                            "rc": -4}}})
    assert parity["mismatches"] == 0 and list(parity["errors"].values()) == ["peer access"]
    # ... but only a setup failure: a timed-out hand-off (TSA_EINTERNAL) fails
    parity, _ = _leg(tsa, orc, synth, {"devices": [0, 1], "16^3": {"score_bits": 12, "one_part": ok(s0),
                                                                  "split": {"parts": 2, "error": "timeout",
                                                                            "rc": -6}}})
    assert parity["mismatches"] == 1 and "errors" not in parity
    # repetitions that disagree always fail, on one GPU and across GPUs
    dis = {"parts": 2, "us": 1.0, "score": None, "disagree": True, "scores": [s0, s0 + 1],
           "error": "repetitions disagree"}
    for devs in ([0, 1], [0, 0]):
        parity, _ = _leg(tsa, orc, synth, {"devices": devs, "16^3": {"score_bits": 12, "one_part": ok(s0),
                                                                    "split": dis}})
        assert parity["mismatches"] == 1 and "errors" not in parity, devs
    parity, _ = _leg(tsa, orc, synth, {"devices": "0,1", "error": "rc=1: boom"})
    assert parity["mismatches"] == 0 and parity["errors"] == {"split over devices": "rc=1: boom"}
    parity, _ = _leg(tsa, orc, synth, {"devices": "0,0", "error": "rc=1: boom"})
    assert parity["mismatches"] == 1
    # a labelled length (the literal 12-bit case) is checked like the others
    parity, _ = _leg(tsa, orc, synth, {"devices": [0, 0], "16^3 (12-bit RTL words, literal)": {
        "score_bits": 12, "one_part": ok(s0), "split": ok(s0)}})
    assert parity["mismatches"] == 0 and len([k for k in parity["configs"] if "literal" in k]) == 2


def test_single_cube_software_baseline(tsa, orc, synth):
    """Every timed single cube carries the 1-core oracle time of the same
    input (median of its runs) and the speedup over it, as the reference's
    Table III "software" row does."""
    import bench
    L, n = 16, 4
    ref = orc.score(*synth.triple(0, L))
    single = {f"configs[2]: {L}^3": {"score": ref, "ms": 0.5}}
    args = Namespace(check=2, score_bits=12, no_extra_configs=True, no_cpu_baseline=True, cpu_seconds=1)
    pending = {(L, 12): _done((ref, [0.002, 0.004, 0.003]))}
    scores = np.array([orc.score(*synth.triple(i, L)) for i in range(n)], dtype=np.int32)

    class GpuStandIn:
        pack_batch = staticmethod(tsa.pack_batch)

        @staticmethod
        def score(a, b, c, device=0):
            return orc.score(a, b, c)

    parity, _ = bench.oracle_leg(args, GpuStandIn, synth, 1, n, L, scores, single, pending)
    assert parity["mismatches"] == 0
    r = single[f"configs[2]: {L}^3"]
    assert r["cpu_ms"] == 3.0 and r["speedup"] == 6.0 and r["cpu_runs"] == 3


def test_profile_window_is_the_timed_launches():
    """roofline.frac is computed from the profiled child's per-dispatch trace
    of the timed launches only: the batch kernel's
    warm-up launches and the single cube's untimed first call are dropped."""
    import bench
    rows = []
    did = 0

    def add(name, ns):
        nonlocal did
        did += 1
        rows.append({"Dispatch_Id": str(did), "Kernel_Name": name,
                     "Start_Timestamp": str(1000 * did), "End_Timestamp": str(1000 * did + ns)})
    add("__amd_rocclr_copyBuffer", 5)
    for ns in (900, 800, 700):  # cold warm-ups
        add("void tsa::pencil_kernel<2, 8, true, false, false, true>(unsigned char const*)", ns)
    for ns in (500, 510, 490, 500):
        add("void tsa::pencil_kernel<2, 8, true, false, false, true>(unsigned char const*)", ns)
    for ns in (99, 30, 31, 29):
        add("void tsa::lap_kernel<1, 4, true, false, false, false, false, false>(unsigned char const*)", ns)
    out = bench.timed_dispatches(list(reversed(rows)), warmup=3, steps=4)
    pk = out["pencil_kernel"]
    assert pk["calls"] == 4 and pk["avg_ns"] == 500.0 and pk["median_ns"] == 500.0
    assert pk["max_ns"] == 510.0 and pk["dispatch_ids"] == [5, 8]
    assert pk["name"] == "void tsa::pencil_kernel<2, 8, true, false, false, true>"
    lk = out["lap_kernel"]
    assert lk["calls"] == 3 and lk["avg_ns"] == 30.0 and lk["dispatch_ids"] == [10, 12]


def test_fallback_summary_flags_any_fallback():
    import bench
    clean = {"lap_timeouts": 0, "uncertified": 0, "invalid_scores": 0, "stable_vs_warmup": True}
    one = {"lap_timeouts": 0, "uncertified": 0, "timed_calls": 5, "invalid_reps": 0, "scores_agree": True}
    s = bench.fallback_summary(clean, {"a": {"fallbacks": one}, "b": {"error": "x"}})
    assert s["all_zero"] is True and list(s["single_cube"]) == ["a"]
    assert not bench.fallback_summary(clean, {"a": {"fallbacks": dict(one, invalid_reps=1)}})["all_zero"]
    assert not bench.fallback_summary(dict(clean, lap_timeouts=1), {})["all_zero"]
    assert not bench.fallback_summary(dict(clean, stable_vs_warmup=False), {})["all_zero"]
    assert bench.split_devices(1) == "0,0" and bench.split_devices(4) == "0,1,2,3"
