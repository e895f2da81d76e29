"""C-ABI library checks that need no GPU: it loads, exports exactly what
include/trialign.h declares, and its host-only entry points behave."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT


def header_functions():
    with open(os.path.join(ROOT, "include", "trialign.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tsa_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_entry_points(tsa):
    assert set(header_functions()) == set(tsa.EXPORTS)


def test_library_exports_every_header_symbol(tsa):
    lib = os.path.join(PKG_DIR, "lib", "libtrialign.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\sT\s(tsa_[a-z0-9_]+)", out))
    for fn in header_functions():
        assert fn in exported, fn
        assert hasattr(tsa.lib(), fn)


def test_library_does_not_link_the_oracle():
    lib = os.path.join(PKG_DIR, "lib", "libtrialign.so")
    out = subprocess.run(["nm", "-D", lib], capture_output=True, text=True, check=True).stdout
    assert "tsao_" not in out
    deps = subprocess.run(["ldd", lib], capture_output=True, text=True).stdout
    assert "tsa_oracle" not in deps


def test_default_params_are_rtl_localparams(tsa):
    p = tsa.TsaParams()
    tsa.lib().tsa_default_params(ctypes.byref(p))
    assert p.as_tuple() == (1, -1, 2, 1, tsa.S3_RTL, 12)
    assert tsa.TsaParams.default().as_tuple() == p.as_tuple()


def test_strerror_and_version(tsa):
    for rc in (0, -1, -2, -3, -4, -5, -6, -99):
        assert isinstance(tsa.lib().tsa_strerror(rc), bytes)
    assert tsa.version().startswith("trialign-mi355x gfx950")


def test_validate(tsa):
    ok = [0, 1, 2, 3, 4]
    assert tsa.validate(ok, ok, ok) == tsa.TSA_OK
    assert tsa.validate([5], ok, ok) == tsa.TSA_EINVAL          # symbol > 4
    assert tsa.validate([], ok, ok) == tsa.TSA_EINVAL           # empty
    assert tsa.validate(ok, ok, ok, tsa.TsaParams.default(s3_mode=7)) == tsa.TSA_EINVAL
    assert tsa.validate(ok, ok, ok, tsa.TsaParams.default(score_bits=17)) == tsa.TSA_EINVAL
    assert tsa.validate(ok, ok, ok, tsa.TsaParams.default(score_bits=3)) == tsa.TSA_EINVAL
    assert tsa.validate(ok, ok, ok, tsa.TsaParams.default(score_bits=0)) == tsa.TSA_OK
    # unbounded arithmetic whose value range cannot fit int16 state storage
    big = tsa.TsaParams.default(match=4000, score_bits=0)
    assert tsa.validate([0] * 20, [0] * 20, [0] * 20, big) == tsa.TSA_ERANGE


def test_workspace_size(tsa, monkeypatch):
    p = tsa.TsaParams.default()
    # the literal helix: one ring of (P + 8) records x M x 64 lanes x 16 B per triple
    monkeypatch.setenv("TSA_PENCIL_MODE", "literal")
    lit = tsa.workspace_size(4, 64, 64, 64, p, "plane")
    assert lit == 4 * (128 + 8) * 64 * 16
    # the literal lap (what the cost model picks for a few small cubes): O(N^2)
    monkeypatch.delenv("TSA_PENCIL_MODE")
    assert tsa.describe_plan(4, 64, 64, 64, p, kernel="plane").startswith("plane literal-lap")
    ll = tsa.workspace_size(1, 256, 256, 256, p, "plane")
    assert tsa.describe_plan(1, 512, 512, 512, p, kernel="plane").startswith("plane literal-lap")
    assert 1.5 < tsa.workspace_size(1, 512, 512, 512, p, "plane") / ll < 12  # 512^3: two per CU
    monkeypatch.setenv("TSA_PENCIL_MODE", "plane")  # the plane sweep itself
    n1 = tsa.workspace_size(1, 64, 64, 64, p, "plane")
    n4 = tsa.workspace_size(4, 64, 64, 64, p, "plane")
    assert n4 == 4 * n1 and n1 >= 4 * 7 * 65 * 65 * 2
    # O(N^2) memory: doubling N roughly quadruples the plane ring
    n2 = tsa.workspace_size(1, 128, 128, 128, p, "plane")
    assert 3.5 < n2 / n1 < 4.5
    with pytest.raises(tsa.TsaError):
        tsa.workspace_size(1, 0, 64, 64, p)


def test_describe_plan(tsa):
    # host-only plan query: the bench workload, the single-cube configs, the
    # streaming lap window of the sync path, and parameter sets the pencil
    # arithmetic does not cover
    p = tsa.TsaParams.default()
    assert tsa.describe_plan(512, 256, 256, 256, p).startswith("pencil helix f16v rtl M=2 NW=8")
    # V-space needs lam = GE = -MISMATCH and the shifted values inside exact f16
    assert tsa.describe_plan(512, 256, 256, 256, tsa.TsaParams.default(gap_extend=2, gap_open=3)
                             ).startswith("pencil helix f16 rtl")
    assert tsa.describe_plan(512, 400, 400, 400, p).startswith("pencil helix f16 rtl M=4")
    # a single cube: the lap kernel (its V-space cell only on request, TSA_LAP_VS=1)
    assert tsa.describe_plan(1, 256, 256, 256, p).startswith("pencil lap f16 rtl M=1")
    import os
    os.environ["TSA_LAP_VS"] = "1"
    try:
        assert tsa.describe_plan(1, 256, 256, 256, p).startswith("pencil lap f16v rtl M=1")
        assert tsa.describe_plan(1, 512, 512, 512, p).startswith("pencil lap f16 rtl M=1")  # beyond exact f16
    finally:
        del os.environ["TSA_LAP_VS"]
    # a few cubes: the lap kernel; many: the helix; a batch beyond the lap
    # grid's dispatch-round rules runs as chunks of triples, one launch each
    assert tsa.describe_plan(4, 256, 256, 256, p, sync=False).startswith("pencil lap f16")
    assert tsa.describe_plan(128, 256, 256, 256, p, sync=False).startswith("pencil helix")
    assert tsa.describe_plan(8, 512, 512, 512, p, sync=False).startswith("pencil lap f16")
    # many large cubes: chunked lap launches (each chunk's rounds looped by its
    # resident workgroups) where the cost model puts them ahead of the helix
    big = tsa.describe_plan(64, 1024, 1024, 1024, tsa.TsaParams.default(score_bits=16))
    assert big.startswith("pencil helix") or (big.startswith("pencil lap") and " chunk=" in big), big
    import os
    os.environ["TSA_PENCIL_MODE"] = "lap"
    try:
        for sync in (True, False):
            plan = tsa.describe_plan(100, 129, 128, 128, p, sync=sync)
            assert plan.startswith("pencil lap") and " chunk=" in plan, plan
        os.environ["TSA_LAP_CHUNK"] = "7"
        assert " chunk=7 " in tsa.describe_plan(100, 129, 128, 128, p, sync=False)
    finally:
        del os.environ["TSA_PENCIL_MODE"]
        os.environ.pop("TSA_LAP_CHUNK", None)
    # M = 2 lap periods are multiples of 4: even (the x = 1 register is then
    # PH ^ (w & 1)), and each wave's lap-wrap events fall on one static step of
    # the four-step group (TSA_EV_STATIC)
    assert "M=2 NW=8 P=260" in tsa.describe_plan(512, 257, 40, 255, p)
    assert "M=2 NW=8 P=256" in tsa.describe_plan(512, 255, 40, 255, p)
    p16 = tsa.TsaParams.default(score_bits=16)
    assert tsa.describe_plan(1, 1024, 1024, 1024, p16).startswith("pencil lap i16 rtl")
    sop = tsa.TsaParams.default(s3_mode=tsa.S3_SOP)
    assert " sop " in tsa.describe_plan(512, 256, 256, 256, sop)
    # the literal kernels by their cost model: the literal lap for a few cubes
    # (lap_kernel LIT), the literal helix for batches, the plane sweep where
    # neither runs (many cubes with LC > 512)
    assert tsa.describe_plan(4, 64, 64, 64, p, kernel="plane").startswith("plane literal-lap M=1")
    assert tsa.describe_plan(512, 256, 256, 256, p, kernel="plane").startswith("plane literal-helix")
    assert tsa.describe_plan(1, 256, 256, 256, p, kernel="plane").startswith("plane literal-lap")
    assert tsa.describe_plan(1, 1024, 1024, 1024, p, kernel="plane").startswith("plane literal-lap M=")
    assert tsa.describe_plan(64, 1024, 1024, 1024, p, kernel="plane").startswith("plane literal-lap")
    assert tsa.describe_plan(4096, 1024, 1024, 1024, p, kernel="plane").startswith("plane literal-lap")
    # without the lap schedule (the helix / sweep rescue of a timed-out lap)
    os.environ["TSA_PENCIL_MODE"] = "literal"
    try:
        assert tsa.describe_plan(4, 64, 64, 64, p, kernel="plane").startswith("plane literal-helix")
    finally:
        del os.environ["TSA_PENCIL_MODE"]
    # gap_extend > gap_open: the widened message groups are not exact -> literal
    ge = tsa.TsaParams.default(gap_open=1, gap_extend=2)
    assert tsa.describe_plan(4, 64, 64, 64, ge).startswith("plane literal-lap")
    assert tsa.describe_plan(512, 64, 64, 64, ge).startswith("plane literal-")
    with pytest.raises(tsa.TsaError) as e:
        tsa.describe_plan(4, 64, 64, 64, ge, kernel="pencil")
    assert e.value.rc == tsa.TSA_ERANGE
    # parameter sets that may wrap: the literal plane kernel on the async path;
    # the synchronous path tries the checked lap kernel first (PLANE rescoring
    # whatever it cannot certify), and so does an explicit kernel="checked"
    p6 = tsa.TsaParams.default(score_bits=6)
    assert tsa.describe_plan(4, 90, 90, 90, p6, sync=False).startswith("plane literal-lap")
    assert tsa.describe_plan(4, 90, 90, 90, p6, sync=True).split(" est=")[0].endswith(" checked")
    assert tsa.describe_plan(1, 1024, 1024, 1024, p, sync=True).startswith("pencil lap i16 rtl")
    assert tsa.describe_plan(1, 1024, 1024, 1024, p, sync=False).startswith("plane literal-lap M=")
    assert tsa.describe_plan(1, 1024, 1024, 1024, p, kernel="checked", sync=False).split(" est=")[0].endswith(" checked")
    # a large batch is checked in chunks of the lap schedule
    plan = tsa.describe_plan(4096, 800, 800, 800, p, sync=True)
    assert plan.startswith("pencil lap i16") and " chunk=" in plan and " checked" in plan, plan


def test_lap_planner_measured_choices(tsa):
    """The lap planner picks the geometries the round-4 sweeps measured fastest
    (profiles/r4m_lapgeo.jsonl, r4t_literal_geo.jsonl,
    r4u_lap_nw.jsonl, r4j_lapab.jsonl). Host-only (the CPU residency model)."""
    p12 = tsa.TsaParams.default()
    p16 = tsa.TsaParams.default(score_bits=16)

    def geo(plan):
        return re.search(r"M=(\d) NW=(\d)", plan).groups()

    want = [
        ((1, 768, p16, "pencil"), ("1", "8")),    # 1.90 ms vs M = 2 2.12
        ((1, 1024, p16, "pencil"), ("2", "8")),   # 2.98 ms vs M = 1 3.08
        ((8, 512, p12, "pencil"), ("2", "8")),    # 2.20 ms vs M = 1 2.69
        ((16, 256, p12, "pencil"), ("2", "8")),   # 0.745 ms vs M = 1 0.847
        ((1, 256, p12, "pencil"), ("1", "4")),
        ((1, 1024, p12, "plane"), ("1", "8")),    # literal: 4.10 ms vs M = 2 4.37
        ((1, 512, p12, "plane"), ("1", "4")),     # literal: 1.046 ms vs NW = 8 1.132
    ]
    for (n, L, p, k), mw in want:
        plan = tsa.describe_plan(n, L, L, L, p, kernel=k, sync=False)
        assert "lap" in plan and geo(plan) == mw, (n, L, k, plan)


def test_lap_rounds_and_ring_memory(tsa):
    """A 1024^3 cube does not fit one round of resident lap workgroups, so it
    runs two rounds -- each workgroup looping over its slot's laps -- with
    boundary rings; the O(N^2) workspace stays within 300 MB (round 2: 580
    MB). Host-only."""
    p16 = tsa.TsaParams.default(score_bits=16)
    plan = tsa.describe_plan(1, 1024, 1024, 1024, p16, sync=False)
    assert plan.startswith("pencil lap i16 rtl M=") and "waves=2" in plan, plan
    assert tsa.workspace_size(1, 1024, 1024, 1024, p16, "pencil") <= 300e6  # M = 1: 1024 workgroups
    # within one round: slim rings only (no boundary ring memory)
    p = tsa.TsaParams.default()
    assert "waves=1" in tsa.describe_plan(1, 512, 512, 512, p, sync=False)
    assert tsa.workspace_size(1, 512, 512, 512, p, "pencil") <= 100e6
    # O(N^2): 256^3 -> 512^3 grows ~4x, x2 more where 512^3 runs two NW = 4
    # workgroups per CU (their slim rings take 96 slots of slack, not 32)
    w256 = tsa.workspace_size(1, 256, 256, 256, p, "pencil")
    assert tsa.workspace_size(1, 512, 512, 512, p, "pencil") / w256 < 9


@pytest.mark.skipif(os.environ.get("TSA_EXPECT_GPU") == "1", reason="GPU box")
def test_no_cpu_fallback_without_gpu(tsa):
    if tsa.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(tsa.TsaError) as e:
        tsa.score([0, 1], [0, 1], [0, 1])
    assert e.value.rc == tsa.TSA_ENODEV
    with pytest.raises(tsa.TsaError) as e:
        tsa.score_batch([([0], [1], [2])])
    assert e.value.rc == tsa.TSA_ENODEV
    with pytest.raises(tsa.TsaError) as e:
        tsa.score_multi([0] * 64, [0] * 64, [0] * 64, [0, 1])
    assert e.value.rc == tsa.TSA_ENODEV
    with pytest.raises(tsa.TsaError) as e:
        tsa.score_batch_devices([([0], [1], [2])], (0, 0))
    assert e.value.rc == tsa.TSA_ENODEV
    # an empty batch is not an error, with or without a device
    assert len(tsa.score_batch_devices([], (0,))) == 0


def test_batch_devices_argument_checks(tsa):
    """tsa_score_batch_devices validates before touching a device: an empty
    device list, a bad symbol or bad offsets are TSA_EINVAL on any host."""
    for devs, trip in [((), [([0], [1], [2])]), ((0, 0), [([0, 9], [1], [2])])]:
        with pytest.raises(tsa.TsaError) as e:
            tsa.score_batch_devices(trip, devs)
        assert e.value.rc == tsa.TSA_EINVAL, devs
    seqs = np.zeros(6, np.uint8)
    with pytest.raises(tsa.TsaError) as e:  # offsets not monotone
        tsa.score_batch_devices(devices=(0,), seqs=seqs, offsets=np.array([0, 3, 2, 6], np.int64))
    assert e.value.rc == tsa.TSA_EINVAL


def test_cli_reports_no_device_or_score():
    cli = os.path.join(PKG_DIR, "bin", "tsa")
    dat = "/root/reference/dat"
    if not os.path.isdir(dat):
        pytest.skip("reference not mounted")
    r = subprocess.run([cli, f"{dat}/A_seq.dat", f"{dat}/B_seq.dat", f"{dat}/C_seq.dat"],
                       capture_output=True, text=True)
    if r.returncode == 0:
        assert "TriAlign Score:" in r.stdout and r.stdout.split()[-1] == "1"
    else:
        assert "no HIP device" in r.stderr


def test_align_argument_checks(tsa):
    # tsa_align_gpu validates before touching a device: a moves buffer shorter
    # than la+lb+lc, null outputs and bad symbols are TSA_EINVAL everywhere
    import ctypes
    a = np.zeros(4, np.uint8)
    p = tsa.TsaParams.default()
    mv = np.zeros(16, np.uint8)
    sc, n = ctypes.c_int32(0), ctypes.c_int32(0)
    st = (ctypes.c_int32 * 3)()
    u8 = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    lib = tsa.lib()
    assert lib.tsa_align_gpu(u8(a), 4, u8(a), 4, u8(a), 4, ctypes.byref(p), ctypes.byref(sc),
                             u8(mv), 11, ctypes.byref(n), st, 0) == tsa.TSA_EINVAL
    assert lib.tsa_align_gpu(u8(a), 4, u8(a), 4, u8(a), 4, ctypes.byref(p), None,
                             u8(mv), 16, ctypes.byref(n), st, 0) == tsa.TSA_EINVAL
    bad = np.array([0, 9, 1, 2], np.uint8)
    assert lib.tsa_align_gpu(u8(bad), 4, u8(a), 4, u8(a), 4, ctypes.byref(p), ctypes.byref(sc),
                             u8(mv), 16, ctypes.byref(n), st, 0) == tsa.TSA_EINVAL
    # traceback helpers are host-only
    assert tsa.path_score([0] * 4, [0] * 4, [0] * 4, (0, 0, 0), [0] * 4) == 12
    assert tsa.render_alignment("ACGT", "AGT", "ACT", (0, 0, 0), [0, 6, 4, 0]) == ("ACGT", "A-GT", "AC-T")


def test_split_cube_argument_checks(tsa):
    """tsa_score_gpu_multi validates before touching a device: an empty device
    list or a bad symbol is TSA_EINVAL on any host."""
    with pytest.raises(tsa.TsaError) as e:
        tsa.score_multi([0] * 8, [0] * 8, [0] * 8, [])
    assert e.value.rc == tsa.TSA_EINVAL
    with pytest.raises(tsa.TsaError) as e:
        tsa.score_multi([0, 7], [0] * 8, [0] * 8, [0, 0])
    assert e.value.rc == tsa.TSA_EINVAL
