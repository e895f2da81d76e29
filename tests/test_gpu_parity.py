"""GPU parity: the HIP kernels through the C-ABI against the CPU oracle, the
committed golden fixtures and size-independent properties. Bit-exact (integer
work). Run on the MI355X box: pytest -m gpu."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KERNELS = ["plane", "pencil", "auto"]
# "plane" runs the literal helix where its cost model picks it (small cubes,
# batches); "plane-sweep" forces the PLANE sweep itself (TSA_PENCIL_MODE=plane)
LITERAL_KERNELS = ["plane", "plane-sweep", "pencil", "auto"]


def _select(kernel, monkeypatch):
    if kernel == "plane-sweep":
        monkeypatch.setenv("TSA_PENCIL_MODE", "plane")
        return "plane"
    return kernel


def _kernel_applies(tsa, kernel, la, lb, lc, p):
    """PENCIL is selectable only where its factored int16 arithmetic is exact
    and the shape fits (LC <= 256, LA/LB <= 4096); the API then returns
    TSA_ERANGE, which these tests treat as 'not applicable'."""
    if kernel != "pencil":
        return True
    try:
        tsa.workspace_size(1, la, lb, lc, p, "pencil")
        return True
    except tsa.TsaError:
        return False


@pytest.mark.parametrize("kernel", LITERAL_KERNELS)
def test_golden_fixtures(gpu, golden, kernel, monkeypatch):
    kernel = _select(kernel, monkeypatch)
    used = 0
    for c in golden:
        p = gpu.TsaParams.default(**c["params"])
        if not _kernel_applies(gpu, kernel, len(c["a"]), len(c["b"]), len(c["c"]), p):
            continue
        used += 1
        assert gpu.score(c["a"], c["b"], c["c"], p, kernel=kernel) == c["score"], c["name"]
    assert used >= 40


def test_golden_final_states(gpu, golden):
    for c in golden:
        p = gpu.TsaParams.default(**c["params"])
        s, fin = gpu.score(c["a"], c["b"], c["c"], p, final_states=True)
        assert s == c["score"] and list(fin) == c["final7"], c["name"]


def test_testbench_input_and_dat_cli(gpu, golden):
    z = [0] * 64
    assert gpu.score(z, z, z) == 192                       # src/TriAlign_tb.sv:423-1960
    by = {c["name"]: c for c in golden}
    t = gpu.TriAlign()
    assert t.run(by["dat"]["a"], by["dat"]["b"], by["dat"]["c"]) == 1 and t.finish
    cli = os.path.join(os.path.dirname(gpu.LIB_PATH), "..", "bin", "tsa")
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"), "tsa_dat")
    os.makedirs(d, exist_ok=True)
    for k in "abc":
        with open(os.path.join(d, f"{k}.dat"), "w") as f:
            f.write("\r\n".join(str(v) for v in by["dat"][k]) + "\r\n")
    r = subprocess.run([cli] + [os.path.join(d, f"{k}.dat") for k in "abc"],
                       capture_output=True, text=True, check=True)
    assert r.stdout.strip().split()[-1] == "1"


@pytest.mark.parametrize("kernel", LITERAL_KERNELS)
@pytest.mark.parametrize("s3_mode,bits", [(0, 12), (1, 12), (0, 0), (0, 16), (1, 9)])
def test_random_small_vs_oracle(gpu, orc, kernel, s3_mode, bits, monkeypatch):
    kernel = _select(kernel, monkeypatch)
    rng = np.random.default_rng(1000 * s3_mode + bits)
    p = gpu.TsaParams.default(s3_mode=s3_mode, score_bits=bits)
    op = orc.default_params(s3_mode=s3_mode, score_bits=bits)
    for _ in range(12):
        la, lb, lc = (int(v) for v in rng.integers(1, 70, 3))
        a, b, c = (rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc))
        if not _kernel_applies(gpu, kernel, la, lb, lc, p):
            continue
        assert gpu.score(a, b, c, p, kernel=kernel) == orc.score(a, b, c, op), (la, lb, lc)


def test_edge_lengths(gpu, orc):
    rng = np.random.default_rng(5)
    for la, lb, lc in [(1, 1, 1), (1, 1, 300), (300, 1, 1), (1, 300, 1), (2, 257, 3), (129, 1, 64),
                       (64, 64, 1), (8, 512, 8), (513, 7, 9)]:
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        assert gpu.score(a, b, c) == orc.score(a, b, c), (la, lb, lc)


def test_wrap_forced(gpu, orc):
    # low-bit SCORE_BITS forces the RTL's candidate wrap (src/PE_1cyc.v:127-133)
    rng = np.random.default_rng(8)
    for bits in (6, 8, 10):
        p, op = gpu.TsaParams.default(score_bits=bits), orc.default_params(score_bits=bits)
        z = [0] * 80
        assert gpu.score(z, z, z, p) == orc.score(z, z, z, op)
        a, b, c = (rng.integers(0, 4, 90).astype(np.uint8) for _ in range(3))
        assert gpu.score(a, b, c, p) == orc.score(a, b, c, op)


def test_params_variants(gpu, orc):
    rng = np.random.default_rng(12)
    a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (40, 33, 47))
    for kw in [dict(match=2, mismatch=-3, gap_open=5, gap_extend=2),
               dict(match=5, mismatch=-4, gap_open=10, gap_extend=1, score_bits=16),
               dict(match=1, mismatch=-1, gap_open=1, gap_extend=2, s3_mode=1),
               dict(match=3, mismatch=0, gap_open=0, gap_extend=0, score_bits=0)]:
        assert gpu.score(a, b, c, gpu.TsaParams.default(**kw)) == orc.score(a, b, c, orc.default_params(**kw)), kw


def test_ragged_batch(gpu, orc):
    rng = np.random.default_rng(21)
    triples = []
    for _ in range(37):
        la, lb, lc = (int(v) for v in rng.integers(1, 90, 3))
        triples.append(tuple(rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc)))
    got = gpu.score_batch(triples)
    seqs, offs = gpu.pack_batch(triples)
    ref = orc.score_batch(seqs, offs, nthreads=8)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("devices", [(0, 0, 0), (0, 0), (0,) * 7])
def test_batch_devices_repeated(gpu, orc, devices):
    """tsa_score_batch_devices with a repeated device list: the host path that
    shards a batch over devices (one thread per distinct device, shards split,
    scores gathered in place) runs on one GPU. Ragged lengths so shards plan
    different kernels (helix, two-triple helix, lap)."""
    rng = np.random.default_rng(len(devices))
    triples = []
    for i in range(23):
        hi = 300 if i % 5 == 0 else 70
        la, lb, lc = (int(v) for v in rng.integers(1, hi, 3))
        triples.append(tuple(rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc)))
    got = gpu.score_batch_devices(triples, devices)
    seqs, offs = gpu.pack_batch(triples)
    assert np.array_equal(got, orc.score_batch(seqs, offs, nthreads=8))
    # more shards than triples: each triple its own shard
    two = triples[:2]
    s2, o2 = gpu.pack_batch(two)
    assert np.array_equal(gpu.score_batch_devices(two, devices), orc.score_batch(s2, o2))
    # error paths: a device out of range refuses before any work
    with pytest.raises(gpu.TsaError) as e:
        gpu.score_batch_devices(triples, (0, gpu.device_count()))
    assert e.value.rc == gpu.TSA_ENODEV


def test_related_high_scores(gpu, orc, synth):
    for seed in range(3):
        a, b, c = synth.related_triple(seed, 200)
        s = gpu.score(a, b, c)
        assert s == orc.score(a, b, c) and s > 100


@pytest.mark.parametrize("kernel", ["plane", "pencil"])
def test_256_cube_vs_oracle(gpu, orc, synth, kernel):
    a, b, c = synth.triple(0, 256)
    assert gpu.score(a, b, c, kernel=kernel) == orc.score(a, b, c)


def test_pencil_shapes_vs_oracle(gpu, orc):
    # helix corner cases: LA < / = / > the lane span, LB not a multiple of the
    # 16-row lap, LC at the 128/256 pair boundaries, tiny and long x
    rng = np.random.default_rng(31)
    for la, lb, lc in [(1, 1, 1), (5, 40, 3), (47, 17, 128), (48, 16, 129), (128, 33, 256),
                       (256, 15, 200), (300, 64, 64), (257, 18, 255), (700, 20, 40),
                       (16, 100, 1), (200, 1, 256), (130, 31, 127)]:
        a, b, c = (rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc))
        assert gpu.score(a, b, c, kernel="pencil") == orc.score(a, b, c), (la, lb, lc)


@pytest.mark.parametrize("mode", ["helix", "lap"])
def test_pencil_wide_positions(gpu, orc, monkeypatch, mode):
    # LC > 256: M = 4 or 8 packed pairs per lane (2 waves per SIMD), both the
    # batch helix and the single-cube lap kernel, f16 and int16 arithmetic
    if mode == "helix":
        monkeypatch.setenv("TSA_PENCIL_MODE", "helix")
    rng = np.random.default_rng(90 if mode == "helix" else 91)
    # 16-bit words: beyond ~680 per side the 12-bit RTL bound no longer holds
    p, op = gpu.TsaParams.default(score_bits=16), orc.default_params(score_bits=16)
    for la, lb, lc in [(64, 20, 257), (300, 33, 512), (40, 17, 513), (257, 40, 700),
                       (130, 24, 1024), (600, 9, 1000)]:
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        assert gpu.score(a, b, c, p, kernel="pencil") == orc.score(a, b, c, op), (mode, la, lb, lc)
    a = rng.integers(0, 4, 700).astype(np.uint8)
    b = a[:64].copy()
    c = a.copy()
    c[::9] = (c[::9] + 1) % 4  # related: scores beyond 2048 need the int16 form
    assert gpu.score(a, b, c, p, kernel="pencil") == orc.score(a, b, c, op), mode


@pytest.mark.parametrize("s3_mode", [0, 1])
def test_vspace_helix(gpu, orc, monkeypatch, s3_mode):
    """The helix's V-space cell (values shifted by lam*(x+y+z), faces injected
    as lam*q; tests/test_cell_algebra.py replays the algebra): ragged batches
    that wrap laps at every phase of the four-step loop, TWO mode (LC <= 64),
    M = 1 and 2, the last wave's early face records; lam = GE = -MISMATCH = 1
    (the exact-f16 form needs |3 MATCH - 3 MISMATCH| <= 7, so lam is 1)."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "helix")
    rng = np.random.default_rng(70 + s3_mode)
    for kw in [dict(), dict(gap_open=3), dict(match=0)]:
        kw = dict(kw, s3_mode=s3_mode)
        p, op = gpu.TsaParams.default(**kw), orc.default_params(**kw)
        for n, hi in ((9, (200, 40, 250)), (21, (100, 30, 64)), (5, (260, 19, 129))):
            triples = [tuple(rng.integers(0, 5, int(rng.integers(1, h + 1))).astype(np.uint8) for h in hi)
                       for _ in range(n)]
            ml = [max(len(t[k]) for t in triples) for k in range(3)]
            assert " f16v " in gpu.describe_plan(n, *ml, p, sync=True), (kw, ml)
            seqs, offs = gpu.pack_batch(triples)
            got = gpu.score_batch(triples, p)
            assert np.array_equal(got, orc.score_batch(seqs, offs, op, nthreads=8)), (kw, ml)
    # related and homopolymer triples: the optimum may leave the z = 0 face at
    # the first steps (position 0's initial faces)
    p = gpu.TsaParams.default(s3_mode=s3_mode)
    triples = []
    for _ in range(40):
        L = int(rng.integers(2, 40))
        a = rng.integers(0, 4, L).astype(np.uint8)
        triples.append((a, a[: int(rng.integers(1, L + 1))].copy(), a[: int(rng.integers(1, L + 1))].copy()))
    seqs, offs = gpu.pack_batch(triples)
    assert np.array_equal(gpu.score_batch(triples, p),
                          orc.score_batch(seqs, offs, orc.default_params(s3_mode=s3_mode), nthreads=8))
    # all-match (the V-space bound's top) and all-distinct triples
    p = gpu.TsaParams.default()
    for a, b, c in ((np.zeros(256, np.uint8),) * 3, tuple(np.full(200, v, np.uint8) for v in (0, 1, 2))):
        assert gpu.score_batch([(a, b, c)] * 3, p)[0] == orc.score(a, b, c)


@pytest.mark.parametrize("geom", [(1, 4), (1, 8), (2, 4), (2, 8), (4, 8)])
@pytest.mark.parametrize("s3_mode", [0, 1])
def test_vspace_lap(gpu, orc, monkeypatch, geom, s3_mode):
    """The lap kernel's V-space cell (lap_kernel VS; tools/lap_emu.py vs=True
    replays it on the CPU): the x = 0 face injected as lam q at x = 1, lap 0's
    y = 0 and tile 0's z = 0 face records written by the loader, the score
    shifted back -- random, related, homopolymer and all-distinct cubes over
    every lap geometry, laps and tiles ragged, against the oracle."""
    m, nw = geom
    monkeypatch.setenv("TSA_LAP_VS", "1")  # opt-in (slower than the message form on MI355X)
    monkeypatch.setenv("TSA_PENCIL_MODE", "lap")
    monkeypatch.setenv("TSA_LAP_M", str(m))
    monkeypatch.setenv("TSA_LAP_NW", str(nw))
    rng = np.random.default_rng(300 + 10 * m + nw + s3_mode)
    cubes = []
    for la, lb, lc in [(70, 41, 140), (9, 33, 300), (128, 17, 64), (33, 80, 200)]:
        cubes.append(tuple(rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc)))
    base = rng.integers(0, 4, 150).astype(np.uint8)
    rel = (base[:150].copy(), base[:120].copy(), base[:140].copy())
    rel[1][::7] = (rel[1][::7] + 1) & 3
    cubes += [rel, (np.zeros(90, np.uint8),) * 3, tuple(np.full(n, v, np.uint8) for n, v in ((80, 0), (66, 1), (130, 2)))]
    for kw in [dict(), dict(gap_open=3), dict(match=0)]:
        kw = dict(kw, s3_mode=s3_mode)
        p, op = gpu.TsaParams.default(**kw), orc.default_params(**kw)
        for a, b, c in cubes:
            assert " f16v " in gpu.describe_plan(1, len(a), len(b), len(c), p, sync=False), kw
            assert gpu.score(a, b, c, p, kernel="pencil") == orc.score(a, b, c, op), (geom, kw, len(a), len(b), len(c))


@pytest.mark.parametrize("arith", ["f16v", "f16", "i16"])
@pytest.mark.parametrize("s3_mode", [0, 1])
def test_pencil_arithmetic_forms(gpu, orc, monkeypatch, arith, s3_mode):
    # helix kernel: exact-f16 (default where the value bound allows) and int16
    # message arithmetic, RTL and sum-of-pairs triple scores, several penalty sets
    monkeypatch.setenv("TSA_PENCIL_MODE", "helix")
    monkeypatch.setenv("TSA_PENCIL_ARITH", arith)
    rng = np.random.default_rng(40 + s3_mode)
    for kw in [dict(), dict(match=2, mismatch=-3, gap_open=5, gap_extend=2),
               dict(match=1, mismatch=0, gap_open=3, gap_extend=1),
               dict(match=3, mismatch=-1, gap_open=2, gap_extend=2, score_bits=16)]:
        kw = dict(kw, s3_mode=s3_mode)
        p, op = gpu.TsaParams.default(**kw), orc.default_params(**kw)
        for la, lb, lc in [(256, 24, 256), (90, 41, 100), (130, 9, 255)]:
            a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
            if rng.random() < 0.5:  # related sequences: long matching runs
                b[: min(la, lb)] = a[: min(la, lb)]
            try:
                got = gpu.score(a, b, c, p, kernel="pencil")
            except gpu.TsaError:
                continue  # pencil not exact for this bound: AUTO would use plane
            assert got == orc.score(a, b, c, op), (arith, kw, la, lb, lc)


def test_pencil_int16_when_f16_range_exceeded(gpu, orc):
    # |values| > 2048: the host must fall back to the int16 form (score_bits 16)
    rng = np.random.default_rng(77)
    p, op = gpu.TsaParams.default(match=5, score_bits=16), orc.default_params(match=5, score_bits=16)
    a = rng.integers(0, 4, 256).astype(np.uint8)
    c = a.copy()
    c[::17] = (c[::17] + 1) % 4
    b = a[:200].copy()
    assert gpu.score(a, b, c, p, kernel="pencil") == orc.score(a, b, c, op)


@pytest.mark.parametrize("mode", ["helix", "lap"])
def test_pencil_single_cube_modes(gpu, orc, synth, monkeypatch, mode):
    # "lap": one 16-row lap per workgroup, laps chained through global memory
    # with progress flags; "helix": one workgroup walks all laps
    if mode == "helix":
        monkeypatch.setenv("TSA_PENCIL_MODE", "helix")
    rng = np.random.default_rng(5 if mode == "helix" else 6)
    for la, lb, lc in [(256, 256, 256), (64, 64, 64), (200, 17, 129), (31, 250, 100), (1, 40, 1),
                       (500, 33, 256)]:
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        assert gpu.score(a, b, c, kernel="pencil") == orc.score(a, b, c), (mode, la, lb, lc)


@pytest.mark.parametrize("nw", ["4", "8"])
def test_pencil_lap_rows_per_lap(gpu, orc, synth, monkeypatch, nw):
    monkeypatch.setenv("TSA_LAP_NW", nw)
    rng = np.random.default_rng(40 + int(nw))
    for la, lb, lc in [(256, 256, 256), (100, 37, 200), (17, 90, 5)]:
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        assert gpu.score(a, b, c, kernel="pencil") == orc.score(a, b, c), (nw, la, lb, lc)


@pytest.mark.parametrize("m", ["1", "2", "4"])
def test_pencil_lap_z_tiles(gpu, orc, monkeypatch, m):
    # single-cube lap kernel with the z axis cut into 64*M-position tiles (M
    # packed pairs per lane) that hand their last position to the next tile's
    # position 0 every step; partial last tiles, one-lap cubes, LA below/above
    # the tile width
    monkeypatch.setenv("TSA_PENCIL_MODE", "lap")
    monkeypatch.setenv("TSA_LAP_M", m)
    rng = np.random.default_rng(60 + int(m))
    p, op = gpu.TsaParams.default(score_bits=16), orc.default_params(score_bits=16)
    for la, lb, lc in [(300, 16, 300), (130, 40, 260), (150, 16, 129), (64, 17, 130),
                       (256, 48, 256), (40, 33, 513), (520, 20, 700)]:
        a = rng.integers(0, 4, max(la, lc)).astype(np.uint8)
        b = a[:lb].copy()
        b[::5] = (b[::5] + 1) % 4
        c = a[:lc].copy()
        c[::9] = (c[::9] + 2) % 4  # related sequences: long matching runs
        assert gpu.score(a[:la], b, c, p, kernel="pencil") == orc.score(a[:la], b, c, op), \
            (m, la, lb, lc)


def test_pencil_lap_mode_small_batch(gpu, orc):
    # several triples in lap mode at once (n * laps <= resident workgroups)
    rng = np.random.default_rng(9)
    triples = [tuple(rng.integers(0, 4, n).astype(np.uint8) for n in (int(rng.integers(1, 260)), int(rng.integers(17, 120)), int(rng.integers(1, 257))))
               for _ in range(12)]
    got = gpu.score_batch(triples)
    seqs, offs = gpu.pack_batch(triples)
    assert np.array_equal(got, orc.score_batch(seqs, offs, nthreads=8))


def test_pencil_lap_streaming_batch(gpu, orc, monkeypatch, tmp_path):
    # sync batch API with more lap workgroups than resident slots: the grid runs
    # in 2-3 dispatch rounds with boundary rings (bounded spins, error word
    # checked, helix rerun on timeout); 60 triples x 8 laps x 2 tiles = 960
    # workgroups (M = 1, NW = 8) for 512 slots. The lap trace proves it ran.
    monkeypatch.setenv("TSA_PENCIL_MODE", "lap")
    trace = tmp_path / "lap.csv"
    monkeypatch.setenv("TSA_LAP_TRACE", str(trace))
    rng = np.random.default_rng(91)
    triples = []
    for _ in range(60):
        la, lc = int(rng.integers(100, 129)), int(rng.integers(1, 129))
        triples.append(tuple(rng.integers(0, 4, n).astype(np.uint8) for n in (la, 128, lc)))
    seqs, offs = gpu.pack_batch(triples)
    before = gpu.fallback_count()
    assert np.array_equal(gpu.score_batch(triples),
                          orc.score_batch(seqs, offs, nthreads=8))
    rows = trace.read_text().splitlines()
    plan = gpu.describe_plan(len(triples), 129, 128, 128, sync=True)
    kv = dict(f.split("=") for f in plan.split() if "=" in f)
    m, nw = int(kv["M"]), int(kv["NW"])
    want = sum(-(-128 // (2 * nw)) * -(-len(t[2]) // (64 * m)) for t in triples)
    assert int(kv["waves"]) > 1 and len(rows) - 1 == want, (plan, len(rows) - 1, want)
    assert gpu.fallback_count() == before, "a lap hand-off timed out and was rescored"


def test_lap_looped_rounds_several_per_cu(gpu, orc, monkeypatch):
    """A looped multi-round lap grid at two or more workgroups per CU (ADVICE
    r4): the residency estimate is load-bearing there -- a physical block that
    only starts once the resident ones finish would leave its round-0
    consumers spinning into a timeout and a counted rescore. Sync and async
    paths: oracle-equal, no fallback counted, no TSA_SCORE_INVALID."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "lap")
    monkeypatch.setenv("TSA_LAP_M", "1")
    monkeypatch.setenv("TSA_LAP_NW", "4")
    rng = np.random.default_rng(123)
    triples = [tuple(rng.integers(0, 4, n).astype(np.uint8) for n in (64, 256, int(rng.integers(65, 129))))
               for _ in range(24)]
    plan = gpu.describe_plan(len(triples), 64, 256, 128, sync=True)
    kv = dict(f.split("=") for f in plan.split() if "=" in f)
    assert int(kv["waves"]) >= 2 and int(kv["wpc"]) >= 2, plan
    seqs, offs = gpu.pack_batch(triples)
    ref = orc.score_batch(seqs, offs, nthreads=8)
    before = gpu.fallback_count()
    assert np.array_equal(gpu.score_batch(triples), ref), plan
    assert gpu.fallback_count() == before, "a lap hand-off timed out and was rescored: " + plan
    import torch
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_sc = torch.zeros(len(triples), dtype=torch.int32, device="cuda")
    p = gpu.TsaParams.default()
    ws = gpu.workspace_size(len(triples), 64, 256, 128, p, "pencil")
    d_ws = torch.empty(ws, dtype=torch.uint8, device="cuda")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), len(triples), 64, 256, 128, d_sc.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, p, "pencil")
    torch.cuda.synchronize()
    assert np.array_equal(d_sc.cpu().numpy(), ref), plan


def test_lap_late_consumer_keeps_its_prologue_records(gpu, orc, monkeypatch):
    """One workgroup per CU, three looped rounds, slim z rings (600^3, int16,
    M = 1, NW = 8): a round-2 z consumer starts only when its physical
    workgroup finishes a round-1 lap, while its producer, resident earlier,
    runs ahead. The producer must not overwrite the records the consumer's
    loader prologue reads (ZT - 2 .. ZT + ZA - 1) before the consumer has
    published any progress -- the z back-pressure once counted them consumed
    at progress 0, and the four-step groups made the producer fast enough to
    overwrite them: every such launch timed out (TSA_SCORE_INVALID)."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "lap")
    monkeypatch.setenv("TSA_LAP_M", "1")
    monkeypatch.setenv("TSA_LAP_NW", "8")
    monkeypatch.setenv("TSA_PENCIL_ARITH", "i16")
    L = 600
    rng = np.random.default_rng(600)
    a, b, c = (rng.integers(0, 4, L).astype(np.uint8) for _ in range(3))
    p = gpu.TsaParams.default(score_bits=16)
    plan = gpu.describe_plan(1, L, L, L, p, "pencil", sync=False)
    kv = dict(f.split("=") for f in plan.split() if "=" in f)
    assert " i16 " in plan and int(kv["waves"]) >= 2 and int(kv["wpc"]) == 1, plan
    ref = orc.score(a, b, c, orc.default_params(score_bits=16))
    for _ in range(3):
        assert _score_async(gpu, [(a, b, c)], p, "pencil", L)[0] == ref, plan


def test_pencil_ragged_batch(gpu, orc):
    rng = np.random.default_rng(77)
    triples = []
    for _ in range(50):
        la, lb, lc = int(rng.integers(1, 300)), int(rng.integers(1, 80)), int(rng.integers(1, 257))
        triples.append(tuple(rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc)))
    seqs, offs = gpu.pack_batch(triples)
    ref = orc.score_batch(seqs, offs, nthreads=8)
    import torch
    n = len(triples)
    mla = max(len(t[0]) for t in triples); mlb = max(len(t[1]) for t in triples); mlc = max(len(t[2]) for t in triples)
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_scores = torch.zeros(n, dtype=torch.int32, device="cuda")
    ws = gpu.workspace_size(n, mla, mlb, mlc, kernel="pencil")
    d_ws = torch.empty(ws, dtype=torch.uint8, device="cuda")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), n, mla, mlb, mlc, d_scores.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, kernel="pencil")
    torch.cuda.synchronize()
    assert np.array_equal(d_scores.cpu().numpy(), ref)


def test_full_size_properties(gpu):
    # all-A n^3 -> 3n (KAT family) at the 256^3 and 1024^3 configs
    z = np.zeros(256, np.uint8)
    assert gpu.score(z, z, z) == 768
    z = np.zeros(1024, np.uint8)
    assert gpu.score(z, z, z, gpu.TsaParams.default(score_bits=0)) == 3072


def test_ab_symmetry_256(gpu, synth):
    a, b, c = synth.triple(3, 256)
    assert gpu.score(a, b, c) == gpu.score(b, a, c)


def test_batch_async_device_pointers(gpu, orc, synth):
    import torch
    n, L = 6, 96
    seqs, offs = synth.batch(0, n, L)
    d_seqs = torch.from_numpy(seqs).cuda()
    d_offs = torch.from_numpy(offs).cuda()
    d_scores = torch.zeros(n, dtype=torch.int32, device="cuda")
    for kernel in ("plane", "pencil", "auto"):
        ws = gpu.workspace_size(n, L, L, L, kernel=kernel)
        d_ws = torch.empty(max(ws, 1), dtype=torch.uint8, device="cuda")
        gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), n, L, L, L, d_scores.data_ptr(),
                              d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream,
                              kernel=kernel)
        torch.cuda.synchronize()
        assert np.array_equal(d_scores.cpu().numpy(), orc.score_batch(seqs, offs, nthreads=6))


def test_1024_cube_config_c4(gpu, orc, synth):
    # configs[3]: one 1024^3 synthetic triple, 16-bit words (beyond the RTL's
    # 512 envelope the 12-bit wrap is not meaningful); lap kernel with 8 packed
    # pairs per lane. The oracle needs ~30 s of one CPU core.
    a, b, c = synth.triple(0, 1024)
    p, op = gpu.TsaParams.default(score_bits=16), orc.default_params(score_bits=16)
    assert gpu.score(a, b, c, p, kernel="pencil") == orc.score(a, b, c, op)



@pytest.mark.parametrize("two", ["0", "1"])
def test_pencil_two_triples_per_wave(gpu, orc, monkeypatch, two):
    # LC <= 64: a wave's halves hold two different triples (TWO) -- ragged
    # pairs whose final cells fall in different steps, an odd batch (the last
    # workgroup scores one triple), LA above and below the 64-step lap period,
    # f16 and int16, both s3 modes
    monkeypatch.setenv("TSA_PENCIL_MODE", "helix")
    monkeypatch.setenv("TSA_PENCIL_TWO", two)
    rng = np.random.default_rng(80 + int(two))
    for kw, arith in [(dict(), "f16"), (dict(s3_mode=1), "f16"), (dict(), "i16"),
                      (dict(match=2, mismatch=-3, gap_open=5, gap_extend=2, score_bits=16), "f16")]:
        monkeypatch.setenv("TSA_PENCIL_ARITH", arith)
        triples = []
        for _ in range(23):
            la, lb, lc = int(rng.integers(1, 140)), int(rng.integers(1, 70)), int(rng.integers(1, 65))
            triples.append(tuple(rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc)))
        seqs, offs = gpu.pack_batch(triples)
        ref = orc.score_batch(seqs, offs, orc.default_params(**kw), nthreads=8)
        got = gpu.score_batch(triples, gpu.TsaParams.default(**kw))
        assert np.array_equal(got, ref), (two, kw, arith)


# ---- round 2: configs[4] shard, the RTL's largest cubes, lap failure path ----

def test_configs4_full_shard_sampled(gpu, orc, synth):
    """configs[4]'s per-GPU shard exactly as bench.py runs it: 512 independent
    256^3 triples resident in HBM, one tsa_score_batch_async launch on torch's
    stream; >= 16 triples spread over the shard (both ends included) against
    the oracle, every score in range."""
    import torch
    n, L = 512, 256
    seqs, offs = synth.batch(0, n, L)
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_scores = torch.full((n,), -7777, dtype=torch.int32, device="cuda")
    ws = gpu.workspace_size(n, L, L, L)
    d_ws = torch.empty(ws, dtype=torch.uint8, device="cuda")
    assert gpu.describe_plan(n, L, L, L, sync=False).startswith("pencil helix f16")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), n, L, L, L, d_scores.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_scores.cpu().numpy()
    idx = sorted(set([0, 1, n - 2, n - 1] + [int(v) for v in np.linspace(0, n - 1, 16)]))
    cs, co = gpu.pack_batch([synth.triple(i, L) for i in idx])
    ref = orc.score_batch(cs, co, nthreads=16)
    assert np.array_equal(got[idx], ref), (idx, got[idx], ref)
    assert got.min() > -3 * L - 16 and got.max() <= 3 * L  # value bound, no sentinel left


@pytest.mark.parametrize("kind", ["random", "all_a", "all_mismatch", "related"])
def test_512_cube_rtl_params(gpu, orc, synth, kind):
    """The RTL's largest input (A_TOTAL_LEN = 512, src/TriAlign_1cyc.v:7) with
    its 12-bit words: the value bound [-1544, 1536] fits 12 bits, so AUTO runs
    the pencil path (factored f16 form) and must equal the literal oracle --
    including the cubes at the two ends of the bound."""
    L = 512
    if kind == "random":
        a, b, c = synth.triple(5, L)
    elif kind == "all_a":          # the upper end: 3 per diagonal step -> 1536
        a = b = c = np.zeros(L, np.uint8)
    elif kind == "all_mismatch":   # a != b != c everywhere: the low side
        a, b, c = (np.full(L, v, np.uint8) for v in (0, 1, 2))
    else:
        a, b, c = synth.related_triple(11, L)
    assert gpu.describe_plan(1, L, L, L).startswith("pencil ")
    got = gpu.score(a, b, c)
    assert got == orc.score(a, b, c), kind
    if kind == "all_a":
        assert got == 3 * L


def test_lap_timeout_is_reported_not_silent(gpu, orc, synth, monkeypatch):
    """Injected lap hand-off timeout (TSA_LAP_SPIN_LIMIT=0: the first poll of
    every consumer gives up): the async path marks the triple
    TSA_SCORE_INVALID; the synchronous path counts the fallback, rescored the
    chunk with the helix kernel and still returns the exact score."""
    import torch
    L = 256
    a, b, c = synth.triple(2, L)
    ref = orc.score(a, b, c)
    monkeypatch.setenv("TSA_LAP_SPIN_LIMIT", "0")
    assert gpu.describe_plan(1, L, L, L, sync=False).startswith("pencil lap")
    seqs, offs = gpu.pack_batch([(a, b, c)])
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_score = torch.zeros(1, dtype=torch.int32, device="cuda")
    ws = gpu.workspace_size(1, L, L, L)
    d_ws = torch.empty(ws, dtype=torch.uint8, device="cuda")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), 1, L, L, L, d_score.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(d_score.item()) == gpu.SCORE_INVALID
    before = gpu.fallback_count()
    assert gpu.score(a, b, c) == ref
    assert gpu.fallback_count() == before + 1
    monkeypatch.delenv("TSA_LAP_SPIN_LIMIT")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), 1, L, L, L, d_score.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(d_score.item()) == ref
    assert gpu.score(a, b, c) == ref and gpu.fallback_count() == before + 1


@pytest.mark.parametrize("m,nw", [(1, 4), (1, 8), (2, 4), (2, 8), (4, 4), (4, 8)])
def test_lap_kernel_geometries_adversarial(gpu, orc, monkeypatch, m, nw):
    """Every (M, NW) geometry of the lap kernel on cubes whose optimum runs
    through lap and tile seams: all-mismatch (values near the low bound; the
    seam cell (1, y, 64M+1) takes its step-0 inputs from the left tile's
    records ZT-2 / ZT-1), all-match, related and random, ragged shapes."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "lap")
    monkeypatch.setenv("TSA_LAP_M", str(m))
    monkeypatch.setenv("TSA_LAP_NW", str(nw))
    rng = np.random.default_rng(100 * m + nw)
    for la, lb, lc in [(100, 100, 100), (130, 70, 300), (64, 33, 129), (200, 41, 257), (17, 90, 65)]:
        for kind in ("mismatch", "match", "related", "random"):
            if kind == "mismatch":
                a, b, c = (np.full(n, v, np.uint8) for n, v in zip((la, lb, lc), (0, 1, 2)))
            elif kind == "match":
                a, b, c = (np.zeros(n, np.uint8) for n in (la, lb, lc))
            elif kind == "related":
                base = rng.integers(0, 4, max(la, lb, lc)).astype(np.uint8)
                a, b, c = base[:la].copy(), base[:lb].copy(), base[:lc].copy()
                b[::7] = (b[::7] + 1) % 4
                c[::5] = (c[::5] + 2) % 4
            else:
                a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
            assert gpu.score(a, b, c, kernel="pencil") == orc.score(a, b, c), (m, nw, la, lb, lc, kind)


def _score_async(gpu, triples, p, kernel, L):
    import torch
    seqs, offs = gpu.pack_batch(triples)
    n = len(triples)
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_score = torch.zeros(n, dtype=torch.int32, device="cuda")
    ws = gpu.workspace_size(n, L, L, L, p, kernel)
    d_ws = torch.empty(max(ws, 16), dtype=torch.uint8, device="cuda")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), n, L, L, L, d_score.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, p, kernel)
    torch.cuda.synchronize()
    return d_score.cpu().numpy()


def _score_async_dims(gpu, a, b, c, p, kernel, env=None):
    """One triple through tsa_score_batch_async with its own max dims, under
    temporary library knobs (env)."""
    import torch
    saved = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        seqs, offs = gpu.pack_batch([(a, b, c)])
        la, lb, lc = len(a), len(b), len(c)
        d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
        d_score = torch.zeros(1, dtype=torch.int32, device="cuda")
        ws = gpu.workspace_size(1, la, lb, lc, p, kernel)
        d_ws = torch.empty(max(ws, 16), dtype=torch.uint8, device="cuda")
        plan = gpu.describe_plan(1, la, lb, lc, p, kernel, sync=False)
        gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), 1, la, lb, lc, d_score.data_ptr(),
                              d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, p, kernel)
        torch.cuda.synchronize()
        return int(d_score.cpu().numpy()[0]), plan
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_lap_multiround_geometry_sweep(gpu):
    """Every forced lap geometry (M 1 / 2, NW 4 / 8, f16 / int16) on large
    ragged cubes whose grids need looped rounds at one or two workgroups per
    CU -- where round 5 found a late consumer's prologue records overwritten --
    against the literal kernel family on the same input (16-bit words: no value
    wraps, so the factored and literal recurrences agree; the oracle would take
    minutes per cube). Async path: a timed-out hand-off reads
    TSA_SCORE_INVALID and fails the comparison."""
    rng = np.random.default_rng(2024)
    p = gpu.TsaParams.default(score_bits=16)
    shapes = [(520, 700, 600), (700, 560, 900), (1000, 300, 400), (300, 1100, 650)]
    rounds = 0
    for la, lb, lc in shapes:
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        ref, ref_plan = _score_async_dims(gpu, a, b, c, p, "plane")
        assert ref > gpu.SCORE_UNCERTIFIED, ref_plan
        for m in (1, 2):
            for nw in (4, 8):
                for arith in ("f16", "i16"):
                    env = {"TSA_PENCIL_MODE": "lap", "TSA_LAP_M": str(m), "TSA_LAP_NW": str(nw),
                           "TSA_PENCIL_ARITH": arith}
                    got, plan = _score_async_dims(gpu, a, b, c, p, "pencil", env)
                    if " lap " not in plan:
                        continue  # geometry not launchable for this shape (planner fell back)
                    kv = dict(f.split("=") for f in plan.split() if "=" in f)
                    rounds += int(kv.get("waves", "1")) > 1
                    assert got == ref, (la, lb, lc, plan, got, ref, ref_plan)
    assert rounds >= 8, rounds  # the sweep did run looped multi-round grids


def test_checked_1024_rtl_words(gpu, orc, synth):
    """The RTL's 12-bit words at 1024^3 (a-priori bound 3072: the factored form
    is not provably exact, round 1 ran 29 ms of PLANE): the checked lap kernel
    monitors every real cell's best and certifies the random cube, so the
    synchronous path returns the literal wrapped recurrence's score without a
    PLANE rescore. Oracle: ~30 s of one core."""
    L = 1024
    a, b, c = synth.triple(5, L)
    p = gpu.TsaParams.default()
    assert gpu.describe_plan(1, L, L, L, p, sync=True).split(" est=")[0].endswith(" checked")
    before = gpu.check_fallback_count()
    got = gpu.score(a, b, c, p)
    assert got == orc.score(a, b, c, orc.default_params())
    assert gpu.check_fallback_count() == before
    assert _score_async(gpu, [(a, b, c)], p, "checked", L)[0] == got


@pytest.mark.parametrize("kind", ["match", "mismatch"])
def test_checked_uncertified_falls_back_to_plane(gpu, orc, kind):
    """Cubes whose values do leave the word: all-match 690^3 with 12-bit words
    (score 2070 wraps), all-mismatch 90^3 with 8-bit words (best down to -180).
    The monitor refuses to certify: async reports TSA_SCORE_UNCERTIFIED, the
    synchronous path rescored with PLANE (counted) and returns the RTL's
    wrapped score. (All-mismatch with 12-bit words does not wrap -- its best
    stays near -2 per position -- and is certified: see the 1024^3 test.)"""
    if kind == "match":
        L, bits = 690, 12
        a = b = c = np.zeros(L, np.uint8)
    else:
        L, bits = 90, 8
        a, b, c = (np.full(L, v, np.uint8) for v in (0, 1, 2))
    p, op = gpu.TsaParams.default(score_bits=bits), orc.default_params(score_bits=bits)
    ref = orc.score(a, b, c, op)
    assert _score_async(gpu, [(a, b, c)], p, "checked", L)[0] == gpu.SCORE_UNCERTIFIED
    before = gpu.check_fallback_count()
    assert gpu.score(a, b, c, p) == ref
    assert gpu.check_fallback_count() == before + 1


def test_checked_narrow_words_batch(gpu, orc):
    """SCORE_BITS 8 and 9 on small cubes: the synchronous batch path tries the
    checked kernel, certifies what stays in range and rescores the rest with
    PLANE -- every score equals the literal wrapped oracle."""
    rng = np.random.default_rng(91)
    for bits in (8, 9):
        triples = [tuple(rng.integers(0, 4, n).astype(np.uint8) for n in (90, 70, 100))
                   for _ in range(3)]
        p, op = gpu.TsaParams.default(score_bits=bits), orc.default_params(score_bits=bits)
        assert gpu.describe_plan(3, 90, 70, 100, p, sync=True).split(" est=")[0].endswith(" checked")
        seqs, offs = gpu.pack_batch(triples)
        assert np.array_equal(gpu.score_batch(triples, p), orc.score_batch(seqs, offs, op, nthreads=3))


@pytest.mark.parametrize("kernel", ["plane", "pencil", "auto"])
def test_packed2_input_matches_bytes(gpu, orc, kernel):
    """tsa_score_batch_async_p2: the same batch, 2-bit packed (ragged lengths,
    so triples start mid-byte; N symbols), scores identically to the
    byte-per-symbol input on every kernel family -- helix (batch), lap (a few
    cubes) and plane -- and to the oracle."""
    import torch
    rng = np.random.default_rng(33)
    for n, L in ((37, 70), (2, 200)):
        triples = [tuple(rng.integers(0, 5, int(rng.integers(1, L + 1))).astype(np.uint8) for _ in range(3))
                   for _ in range(n)]
        seqs, offs = gpu.pack_batch(triples)
        ml = [max(len(t[k]) for t in triples) for k in range(3)]
        p = gpu.TsaParams.default()
        ref = orc.score_batch(seqs, offs, orc.default_params(), nthreads=8)
        ws = gpu.workspace_size(n, *ml, p, kernel)
        d_ws = torch.empty(max(ws, 16), dtype=torch.uint8, device="cuda")
        d_offs = torch.from_numpy(offs).cuda()
        st = torch.cuda.current_stream().cuda_stream
        out = []
        for packed in (False, True):
            d_seqs = torch.from_numpy(gpu.pack2(seqs) if packed else seqs).cuda()
            d_sc = torch.zeros(n, dtype=torch.int32, device="cuda")
            fn = gpu.score_batch_async_p2 if packed else gpu.score_batch_async
            fn(d_seqs.data_ptr(), d_offs.data_ptr(), n, *ml, d_sc.data_ptr(), d_ws.data_ptr(), ws, st, p, kernel)
            torch.cuda.synchronize()
            out.append(d_sc.cpu().numpy())
        assert np.array_equal(out[0], ref) and np.array_equal(out[1], ref), (kernel, n, L)


# ---- one cube split over devices by laps (tsa_score_gpu_multi)
@pytest.mark.parametrize("L,parts", [(64, 2), (128, 2), (256, 2), (256, 4), (512, 3)])
def test_split_cube_matches_oracle(gpu, orc, synth, L, parts):
    """The cube's laps cut into `parts` contiguous runs, each its own launch
    with its own fine-grained workspace, handing y records to the next by
    system-scope stores -- on one box the parts share device 0 (concurrent
    launches on separate streams), which runs the same protocol as the
    multi-GPU case minus the xGMI hop. Must equal the literal oracle."""
    a, b, c = synth.triple(40 + L + parts, L)
    got, wall = gpu.score_multi(a, b, c, [0] * parts)
    assert got == orc.score(a, b, c)
    assert wall > 0


@pytest.mark.parametrize("kind", ["all_a", "all_mismatch", "related"])
def test_split_cube_extremes(gpu, orc, synth, monkeypatch, kind):
    """Seam cases across the part boundary: the optimum of all-A runs down the
    diagonal through every boundary lap; all-mismatch sits at the low bound."""
    L = 192
    if kind == "all_a":
        a = b = c = np.zeros(L, np.uint8)
    elif kind == "all_mismatch":
        a, b, c = (np.full(L, v, np.uint8) for v in (0, 1, 2))
    else:
        a, b, c = synth.related_triple(7, L)
    got, _ = gpu.score_multi(a, b, c, [0, 0])
    assert got == orc.score(a, b, c), kind
    if kind == "all_a":
        assert got == 3 * L


def test_split_cube_int16_and_ragged(gpu, orc, synth):
    """Ragged lengths (lap and tile counts not multiples of the part count) and
    the int16 form (match 5 with 16-bit words: the bound leaves the exact-f16
    range at 150^3)."""
    a, b, c = synth.triple(3, 150)
    b, c = b[:101], c[:77]
    assert gpu.score_multi(a, b, c, [0, 0, 0])[0] == orc.score(a, b, c)
    kw = dict(match=5, mismatch=-4, gap_open=10, gap_extend=1, score_bits=16)
    a, b, c = synth.triple(9, 150)
    got = gpu.score_multi(a, b, c, [0, 0], gpu.TsaParams.default(**kw))[0]
    assert got == orc.score(a, b, c, orc.default_params(**kw))


def test_split_cube_errors(gpu, synth):
    """Fewer laps than parts and bad device ids are refused with the
    reference-style error codes, never a silent score."""
    a, b, c = synth.triple(1, 16)
    with pytest.raises(gpu.TsaError) as e:
        gpu.score_multi(a, b, c, [0] * 8)   # 16 rows = 2 laps < 8 parts
    assert e.value.rc == gpu.TSA_ERANGE
    with pytest.raises(gpu.TsaError) as e:
        gpu.score_multi(a, b, c, [gpu.device_count()])
    assert e.value.rc == gpu.TSA_ENODEV


@pytest.mark.parametrize("kw", [dict(score_bits=6), dict(gap_open=1, gap_extend=2, score_bits=12),
                                dict(score_bits=9, s3_mode=1)])
def test_split_cube_literal(gpu, orc, synth, kw):
    """Parameter sets the factored form cannot run exactly split in the
    literal arithmetic (lap_kernel LIT with system-scope hand-offs): narrow
    words that wrap, GO < GE, SOP s3 -- 2 and 3 parts, ragged, equal to the
    oracle's literal score."""
    p, op = gpu.TsaParams.default(**kw), orc.default_params(**kw)
    rng = np.random.default_rng(55)
    h = rng.integers(0, 4, 170).astype(np.uint8)
    cases = [synth.triple(5, 150), (h, h[:133].copy(), h[:149].copy())]
    for a, b, c in cases:
        ref = orc.score(a, b, c, op)
        for parts in ([0, 0], [0, 0, 0]):
            assert gpu.score_multi(a, b, c, parts, p)[0] == ref, (kw, parts, len(b))


def test_split_cube_literal_1024_rtl_words(gpu, orc, synth):
    """configs[3]'s 1024^3 cube with the RTL's 12-bit words (beyond the
    factored form's a-priori bound) split in 2 parts in the literal
    arithmetic: the oracle's literal score."""
    a, b, c = synth.triple(0, 1024)
    p = gpu.TsaParams.default(score_bits=12)
    assert gpu.score_multi(a, b, c, [0, 0], p)[0] == orc.score(a, b, c, orc.default_params(score_bits=12))


def test_split_cube_timeout_is_reported_not_silent(gpu, synth, monkeypatch):
    """Injected hand-off timeout (TSA_LAP_SPIN_LIMIT=0: a consumer's first
    poll gives up) on the split path: TSA_EINTERNAL, never a score; the next
    call with the default limit is exact again."""
    a, b, c = synth.triple(5, 128)
    monkeypatch.setenv("TSA_LAP_SPIN_LIMIT", "0")
    with pytest.raises(gpu.TsaError) as e:
        gpu.score_multi(a, b, c, [0, 0])
    assert e.value.rc == gpu.TSA_EINTERNAL
    monkeypatch.delenv("TSA_LAP_SPIN_LIMIT")
    import oracle
    assert gpu.score_multi(a, b, c, [0, 0])[0] == oracle.score(a, b, c)


@pytest.mark.parametrize("devs", [[0, 1], [0, 1, 1], [1, 0]])
def test_split_cube_across_devices(gpu, orc, synth, devs):
    """The real multi-GPU split: peer access, fine-grained rings on distinct
    devices and system-scope hand-offs over xGMI (skipped on a one-GPU box).
    256^3 and a ragged shape; no fallback may fire."""
    if gpu.device_count() < 2:
        pytest.skip("needs two HIP devices")
    before = (gpu.fallback_count(), gpu.check_fallback_count())
    a, b, c = synth.triple(11, 256)
    assert gpu.score_multi(a, b, c, devs)[0] == orc.score(a, b, c)
    a, b, c = synth.triple(12, 200)
    b, c = b[:173], c[:131]
    assert gpu.score_multi(a, b, c, devs)[0] == orc.score(a, b, c)
    assert (gpu.fallback_count(), gpu.check_fallback_count()) == before


# ---- the literal helix (csrc/literal_kernel.hip): TSA_KERNEL_PLANE's batch path
@pytest.mark.parametrize("bits,s3_mode", [(12, 0), (12, 1), (9, 0), (6, 1), (4, 0), (16, 0)])
def test_literal_helix_matches_oracle(gpu, orc, monkeypatch, bits, s3_mode):
    """The RTL's literal arithmetic in push form on the helix schedule (every
    candidate wrapped to SCORE_BITS by int16 arithmetic on values shifted left
    by 16 - SCORE_BITS; tools/literal_emu.py replays it): narrow words that
    wrap, both s3 modes, ragged batches over M = 1, 2 and 4, related triples."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "literal")
    rng = np.random.default_rng(200 + bits + s3_mode)
    p, op = gpu.TsaParams.default(score_bits=bits, s3_mode=s3_mode), orc.default_params(score_bits=bits, s3_mode=s3_mode)
    for n, hi in ((7, (150, 30, 100)), (5, (260, 21, 256)), (3, (40, 17, 129)), (3, (90, 12, 512))):
        triples = [tuple(rng.integers(0, 5, int(rng.integers(1, h + 1))).astype(np.uint8) for h in hi)
                   for _ in range(n)]
        a = rng.integers(0, 4, 120).astype(np.uint8)
        triples.append((a, a[:60].copy(), a[:110].copy()))  # related: high scores
        for _ in range(12):  # short related / homopolymer triples
            L = int(rng.integers(2, 30))
            h = rng.integers(0, 4, L).astype(np.uint8)
            triples.append((h, h[: int(rng.integers(1, L + 1))].copy(), h[: int(rng.integers(1, L + 1))].copy()))
        ml = [max(len(t[k]) for t in triples) for k in range(3)]
        assert gpu.describe_plan(len(triples), *ml, p, kernel="plane").startswith("plane literal-helix")
        seqs, offs = gpu.pack_batch(triples)
        ws = gpu.workspace_size(len(triples), *ml, p, "plane")
        import torch
        d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
        d_sc = torch.zeros(len(triples), dtype=torch.int32, device="cuda")
        d_ws = torch.empty(max(ws, 16), dtype=torch.uint8, device="cuda")
        gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), len(triples), *ml, d_sc.data_ptr(),
                              d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, p, "plane")
        torch.cuda.synchronize()
        got = d_sc.cpu().numpy()
        assert np.array_equal(got, orc.score_batch(seqs, offs, op, nthreads=8)), (bits, s3_mode, ml)


def test_literal_helix_final_states_and_wrap(gpu, orc, golden, monkeypatch):
    """Final 7-tuples from the literal helix (the 84-bit SRAM word,
    src/TriAlign_1cyc.v:130,138) on the golden fixtures, and an all-match cube
    whose diagonal wraps a 9-bit word (3 x 120 = 360 > 255)."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "literal")
    used = 0
    for c in golden:
        if len(c["c"]) > 256 or "final7" not in c:
            continue
        p = gpu.TsaParams.default(**c["params"])
        s, fin = gpu.score(c["a"], c["b"], c["c"], p, final_states=True)
        assert (s, list(fin)) == (c["score"], c["final7"]), c["name"]
        used += 1
    assert used >= 10
    a = np.zeros(120, np.uint8)
    p9, o9 = gpu.TsaParams.default(score_bits=9), orc.default_params(score_bits=9)
    ref = orc.score(a, a, a, o9, final_states=True)
    s, fin = gpu.score(a, a, a, p9, final_states=True)
    assert (s, tuple(fin)) == ref and ref[0] != 360


# ---- the literal lap schedule (lap_kernel LIT): TSA_KERNEL_PLANE's single-cube path
LIT_GEOMS = [("1", "4"), ("1", "8"), ("2", "4"), ("2", "8")]


@pytest.mark.parametrize("m,nw", LIT_GEOMS)
@pytest.mark.parametrize("bits,s3_mode", [(12, 0), (6, 1), (16, 0)])
def test_literal_lap_matches_oracle(gpu, orc, monkeypatch, m, nw, bits, s3_mode):
    """The RTL's literal arithmetic on the single-cube lap schedule
    (tools/litlap_emu.py replays it): scores and final 7-tuples equal the
    oracle's on ragged cubes over several laps and z-tiles, related and
    homopolymer triples, narrow words that wrap, both s3 modes."""
    monkeypatch.setenv("TSA_PENCIL_MODE", "litlap")
    monkeypatch.setenv("TSA_LAP_M", m)
    monkeypatch.setenv("TSA_LAP_NW", nw)
    rng = np.random.default_rng(300 + 7 * int(m) + int(nw) + bits + s3_mode)
    p, op = gpu.TsaParams.default(score_bits=bits, s3_mode=s3_mode), orc.default_params(score_bits=bits, s3_mode=s3_mode)
    shapes = [(64, 64, 64), (37, 70, 131), (90, 17, 65), (5, 33, 200), (120, 9, 129)]
    cases = [tuple(rng.integers(0, 5, n).astype(np.uint8) for n in sh) for sh in shapes]
    h = rng.integers(0, 4, 150).astype(np.uint8)
    cases.append((h, h[:41].copy(), h[:140].copy()))                     # related: high scores
    z = np.zeros(100, np.uint8)
    cases.append((z, z[:50].copy(), z[:90].copy()))                      # homopolymer (wraps at 6 bits)
    for a, b, c in cases:
        plan = gpu.describe_plan(1, len(a), len(b), len(c), p, kernel="plane", sync=True)
        assert plan.startswith(f"plane literal-lap M={m} NW={nw}"), plan
        s, fin = gpu.score(a, b, c, p, kernel="plane", final_states=True)
        assert (s, tuple(fin)) == orc.score(a, b, c, op, final_states=True), (len(a), len(b), len(c), plan)


def test_literal_lap_batch_and_go_below_ge(gpu, orc, monkeypatch):
    """A batch of ragged cubes in one literal lap launch (columns of several
    triples) through the async entry point, and a parameter set the factored
    form cannot run (GO < GE), whose AUTO plan is then the literal lap."""
    import torch
    rng = np.random.default_rng(77)
    triples = [tuple(rng.integers(0, 5, int(rng.integers(20, 160))).astype(np.uint8) for _ in range(3))
               for _ in range(5)]
    p, op = gpu.TsaParams.default(score_bits=9), orc.default_params(score_bits=9)
    ml = [max(len(t[k]) for t in triples) for k in range(3)]
    monkeypatch.setenv("TSA_PENCIL_MODE", "litlap")
    assert gpu.describe_plan(len(triples), *ml, p, kernel="plane").startswith("plane literal-lap")
    seqs, offs = gpu.pack_batch(triples)
    ws = gpu.workspace_size(len(triples), *ml, p, "plane")
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_sc = torch.zeros(len(triples), dtype=torch.int32, device="cuda")
    d_ws = torch.zeros(max(ws, 16), dtype=torch.uint8, device="cuda")
    gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), len(triples), *ml, d_sc.data_ptr(),
                          d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, p, "plane")
    torch.cuda.synchronize()
    assert np.array_equal(d_sc.cpu().numpy(), orc.score_batch(seqs, offs, op, nthreads=8))
    monkeypatch.delenv("TSA_PENCIL_MODE")
    kw = dict(gap_open=1, gap_extend=2, score_bits=12)
    p2, o2 = gpu.TsaParams.default(**kw), orc.default_params(**kw)
    a, b, c = (rng.integers(0, 4, 256).astype(np.uint8) for _ in range(3))
    assert gpu.describe_plan(1, 256, 256, 256, p2, kernel="auto", sync=True).startswith("plane literal-lap")
    assert gpu.score(a, b, c, p2) == orc.score(a, b, c, o2)


def test_literal_lap_1024_rtl_words(gpu, orc, synth):
    """configs[3]'s 1024^3 cube in the RTL's literal 12-bit arithmetic on the
    literal lap (kernel=plane): the score and final 7-tuple equal the
    oracle's, with no lap fallback."""
    a, b, c = synth.triple(3, 1024)
    p, op = gpu.TsaParams.default(score_bits=12), orc.default_params(score_bits=12)
    plan = gpu.describe_plan(1, 1024, 1024, 1024, p, kernel="plane", sync=True)
    assert plan.startswith("plane literal-lap"), plan
    before = gpu.fallback_count()
    s, fin = gpu.score(a, b, c, p, kernel="plane", final_states=True)
    assert (s, tuple(fin)) == orc.score(a, b, c, op, final_states=True)
    assert gpu.fallback_count() == before


@pytest.mark.parametrize("kernel,mode", [("pencil", "lap"), ("plane", "litlap")])
def test_lap_chunked_batch(gpu, orc, monkeypatch, kernel, mode):
    """A batch run as several lap launches of a few triples each, one after
    another on the stream (lap_geom_chunked; TSA_LAP_CHUNK forces 3): the
    last, smaller chunk on its own geometry inside the batch's workspace,
    the factored and the literal form, async path -- every score the oracle's."""
    import torch
    monkeypatch.setenv("TSA_PENCIL_MODE", mode)
    monkeypatch.setenv("TSA_LAP_CHUNK", "3")
    rng = np.random.default_rng(91 if kernel == "pencil" else 92)
    triples = [tuple(rng.integers(0, 5, int(rng.integers(lo, hi))).astype(np.uint8) for lo, hi in
                     ((40, 150), (17, 45), (65, 140))) for _ in range(8)]
    p, op = gpu.TsaParams.default(score_bits=12), orc.default_params(score_bits=12)
    ml = [max(len(t[k]) for t in triples) for k in range(3)]
    plan = gpu.describe_plan(len(triples), *ml, p, kernel=kernel, sync=False)
    assert " lap" in plan and "literal-lap" in plan if kernel == "plane" else " lap " in plan
    assert "chunk=3" in plan, plan
    seqs, offs = gpu.pack_batch(triples)
    ws = gpu.workspace_size(len(triples), *ml, p, kernel)
    d_seqs, d_offs = torch.from_numpy(seqs).cuda(), torch.from_numpy(offs).cuda()
    d_sc = torch.full((len(triples),), -7, dtype=torch.int32, device="cuda")
    d_ws = torch.zeros(max(ws, 16), dtype=torch.uint8, device="cuda")
    for _ in range(2):  # a second pass over the same workspace: new epochs, stale rings ignored
        gpu.score_batch_async(d_seqs.data_ptr(), d_offs.data_ptr(), len(triples), *ml, d_sc.data_ptr(),
                              d_ws.data_ptr(), ws, torch.cuda.current_stream().cuda_stream, p, kernel)
        torch.cuda.synchronize()
        assert np.array_equal(d_sc.cpu().numpy(), orc.score_batch(seqs, offs, op, nthreads=8)), plan
