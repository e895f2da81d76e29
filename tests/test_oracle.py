"""CPU oracle checks: the restatement against the reference-derived known
answers, the cycle-level RTL model, its own second traversal, and the
properties SURVEY.md 4 lists. TEST INFRASTRUCTURE ONLY (no product code)."""
import numpy as np
import pytest


def test_golden_fixtures(orc, golden):
    for c in golden:
        p = orc.default_params(**c["params"])
        s, fin = orc.score(c["a"], c["b"], c["c"], p, final_states=True)
        assert s == c["score"], c["name"]
        assert list(fin) == c["final7"], c["name"]
        assert orc.score(c["a"], c["b"], c["c"], p, method="diag") == c["score"], c["name"]


def test_testbench_known_answer(orc):
    # src/TriAlign_tb.sv:423-1960 loads all-A; every M step is +3, nothing else
    # is positive, so the 64^3 score is 3*64 (KAT 1).
    z = [0] * 64
    assert orc.score(z, z, z) == 192
    for n in (8, 16, 32, 48):
        assert orc.score([0] * n, [0] * n, [0] * n) == 3 * n


def test_dat_triple_and_survey_values(golden):
    by = {c["name"]: c for c in golden}
    assert by["dat"]["score"] == 1
    assert by["dat"]["final7"] == [-1, 1, -4, -5, 1, -7, -2]
    assert by["dat_prefix8"]["score"] == -3 and by["dat_prefix16"]["score"] == -5
    assert by["homopolymers_16"]["score"] == -32
    assert by["dat"]["rtl_model"]["score"] == 1


@pytest.mark.parametrize("seed", range(6))
def test_rtl_model_matches_restatement_in_envelope(orc, seed):
    rng = np.random.default_rng(seed)
    for _ in range(4):
        la = 8 * int(rng.integers(1, 9)); lb = 8 * int(rng.integers(1, la // 8 + 1)); lc = 8 * int(rng.integers(1, 9))
        a, b, c = (rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc))
        r, isx, _ = orc.rtl_run(a, b, c)
        assert not isx
        assert r == orc.score(a, b, c)


def test_rtl_model_long_pencil_ring(orc):
    # 128 x 64 x 40: 8 x 5 pencils, y-face ring wraps several times
    rng = np.random.default_rng(7)
    a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (128, 64, 40))
    r, isx, cyc = orc.rtl_run(a, b, c)
    assert not isx and r == orc.score(a, b, c)
    # cycle model of SURVEY.md 3(c), 1cyc controller: per pencil 65 load + LA+16 compute
    assert cyc == (64 // 8) * (40 // 8) * (65 + 128 + 16) + 1


def test_rtl2_model_testbench_and_dat(orc, golden):
    """The 2-cycle variant (oracle/rtl_model_2cyc.c) on the testbench's own
    input and the reference's dat triple: the same scores as the 1-cycle
    variant and the restatement."""
    z = [0] * 64
    r, isx, cyc = orc.rtl2_run(z, z, z)
    assert (r, isx) == (192, False)
    # per pencil 65 INITIAL clocks, then a COMPUTE + WAIT pair per step for
    # A_idx + 16 steps (src/TriAlign_2cyc.v:354-355,433-482)
    assert cyc == 64 * (65 + 2 * (64 + 16)) + 1
    by = {c["name"]: c for c in golden}
    assert by["dat"]["rtl2_model"] == {"score": 1, "x": False, "cycles": cyc, "agrees": True,
                                       "source": by["dat"]["rtl2_model"]["source"]}
    assert by["dat"]["rtl2_model"]["source"].startswith("model-derived")


def test_golden_rtl2_records(orc, golden, tsa):
    """golden.json records, for every default-parameter case the 2-cycle RTL
    can take, its model's score and whether it agrees with the restatement;
    agreement is exactly the 2-cycle envelope (rtl_envelope(variant="2cyc"))."""
    seen = 0
    for c in golden:
        r = c.get("rtl2_model")
        if r is None:
            continue
        seen += 1
        la, lb, lc = len(c["a"]), len(c["b"]), len(c["c"])
        assert r["agrees"] == ((not r["x"]) and r["score"] == c["score"]), c["name"]
        assert r["agrees"] == tsa.rtl_envelope(la, lb, lc, variant="2cyc"), c["name"]
        if la * lb * lc <= 64 ** 3:
            s, isx, cyc = orc.rtl2_run(c["a"], c["b"], c["c"])
            assert (s, isx, cyc) == (r["score"], r["x"], r["cycles"]), c["name"]
    assert seen >= 30


RTL2_SHAPES = [(n, n, n) for n in range(8, 137, 8)] + [
    (64, 32, 64), (64, 64, 32), (64, 64, 8), (32, 64, 8), (128, 64, 64), (64, 64, 128),
    (48, 48, 96), (96, 96, 16), (40, 40, 80)]


def test_rtl2_envelope_is_where_the_model_agrees(orc, tsa):
    """The 2-cycle variant's y-face store (3 groups x 2 x 8 SRAMs, group and
    page from index bits shared with B_idx, src/TriAlign_2cyc.v:85-92,141-157,
    176-180) only carries every face to its reader for some shapes: LB = LA
    (or a single z pencil), and no bank shared by a pencil's write, read and
    corner slots -- 8, 16, 40, 48, 64, 128 cubes here; 24, 32, 56, 72-120,
    136 cubes and LB != LA come back X or wrong. The host-side rule
    (_rtl2_ring_ok) is checked against the clocked model on every shape."""
    for la, lb, lc in RTL2_SHAPES:
        agree = []
        for seed in range(3):
            rng = np.random.default_rng(seed)
            a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
            s, isx, _ = orc.rtl2_run(a, b, c)
            agree.append((not isx) and s == orc.score(a, b, c))
        want = tsa.rtl_envelope(la, lb, lc, variant="2cyc")
        assert (all(agree) if want else not all(agree)), ((la, lb, lc), agree, want)
    assert tsa.rtl_envelope(64, 64, 64, variant="2cyc") and tsa.rtl_envelope(256, 256, 256, variant="2cyc")
    assert not tsa.rtl_envelope(96, 96, 96, variant="2cyc") and tsa.rtl_envelope(96, 96, 96)


def test_factored_form_equals_literal(orc):
    rng = np.random.default_rng(11)
    for k in range(40):
        la, lb, lc = (int(v) for v in rng.integers(1, 30, 3))
        a, b, c = (rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc))
        p = orc.default_params(s3_mode=k % 2, score_bits=0)
        assert orc.score(a, b, c, p, method="msg") == orc.score(a, b, c, p)


def test_ab_symmetry_rtl_s3(orc):
    # penalty table is x<->y symmetric and RTL s3 is a<->b symmetric
    rng = np.random.default_rng(3)
    for _ in range(20):
        la, lb, lc = (int(v) for v in rng.integers(1, 20, 3))
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        assert orc.score(a, b, c) == orc.score(b, a, c)


def test_sop_full_permutation_invariance(orc):
    import itertools
    rng = np.random.default_rng(5)
    p = orc.default_params(s3_mode=1)
    for _ in range(8):
        seqs = [rng.integers(0, 4, int(n)).astype(np.uint8) for n in rng.integers(1, 16, 3)]
        ref = orc.score(*seqs, p)
        for perm in itertools.permutations(range(3)):
            assert orc.score(*(seqs[i] for i in perm), p) == ref


def test_rtl_s3_quirk_differs_from_sop(orc):
    # a==b!=c scores 0 in the RTL (src/PE_1cyc.v:162) but -1 as sum of pairs
    a, b, c = [0], [0], [1]
    _, fin = orc.score(a, b, c, orc.default_params(score_bits=0), final_states=True)
    assert fin[0] == 0  # M = 0 + s3
    _, fin = orc.score(a, b, c, orc.default_params(s3_mode=1, score_bits=0), final_states=True)
    assert fin[0] == -1


def test_wrap_changes_result_only_when_range_exceeded(orc):
    z = [0] * 48
    assert orc.score(z, z, z, orc.default_params(score_bits=0)) == 144
    assert orc.score(z, z, z, orc.default_params(score_bits=12)) == 144
    assert orc.score(z, z, z, orc.default_params(score_bits=8)) != 144  # 144 > 127 wraps


def test_state_range_small_for_random(orc):
    rng = np.random.default_rng(9)
    a, b, c = (rng.integers(0, 4, 64).astype(np.uint8) for _ in range(3))
    lo, hi = orc.state_range(a, b, c)
    assert -40 < lo <= 0 <= hi < 40


def test_generator_matches_python(orc, synth):
    for seed in (synth.SEED_BASE, synth.SEED_BASE + 5, 12345):
        for n in (1, 31, 32, 33, 257):
            assert np.array_equal(orc.gen_uniform(seed, n), synth.gen_uniform(seed, n))


def test_batch_threads(orc, synth):
    seqs, offs = synth.batch(0, 6, 20, 17, 23)
    s1 = orc.score_batch(seqs, offs, nthreads=1)
    s3 = orc.score_batch(seqs, offs, nthreads=3)
    assert np.array_equal(s1, s3)
    for i in range(6):
        o = offs[3 * i:3 * i + 4]
        assert s1[i] == orc.score(seqs[o[0]:o[1]], seqs[o[1]:o[2]], seqs[o[2]:o[3]])
