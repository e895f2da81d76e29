"""The helix kernel's schedule (positions, the two-step wave skew, LDS record
slots, the wave-0 ring with its face rows, x = 1 injection, z-shifts, TWO mode)
replayed on CPU by tools/pencil_emu.py must reproduce the oracle, in the
message form and in the V-space form (values shifted by lam*(x+y+z), faces
injected as lam*q). Guards the algorithm independently of the GPU."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("vs", [False, True])
@pytest.mark.parametrize("la,lb,lc,sop", [(64, 20, 64, 0), (47, 17, 128, 1), (60, 1, 65, 0),
                                          (130, 12, 200, 0), (5, 19, 3, 1), (300, 3, 40, 0),
                                          (8, 8, 8, 0)])
def test_emulated_schedule_matches_oracle(orc, la, lb, lc, sop, vs):
    import pencil_emu
    rng = np.random.default_rng(la * 1000 + lb * 10 + lc)
    a, b, c = (rng.integers(0, 5, n) for n in (la, lb, lc))
    got = pencil_emu.emulate([(a, b, c)], sop=bool(sop), vs=vs)
    assert got == [orc.score(a, b, c, orc.default_params(s3_mode=sop, score_bits=0))]


@pytest.mark.parametrize("vs", [False, True])
def test_emulated_two_triples(orc, vs):
    """TWO mode (LC <= 64): the halves of every register score two triples of
    different lengths at the same positions."""
    rng = np.random.default_rng(3)
    t1 = tuple(rng.integers(0, 4, n) for n in (40, 13, 64))
    t2 = tuple(rng.integers(0, 4, n) for n in (70, 9, 30))
    import pencil_emu
    got = pencil_emu.emulate([t1, t2], vs=vs)
    p = orc.default_params(score_bits=0)
    assert got == [orc.score(*t1, p), orc.score(*t2, p)]


def test_emulated_vspace_lam2(orc):
    kw = dict(match=2, mismatch=-2, go=3, ge=2)
    import pencil_emu
    rng = np.random.default_rng(11)
    a, b, c = (rng.integers(0, 4, n) for n in (50, 11, 90))
    p = orc.default_params(score_bits=0, match=2, mismatch=-2, gap_open=3, gap_extend=2)
    assert pencil_emu.emulate([(a, b, c)], vs=True, **kw) == [orc.score(a, b, c, p)]


@pytest.mark.parametrize("la,lb,lc,sop,bits", [(8, 8, 8, 0, 12), (20, 9, 30, 0, 12), (47, 17, 128, 1, 12),
                                               (60, 3, 130, 0, 12), (30, 20, 40, 0, 5), (25, 17, 33, 1, 4),
                                               (4, 2, 260, 0, 6)])
def test_emulated_literal_helix(orc, la, lb, lc, sop, bits):
    """tools/literal_emu.py: the literal push form on the helix schedule (the
    x = 0 face column, row 0's pushes in the ring, the z = 0 pushes of a zero
    cell with position 0's own symbols) equals the literal oracle, final
    7-tuple included, also for words narrow enough to wrap."""
    import literal_emu
    rng = np.random.default_rng(la * 1000 + lb * 10 + lc)
    a, b, c = (rng.integers(0, 5, n) for n in (la, lb, lc))
    s, fin = literal_emu.emulate(a, b, c, sop=bool(sop), bits=bits)
    assert (s, tuple(fin)) == orc.score(a, b, c, orc.default_params(s3_mode=sop, score_bits=bits),
                                        final_states=True)


def test_emulated_related_triples(orc):
    """Related and homopolymer triples (long matching runs: the optimum leaves
    the z = 0 face at the very first steps) in the V-space and literal forms."""
    import literal_emu
    import pencil_emu
    rng = np.random.default_rng(1)
    for _ in range(60):
        L = int(rng.integers(2, 20))
        a = rng.integers(0, 4, L).astype(np.uint8)
        t = (a, a[: int(rng.integers(1, L + 1))].copy(), a[: int(rng.integers(1, L + 1))].copy())
        assert pencil_emu.emulate([t], vs=True) == [orc.score(*t, orc.default_params(score_bits=0))], t
        assert literal_emu.emulate(*t)[0] == orc.score(*t), t
