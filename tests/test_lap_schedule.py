"""The single-cube lap kernel's schedule (csrc/lap_kernel.hip) replayed on the
CPU by tools/lap_emu.py -- two DP rows per wave in the 16-bit halves, laps of
2*NW rows chained through tagged y records, z-tiles of 64*M positions chained
through z records -- must reproduce the oracle exactly, including the tile and
lap seams the adversarial inputs stress (all-mismatch and all-match cubes)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from lap_emu import emulate  # noqa: E402

CASES = [((20, 11, 70), 2, 1), ((5, 3, 1), 2, 1), ((1, 1, 1), 2, 1), ((30, 9, 130), 2, 2),
         ((7, 17, 64), 4, 1), ((40, 4, 65), 2, 1), ((50, 8, 129), 4, 2), ((12, 13, 300), 2, 4),
         # the seam cell (1, y, 64M+1) of a deep cube: its step-0 inputs come from the
         # left tile's records ZT-2 / ZT-1 (all-mismatch exposes a face value there)
         ((10, 20, 66), 2, 1), ((20, 40, 70), 2, 1), ((16, 24, 130), 4, 2)]


@pytest.mark.parametrize("sk", [1, 2])
@pytest.mark.parametrize("shape,nw,m", CASES)
@pytest.mark.parametrize("kind", ["random", "mismatch", "match"])
def test_lap_schedule_vs_oracle(orc, shape, nw, m, kind, sk):
    la, lb, lc = shape
    rng = np.random.default_rng(la * 7 + lb * 3 + lc)
    if kind == "random":
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in shape)
    elif kind == "mismatch":
        a, b, c = (np.full(n, v, np.uint8) for n, v in zip(shape, (0, 1, 2)))
    else:
        a, b, c = (np.zeros(n, np.uint8) for n in shape)
    sop = bool(rng.integers(0, 2))
    op = orc.default_params(score_bits=16, s3_mode=int(sop))
    assert emulate(a, b, c, sop=sop, NW=nw, M=m, SK=sk) == orc.score(a, b, c, op)


@pytest.mark.parametrize("shape,nw,m", CASES)
@pytest.mark.parametrize("kind", ["random", "mismatch", "match", "related"])
def test_lap_schedule_vspace_vs_oracle(orc, shape, nw, m, kind):
    """The V-space lap (lap_kernel VS, the f16 cell of the RTL constants):
    values shifted by lam (x+y+z), the x = 0 face injected as lam q at x = 1,
    lap 0's y = 0 and tile 0's z = 0 records written as lam q face values --
    the same score as the oracle over laps, tiles, NW and M (the homopolymer
    and related cubes exercise every face)."""
    la, lb, lc = shape
    rng = np.random.default_rng(la * 5 + lb * 11 + lc)
    if kind == "random":
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in shape)
    elif kind == "mismatch":
        a, b, c = (np.full(n, v, np.uint8) for n, v in zip(shape, (0, 1, 2)))
    elif kind == "match":
        a, b, c = (np.zeros(n, np.uint8) for n in shape)
    else:
        base = rng.integers(0, 4, max(shape)).astype(np.uint8)
        a, b, c = (base[:n].copy() for n in shape)
        b[::5] = (b[::5] + 1) & 3
    sop = bool(rng.integers(0, 2))
    op = orc.default_params(score_bits=16, s3_mode=int(sop))
    assert emulate(a, b, c, sop=sop, NW=nw, M=m, vs=True) == orc.score(a, b, c, op)


def test_lap_vspace_split_cell_algebra():
    """csrc/lap_kernel.hip:lap_pre_vs / lap_post_vs (the V-space cell split at
    the row above) equal cell_messages_vs (pencil_common.h) for any inputs,
    GO >= GE and lam = GE = -MISMATCH (DO = GO - GE >= 0, CP = GO >= lam)."""
    from lap_emu import vs_cell
    rng = np.random.default_rng(11)
    for _ in range(20000):
        lam = int(rng.integers(1, 5))
        go = int(rng.integers(lam, 9))
        cP, dO = go - lam + lam, go - lam
        X, Y, Z, XY, XZ, YZ, Mv = (int(v) for v in rng.integers(-40, 40, 7))
        Gx, Gy, Gz = max(Y, Z, YZ), max(X, Z, XZ), max(X, Y, XY)
        best = max(Gx, Gy, XY, Mv)
        b1 = best - dO
        pxy, pyz, pxz = max(Gz, b1), max(Gx, b1), max(Gy, b1)
        qxy, qyz, qxz = pxy - cP, pyz - cP, pxz - cP
        ref = (best, max(X - lam, qxy, qxz), max(Y - lam, qxy, qyz), max(Z - lam, qyz, qxz), pxy, pyz, pxz)
        got = tuple(int(v) for v in vs_cell(*(np.int64(v) for v in (X, Y, Z, XY, YZ, XZ, Mv)), lam, cP, dO))
        assert got == ref


def test_lap_split_cell_algebra():
    """csrc/lap_kernel.hip:lap_pre_*/lap_post_* fold every message to
    max(Y - c, N) with the N's independent of the row above (Y = Iy's input);
    with GO >= GE that equals the grouped message form of cell_messages_f16
    (pencil_common.h) for any inputs -- checked exhaustively over a random
    sample of integer inputs, penalties and folded mismatch."""
    rng = np.random.default_rng(7)
    for _ in range(20000):
        ge = int(rng.integers(0, 7))
        go = int(rng.integers(ge, 10))
        mm = int(rng.integers(-3, 2))
        E, O, E2, OE, O2 = ge - mm, go - mm, 2 * ge, go + ge, 2 * go
        X, Y, Z, XY, XZ, YZ, Mv = (int(v) for v in rng.integers(-40, 40, 7))
        S3 = max(X, Y, Z)
        A1, A2, A3 = max(S3, XY, XZ), max(S3, YZ, XY), max(YZ, XZ, S3)
        C1, C2, C3 = max(X, XY, Y), max(Y, YZ, Z), max(Z, XZ, X)
        best = max(A1, YZ, Mv)
        ref = (best, max(X - E2, A1 - OE, best - O2), max(Y - E2, A2 - OE, best - O2),
               max(Z - E2, A3 - OE, best - O2), max(C1 - E, best - O), max(C2 - E, best - O),
               max(C3 - E, best - O))
        pXZ = max(X, Z)
        U1, U2, U3 = max(pXZ, XY, XZ), max(pXZ, XY, YZ), max(pXZ, YZ, XZ)
        W = max(U1, YZ, Mv)
        N = (max(X - E2, U1 - OE, W - O2), max(U2 - OE, W - O2), max(Z - E2, U3 - OE, W - O2),
             max(max(X, XY) - E, W - O), max(max(YZ, Z) - E, W - O), max(max(pXZ, XZ) - E, W - O))
        got = (max(Y, W), max(Y - OE, N[0]), max(Y - E2, N[1]), max(Y - OE, N[2]),
               max(Y - E, N[3]), max(Y - E, N[4]), max(Y - O, N[5]))
        assert got == ref


@pytest.mark.parametrize("shape,kw", [((20, 11, 70), {}), ((25, 17, 33), {"sop": True}),
                                      ((30, 20, 40), {"bits": 5}), ((40, 19, 70), {"NW": 4}),
                                      ((20, 9, 150), {"M": 2}), ((12, 30, 5), {"NW": 8})])
def test_literal_lap_schedule_matches_oracle(orc, shape, kw):
    """tools/litlap_emu.py: the lap schedule with the literal push-form cell
    (x' = 0 face column, step-varying y = 0 / z = 0 faces of zero cells,
    successor symbols, wrapped candidates) equals the literal oracle, final
    7-tuple included, over laps, tiles, NW and M."""
    import litlap_emu
    rng = np.random.default_rng(sum(shape))
    a, b, c = (rng.integers(0, 5, n) for n in shape)
    got = litlap_emu.emulate(a, b, c, **kw)
    p = orc.default_params(s3_mode=int(kw.get("sop", False)), score_bits=kw.get("bits", 12))
    s, fin = orc.score(a, b, c, p, final_states=True)
    assert (got[0], tuple(got[1])) == (s, tuple(fin))
