"""The helix kernel's shifted ("V-space") cell, replayed on the CPU.

The pencil kernels send messages max_s(S[s] - P[T][s]) (src/PE_1cyc.v:164-218)
between cells. The helix's canonical form stores every value of cell
(x, y, z) shifted by lam * (x + y + z) -- a potential, so every path into a
cell gains the same amount and no max changes -- with lam = (GE - MISMATCH)/2.
Then (pencil_common.h, cell_messages_vs):
  * the pair targets' extend penalty vanishes:  Ixy' = max(max(Ix, Iy, Ixy), best - (GO - GE)),
  * the single targets reuse the pair messages: Ix'  = max(Ix - (2 GE - lam),
                                                        max(Ixy', Ixz') - (GO + MISMATCH + lam)),
  * M adds no constant when 3 MISMATCH + 3 lam = 0 (the RTL constants),
  * a zero face cell at coordinate sum q sends q - (2 GE - lam) to a single
    target and q to a pair target and to M.
This replays that algebra cell by cell and checks it against the literal
oracle, for the RTL constants and for other parameter sets
whose lam is an integer.
"""
import numpy as np
import pytest


def vspace_score(A, B, C, match=1, mismatch=-1, GO=2, GE=1, sop=False):
    lam2 = GE - mismatch
    assert lam2 % 2 == 0, "lam must be an integer"
    lam = lam2 // 2
    la, lb, lc = len(A), len(B), len(C)
    dm = match - mismatch
    c3 = 3 * mismatch if not sop else None
    cM = None if sop else c3 + 3 * lam          # constant added to M (0 for the RTL constants)
    cS = 2 * GE - lam                           # single target: own-state extend
    cP = GO + mismatch + lam                    # single target from the pair messages
    dO = GO - GE                                # pair target: best - (GO - GE)
    # message arrays per cell: single (Ix, Iy, Iz), pair (Ixy, Iyz, Ixz), best
    NEG = None
    mIx = {}; mIy = {}; mIz = {}; mIxy = {}; mIyz = {}; mIxz = {}; mB = {}

    def face(x, y, z):
        return x == 0 or y == 0 or z == 0

    def get(tab, x, y, z, kind):
        if face(x, y, z):
            q = lam * (x + y + z)
            return q - cS if kind == "single" else q
        return tab[(x, y, z)]

    for x in range(1, la + 1):
        for y in range(1, lb + 1):
            for z in range(1, lc + 1):
                a, b, c = A[x - 1] & 3, B[y - 1] & 3, C[z - 1] & 3
                X = get(mIx, x - 1, y, z, "single")
                Y = get(mIy, x, y - 1, z, "single")
                Z = get(mIz, x, y, z - 1, "single")
                XY = get(mIxy, x - 1, y - 1, z, "pair") + (dm if a == b else 0)
                YZ = get(mIyz, x, y - 1, z - 1, "pair") + (dm if b == c else 0)
                XZ = get(mIxz, x - 1, y, z - 1, "pair") + (dm if a == c else 0)
                inM = get(mB, x - 1, y - 1, z - 1, "best")
                if sop:
                    s3 = (match if a == b else mismatch) + (match if b == c else mismatch) + \
                         (match if a == c else mismatch)
                    Mv = inM + s3 + 3 * lam
                else:
                    s3d = (3 * match if b == c else 2 * (match + mismatch)) - 3 * mismatch if a == b else 0
                    Mv = inM + s3d + cM
                Gx, Gy, Gz = max(Y, Z, YZ), max(X, Z, XZ), max(X, Y, XY)
                best = max(Gx, Gy, Gz, Mv)
                b1 = best - dO
                pxy, pyz, pxz = max(Gz, b1), max(Gx, b1), max(Gy, b1)
                mIxy[(x, y, z)], mIyz[(x, y, z)], mIxz[(x, y, z)] = pxy, pyz, pxz
                mIx[(x, y, z)] = max(X - cS, max(pxy, pxz) - cP)
                mIy[(x, y, z)] = max(Y - cS, max(pxy, pyz) - cP)
                mIz[(x, y, z)] = max(Z - cS, max(pyz, pxz) - cP)
                mB[(x, y, z)] = best
    return mB[(la, lb, lc)] - lam * (la + lb + lc)


@pytest.mark.parametrize("kw", [
    {},                                                    # RTL constants (lam = 1)
    dict(match=2, mismatch=-2, GO=3, GE=2),                 # lam = 2
    dict(match=1, mismatch=-3, GO=4, GE=1),                 # lam = 2, M constant != 0
    dict(match=3, mismatch=0, GO=2, GE=2),                  # lam = 1
    dict(sop=True),                                         # sum-of-pairs s3
])
def test_vspace_cell_matches_oracle(orc, kw):
    rng = np.random.default_rng(5)
    p = orc.default_params(score_bits=0, match=kw.get("match", 1), mismatch=kw.get("mismatch", -1),
                           gap_open=kw.get("GO", 2), gap_extend=kw.get("GE", 1),
                           s3_mode=1 if kw.get("sop") else 0)
    for _ in range(12):
        A, B, C = (rng.integers(0, 5, int(rng.integers(1, 9))).astype(np.uint8) for _ in range(3))
        assert vspace_score(list(A), list(B), list(C), **kw) == orc.score(A, B, C, p), kw
    same = np.zeros(7, np.uint8)
    assert vspace_score(list(same), list(same), list(same), **kw) == orc.score(same, same, same, p)
