#!/usr/bin/env python3
"""CPU replay of the single-cube lap kernel's schedule (csrc/lap_kernel.hip).

TEST/DESIGN INFRASTRUCTURE: this is how the kernel's index and timing logic is
checked before it runs on a GPU (tests/test_lap_schedule.py). It executes the
kernel's dataflow register by register -- the same positions, halves, record
hand-offs, z-shifts, x = 1 injections, A-table offsets and final-cell capture
-- with exact integer arithmetic in the message form, and must reproduce the
oracle's score.

Layout (one workgroup = one (lap L, z-tile q) of a triple):
  * NW waves; wave w holds DP rows y = L*RW + 2w + 1 (low 16-bit half) and
    2w + 2 (high half), RW = 2*NW rows per lap;
  * lane l, register i is tile position k = M*l + i, z = q*ZT + k + 1, ZT = 64*M;
  * at local step t the position (k) of half h of wave w computes
    x = u + 1 with u = t - (2w + h) - k (one step of skew per row and per z);
  * the row above of the low half is wave w-1's high half (wave 0: the
    previous lap's last wave, record t + RW - 1; lap 0: the y = 0 face), the
    row above of the high half is the wave's own low half one step earlier:
    REC = {above.hi -> lo, own_prev.lo -> hi} per record word;
  * z-1 neighbours: registers shift up one position per step; position 0
    takes the previous tile's last position, record t + ZT of that tile.
"""
from __future__ import annotations

import numpy as np

NEG = -(1 << 40)


def penalties(go, ge):
    GO2, GE2, GOGE = 2 * go, 2 * ge, go + ge
    return np.array([[0, 0, 0, 0, 0, 0, 0],
                     [GO2, GE2, GOGE, GOGE, GOGE, GO2, GOGE],
                     [GO2, GOGE, GE2, GOGE, GOGE, GOGE, GO2],
                     [GO2, GOGE, GOGE, GE2, GO2, GOGE, GOGE],
                     [go, ge, ge, go, ge, go, go],
                     [go, go, ge, ge, go, ge, go],
                     [go, ge, go, ge, go, go, ge]], dtype=np.int64)


def codes(seq, n):
    """One-hot codes (1 << s), 0 beyond the sequence (padding)."""
    out = np.zeros(n, np.int64)
    s = np.asarray(seq, np.int64)[:n] & 3
    out[: len(s)] = 1 << s
    return out


def vs_cell(X, Y, Z, XY, YZ, XZ, Mv, lam, cP, dO):
    """lap_kernel.hip's V-space cell split at the row above (lap_pre_vs before
    Y lands, lap_post_vs after): inputs with their pair / triple scores added,
    returns (best, Ix', Iy', Iz', Ixy', Iyz', Ixz')."""
    gx, gz, Gy = np.maximum(Z, YZ), np.maximum(X, XY), np.maximum(np.maximum(X, Z), XZ)
    W = np.maximum(np.maximum(gx, Gy), np.maximum(XY, Mv))
    WD = W - dO
    NXY, NYZ, NXZ = np.maximum(gz, WD), np.maximum(gx, WD), np.maximum(Gy, WD)
    N1 = np.maximum(np.maximum(X - lam, NXY - cP), NXZ - cP)
    N2 = np.maximum(NXY - cP, NYZ - cP)
    N3 = np.maximum(np.maximum(Z - lam, NYZ - cP), NXZ - cP)
    return (np.maximum(Y, W), np.maximum(Y - cP, N1), np.maximum(Y - lam, N2), np.maximum(Y - cP, N3),
            np.maximum(Y, NXY), np.maximum(Y, NYZ), np.maximum(Y - dO, NXZ))


def emulate(a, b, c, match=1, mismatch=-1, go=2, ge=1, sop=False, NW=2, M=1, SK=1, cells=None, vs=False):
    """Score of one triple by the lap schedule (no wrap: valid where the
    factored form is exact). vs: the V-space cell (lap_kernel VS: values
    shifted by lam (x+y+z), lam = GE = -MISMATCH) with its face values --
    x = 1 injection, lap 0's y = 0 records, tile 0's z = 0 records."""
    lam = ge if vs else 0
    assert not vs or ge == -mismatch
    cP, dO, dm = go + mismatch + lam, go - ge, match - mismatch
    la, lb, lc = len(a), len(b), len(c)
    P = penalties(go, ge)
    RW, ZT = 2 * NW, 64 * M
    G, GZ = -(-lb // RW), -(-lc // ZT)
    f_single = -int(P[1].min())
    f_pair = -int(P[4].min())
    face = (f_single, f_pair, f_pair, 0)          # y = 0 face record {Iy, Ixy, Iyz, best}
    s3_ne = 3 * mismatch
    s3_ab = 2 * (match + mismatch)                # src/PE_1cyc.v:162 precedence
    s3_eq = 3 * match
    # SK: steps between a wave's high row and the next wave's low row (the
    # kernel reads the wave above's record SK steps old); wave w's rows sit at
    # step offsets WO*w (low half) and WO*w + 1 (high half), WO = SK + 1
    WO = SK + 1
    tau = lambda r: WO * (r >> 1) + (r & 1)
    YOFF = WO * (NW - 1) + 1           # lap L+1 step t reads lap L's record t + YOFF
    # A table: entry j holds x = j - OFF (lo) and x = j - OFF - 1 (hi)
    OFF = WO * NW + ZT
    yrec = {}   # (L, q) -> list over steps of 4 arrays [M, 64, 2] (last wave's out record)
    zrec = {}   # (L, q) -> list over steps of [NW][4] pairs (lane 63, reg M-1)
    score = None
    lanes = np.arange(64)
    for L in range(G):
        for q in range(GZ):
            zt_q = min(ZT, lc - q * ZT)
            rows = min(RW, lb - L * RW)
            T = la + tau(rows - 1) + (zt_q - 1)       # last real cell of the WG at step T-1
            A = codes(a, la)
            Bc = codes(b, lb)
            Cc = codes(c, lc)
            # per position k: c code (both halves), per half h: b code of row 2w+h
            kpos = M * lanes[None, :] + np.arange(M)[:, None]      # [M, 64]
            zc = q * ZT + kpos
            cpos = np.where(zc < lc, Cc[np.minimum(zc, lc - 1)], 0)
            # state per wave: [M, 64, 2] arrays
            shape = (NW, M, 64, 2)
            oIx = np.full(shape, f_single, np.int64)
            shIz = np.full(shape, f_single, np.int64)
            svIxy = np.full(shape, f_pair, np.int64)
            svIyz = np.full(shape, f_pair, np.int64)
            shIxz = np.full((2,) + shape, f_pair, np.int64)
            svM = np.zeros((2,) + shape, np.int64)
            own_prev = np.zeros((4,) + shape, np.int64)
            out_prev = np.zeros((4,) + shape, np.int64)    # wave w's record of step t-1
            if q == 0 and vs:  # tile 0: the face records of steps -1 and -2 (zface_vs)
                for w in range(NW):
                    for tt, ph in ((-1, 1), (-2, 0)):
                        g1, g2 = lam * (tt + L * RW + 2), lam * (tt + L * RW + 3)
                        if tt == -1:
                            shIz[w, 0, 0] = g1
                            svIyz[w, 0, 0] = g1
                        shIxz[ph, w, 0, 0] = g2
                        svM[ph, w, 0, 0] = g1
            if q > 0:
                # position 0 before step 0: the shifts of steps -2 and -1 would have
                # brought in the left tile's records ZT-2 and ZT-1 (Iz, Iyz feed the
                # next step, Ixz, M the one after: PH slots 0 and 1)
                left = zrec[(L, q - 1)]
                for w in range(NW):
                    r1, r2 = left[ZT - 1][w], left[ZT - 2][w]
                    shIz[w, 0, 0] = r1[0]
                    svIyz[w, 0, 0] = r1[2]
                    shIxz[1, w, 0, 0] = r1[1]
                    svM[1, w, 0, 0] = r1[3]
                    shIxz[0, w, 0, 0] = r2[1]
                    svM[0, w, 0, 0] = r2[3]
            ys, zs = [], []
            out_hist = []
            for t in range(T):
                PH = t & 1
                out_now = np.zeros_like(out_prev)
                zstep = [None] * NW
                for w in range(NW):
                    # A codes: lo u = t - 2w - k, hi u - 1 (table entry j = u + OFF)
                    j = t - WO * w - kpos + OFF
                    ulo = j - OFF
                    alo = np.where((ulo >= 0) & (ulo < la), A[np.clip(ulo, 0, la - 1)], 0)
                    ahi = np.where((ulo - 1 >= 0) & (ulo - 1 < la), A[np.clip(ulo - 1, 0, la - 1)], 0)
                    acode = np.stack([alo, ahi], -1)
                    rowi = L * RW + 2 * w + np.arange(2)
                    bcode = np.where(rowi < lb, Bc[np.minimum(rowi, lb - 1)], 0)[None, None, :]
                    ccode = cpos[:, :, None]
                    # ---- the row above
                    if w == 0:
                        if L == 0:
                            fc = face
                            if vs:  # the loader's yface_vs(t): zoff = q ZT
                                fc = (lam * (t + q * ZT + 1),) + (lam * (t + q * ZT + 2),) * 3
                            above = np.array(fc, np.int64)[:, None, None, None] * np.ones((4, M, 64, 2), np.int64)
                        else:
                            prev = yrec[(L - 1, q)]
                            r = t + YOFF
                            above = prev[min(r, len(prev) - 1)]
                    else:  # the record wave w-1 wrote SK steps ago
                        above = out_hist[t - SK][:, w - 1] if t >= SK else np.zeros((4, M, 64, 2), np.int64)
                    REC = np.empty((4, M, 64, 2), np.int64)
                    REC[..., 0] = above[..., 1]
                    REC[..., 1] = own_prev[:, w][..., 0]
                    inIx = oIx[w].copy()
                    inIy = REC[0].copy()
                    inIz = shIz[w].copy()
                    inIxy = svIxy[w].copy()
                    inIyz = svIyz[w].copy()
                    inIxz = shIxz[PH, w].copy()
                    inM = svM[PH, w].copy()
                    # ---- x = 1 injection (u == 0)
                    u = np.stack([ulo, ulo - 1], -1) * np.ones((M, 64, 2), np.int64)
                    inj = u == 0
                    if vs:  # lam (t + L RW + zoff + 1) for both halves; M one lam less
                        hx = lam * (t + L * RW + q * ZT + 1)
                        inIx[inj], inIxy[inj], inIxz[inj], inM[inj] = hx, hx, hx, hx - lam
                    else:
                        inIx[inj] = f_single
                        inIxy[inj] = f_pair
                        inIxz[inj] = f_pair
                        inM[inj] = 0
                    # ---- scores (one-hot codes; 0 = padding never matches)
                    eab = (acode & bcode) != 0
                    eac = (acode & ccode) != 0
                    ebc = (bcode & ccode) != 0
                    s2 = lambda e: np.where(e, match, mismatch)
                    if sop:
                        s3 = s2(eab) + s2(ebc) + s2(eac)
                    else:
                        s3 = np.where(eab, np.where(ebc, s3_eq, s3_ab), s3_ne)
                    if vs:  # the kernel's V-space inputs: pair scores as dm [match], M's + 3 lam = 0 (RTL)
                        if sop:
                            Mv = inM + s3 + 3 * lam
                        else:
                            Mv = inM + np.where(eab, np.where(ebc, s3_eq, s3_ab) - s3_ne, 0) + s3_ne + 3 * lam
                        S = np.stack([Mv, inIx, inIy, inIz, inIxy + dm * eab, inIyz + dm * ebc, inIxz + dm * eac])
                        msg = np.stack(vs_cell(inIx, inIy, inIz, S[4], S[5], S[6], Mv, lam, cP, dO))
                    else:
                        S = np.stack([inM + s3, inIx, inIy, inIz, inIxy + s2(eab), inIyz + s2(ebc),
                                      inIxz + s2(eac)])
                        msg = np.stack([(S - P[T_][:, None, None, None]).max(0) for T_ in range(7)])
                    if cells is not None:  # debugging: the 7 states of every real cell
                        for i in range(M):
                            for l in range(64):
                                for h in range(2):
                                    x, y, z = int(u[i, l, h]) + 1, L * RW + 2 * w + h + 1, q * ZT + M * l + i + 1
                                    if 1 <= x <= la and y <= lb and z <= lc:
                                        cells[(x, y, z)] = S[:, i, l, h].copy()
                    best = msg[0]
                    nIx, oIy, oIz, oIxy, oIyz, oIxz = msg[1], msg[2], msg[3], msg[4], msg[5], msg[6]
                    out = np.stack([oIy, oIxy, oIyz, best])
                    out_now[:, w] = out
                    own_prev[:, w] = out
                    # ---- final cell (la, lb, lc)
                    if L == G - 1 and q == GZ - 1:
                        rf = (lb - 1) - L * RW
                        kf = (lc - 1) - q * ZT
                        if rf // 2 == w and t == (la - 1) + tau(rf) + kf:
                            score = int(best[kf % M, kf // M, rf % 2]) - lam * (la + lb + lc)
                    # ---- z staging: lane 63, register M-1
                    zstep[w] = (oIz[M - 1, 63].copy(), oIxz[M - 1, 63].copy(),
                                REC[2][M - 1, 63].copy(), REC[3][M - 1, 63].copy())
                    # ---- advance
                    oIx[w] = nIx
                    svIxy[w] = REC[1]
                    if q > 0:
                        left = zrec[(L, q - 1)]
                        rz = t + ZT
                        fz = left[min(rz, len(left) - 1)][w]
                    elif vs:  # the loader's zface_vs(t + ZT)
                        g1, g2 = lam * (t + L * RW + 2), lam * (t + L * RW + 3)
                        fz = (np.array([g1] * 2), np.array([g2] * 2), np.array([g1] * 2), np.array([g1] * 2))
                    else:
                        fz = (np.array([f_single] * 2), np.array([f_pair] * 2),
                              np.array([f_pair] * 2), np.array([0, 0]))

                    def zshift(src, f):
                        v = np.empty_like(src)
                        v[1:] = src[:-1]
                        v[0, 1:] = src[M - 1, :-1]
                        v[0, 0] = f
                        return v
                    shIz[w] = zshift(oIz, fz[0])
                    shIxz[PH, w] = zshift(oIxz, fz[1])
                    svIyz[w] = zshift(REC[2], fz[2])
                    svM[PH, w] = zshift(REC[3], fz[3])
                out_prev = out_now
                out_hist.append(out_now)
                ys.append(out_now[:, NW - 1].copy())
                zs.append(zstep)
            yrec[(L, q)] = ys
            zrec[(L, q)] = zs
    return score


if __name__ == "__main__":
    import sys
    rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
    a, b, c = (rng.integers(0, 4, n) for n in (20, 11, 70))
    print(emulate(a, b, c, NW=2, M=1))
