#!/usr/bin/env python3
"""CPU replay of the LITERAL lap schedule (csrc/lap_kernel.hip, LIT): the
single-cube lap kernel's dataflow with the literal push-form cell of the
literal helix (tools/literal_emu.py, csrc/literal_kernel.hip).

TEST/DESIGN INFRASTRUCTURE (tests/test_lap_schedule.py). Same positions,
halves, record hand-offs and z-shifts as tools/lap_emu.py; what differs:
  * a position computes cell x' = u (not u + 1): x' = 0 is the x = 0 face,
    a cell whose 7 inputs are forced to 0 and whose pushes are the faces of
    x = 1 (one more step per workgroup);
  * the cell pushes to its successors with THEIR symbols: a[u] (= a_{x'+1},
    the same table entry the message form reads), b of the next row, c of
    the next z;
  * the y = 0 face (lap 0) and the z = 0 face (tile 0) are zero cells pushing
    with the receivers' symbols, so they vary with the step;
  * every candidate is wrapped to SCORE_BITS before its max (src/PE_1cyc.v:
    127-133); the final cell's 7 input states are captured.

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


def emulate(a, b, c, match=1, mismatch=-1, go=2, ge=1, sop=False, bits=12, NW=2, M=1, SK=1):
    """(score, final7) of one triple by the literal lap schedule."""
    la, lb, lc = len(a), len(b), len(c)
    P = penalties(go, ge)
    RW, ZT = 2 * NW, 64 * M
    G, GZ = -(-lb // RW), -(-lc // ZT)

    def wrap(v):
        if bits == 0:
            return v
        m = 1 << bits
        return ((v + (m >> 1)) % m) - (m >> 1)

    A, Bc, Cc = codes(a, la), codes(b, lb), codes(c, lc)

    def code_at(arr, n, idx):  # code of 0-based index idx (0 outside [0, n))
        idx = np.asarray(idx)
        return np.where((idx >= 0) & (idx < n), arr[np.clip(idx, 0, max(n - 1, 0))], 0)

    def s2(p_, q_):
        return np.where((p_ & q_) != 0, match, mismatch)

    def s3f(an, bn, cn):
        if sop:
            return s2(an, bn) + s2(bn, cn) + s2(an, cn)
        eab, ebc = (an & bn) != 0, (bn & cn) != 0
        return np.where(eab, np.where(ebc, 3 * match, 2 * (match + mismatch)), 3 * mismatch)

    def push(Sst, an, bn, cn):
        """The 7 values a cell with states Sst = [M, X, Y, Z, XY, YZ, XZ] pushes
        (targets Ix, Iy, Iz, Ixy, Iyz, Ixz, M), successor codes an/bn/cn."""
        add = {1: 0, 2: 0, 3: 0, 4: s2(an, bn), 5: s2(bn, cn), 6: s2(an, cn), 0: s3f(an, bn, cn)}
        out = {}
        for T_ in range(7):
            cand = [wrap(Sst[s] - P[T_][s] + wrap(add[T_])) for s in range(7)]
            out[T_] = np.maximum.reduce(cand)
        return out

    def zero_push(an, bn, cn):
        z = np.zeros(np.broadcast(an, bn, cn).shape, np.int64)
        return push([z] * 7, an, bn, cn)

    WO = SK + 1
    tau = lambda r: WO * (r >> 1) + (r & 1)
    YOFF = WO * (NW - 1) + 1
    yrec, zrec = {}, {}
    score = fin = None
    lanes = np.arange(64)
    kpos = M * lanes[None, :] + np.arange(M)[:, None]      # [M, 64]
    for L in range(G):
        for q in range(GZ):
            zt_q = min(ZT, lc - q * ZT)
            rows = min(RW, lb - L * RW)
            T = la + tau(rows - 1) + (zt_q - 1) + 1    # x' = la of the last position at step T-1
            zc = q * ZT + kpos                          # 0-based z - 1
            cnext = code_at(Cc, lc, zc + 1)[:, :, None] * np.ones((1, 1, 2), np.int64)   # c_{z+1}
            c1 = int(Cc[0]) if lc else 0
            shape = (NW, M, 64, 2)
            oIx = np.zeros(shape, np.int64)
            shIz = np.zeros(shape, np.int64)
            svIxy = np.zeros(shape, np.int64)
            svIyz = np.zeros(shape, np.int64)
            shIxz = np.zeros((2,) + shape, np.int64)
            svM = np.zeros((2,) + shape, np.int64)
            own_prev = np.zeros((4,) + shape, np.int64)
            if q > 0:
                left = zrec[(L, q - 1)]
                for w in range(NW):
                    r1, r2 = left[ZT - 1][w], left[ZT - 2][w]
                    shIz[w, 0, 0] = r1[0]
                    svIyz[w, 0, 0] = r1[2]
                    shIxz[1, w, 0, 0] = r1[1]
                    svM[1, w, 0, 0] = r1[3]
                    shIxz[0, w, 0, 0] = r2[1]
                    svM[0, w, 0, 0] = r2[3]
            else:
                # wave 0's low half reaches x' = 1 at step 1: its Ixz / M inputs
                # from the z = 0 face (x' - 1 = 0) would have been shifted in at
                # step -1 (tools/literal_emu.py: the same initial faces)
                a0 = int(A[0]) if la else 0
                by = int(Bc[L * RW]) if L * RW < lb else 0
                f = zero_push(np.array(a0), np.array(by), np.array(c1))
                shIxz[1, 0, 0, 0, 0] = int(f[6])
                svM[1, 0, 0, 0, 0] = int(f[0])
            ys, zs, out_hist = [], [], []
            for t in range(T):
                PH = t & 1
                out_now = np.zeros((4,) + shape, np.int64)
                zstep = [None] * NW
                for w in range(NW):
                    ulo = t - WO * w - kpos                     # x' of the low half
                    u = np.stack([ulo, ulo - 1], -1)            # [M, 64, 2]
                    an = code_at(A, la, u)                      # a_{x'+1} = a[x']
                    rowi = L * RW + 2 * w + np.arange(2)        # 0-based rows y - 1 of the halves
                    bnext = code_at(Bc, lb, rowi + 1)[None, None, :] * np.ones((M, 64, 1), np.int64)  # b_{y+1}
                    # ---- the row above
                    if w == 0:
                        if L == 0:  # row 0: zero cells pushing into row 1 at the same x'
                            b1 = np.full((M, 64), int(Bc[0]) if lb else 0)
                            fo = zero_push(an[..., 0], b1, cnext[..., 0])
                            lo = np.stack([fo[2], fo[3 + 1], fo[5], fo[0]])     # {Iy, Ixy, Iyz, M}
                            above = np.stack([lo, lo], -1)
                        else:
                            prev = yrec[(L - 1, q)]
                            r = t + YOFF
                            above = prev[min(r, len(prev) - 1)]
                    else:
                        above = out_hist[t - SK][:, w - 1] if t >= SK else np.zeros((4, M, 64, 2), np.int64)
                    REC = np.empty((4, M, 64, 2), np.int64)
                    REC[..., 0] = above[..., 1] if not (w == 0 and L == 0) else above[..., 0]
                    REC[..., 1] = own_prev[:, w][..., 0]
                    X, Y, Z = oIx[w].copy(), REC[0].copy(), shIz[w].copy()
                    XY, YZ = svIxy[w].copy(), svIyz[w].copy()
                    XZ, MM = shIxz[PH, w].copy(), svM[PH, w].copy()
                    inj = u == 0                                # x' = 0: the face cell
                    for v in (X, Y, Z, XY, YZ, XZ, MM):
                        v[inj] = 0
                    Sst = [MM, X, Y, Z, XY, YZ, XZ]
                    if L == G - 1 and q == GZ - 1:
                        rf = (lb - 1) - L * RW
                        kf = (lc - 1) - q * ZT
                        if rf // 2 == w and t == la + tau(rf) + kf:
                            fin = [int(v[kf % M, kf // M, rf % 2]) for v in Sst]
                            score = max(fin)
                    o = push(Sst, an, bnext, cnext)
                    out = np.stack([o[2], o[4], o[5], o[0]])    # {Iy, Ixy, Iyz, M} to the row below
                    out_now[:, w] = out
                    own_prev[:, w] = out
                    zstep[w] = (o[3][M - 1, 63].copy(), o[6][M - 1, 63].copy(),
                                REC[2][M - 1, 63].copy(), REC[3][M - 1, 63].copy())
                    oIx[w] = o[1]
                    svIxy[w] = REC[1]
                    if q > 0:
                        left = zrec[(L, q - 1)]
                        fz = left[min(t + ZT, len(left) - 1)][w]
                    else:  # z = 0: zero cells (x', y, 0) pushing into position 0
                        hs = np.arange(2)
                        a1 = code_at(A, la, t + 1 - (WO * w + hs))       # a_{x'} of position 0 two steps on
                        by = code_at(Bc, lb, rowi)                       # b_y of each half
                        fzp = zero_push(a1, by, np.full(2, c1))
                        fz = (fzp[3], fzp[6], fzp[5], fzp[0])

                    def zshift(src, f):
                        v = np.empty_like(src)
                        v[1:] = src[:-1]
                        v[0, 1:] = src[M - 1, :-1]
                        v[0, 0] = f
                        return v
                    shIz[w] = zshift(o[3], fz[0])
                    shIxz[PH, w] = zshift(o[6], fz[1])
                    svIyz[w] = zshift(REC[2], fz[2])
                    svM[PH, w] = zshift(REC[3], fz[3])
                out_hist.append(out_now)
                ys.append(out_now[:, NW - 1].copy())
                zs.append(zstep)
            yrec[(L, q)] = ys
            zrec[(L, q)] = zs
    return score, fin


if __name__ == "__main__":
    import sys
    rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
    a, b, c = (rng.integers(0, 4, n) for n in (20, 11, 70))
    print(emulate(a, b, c, NW=2, M=1))
