"""CPU replay of the literal helix (csrc/pencil_kernel.hip, LIT): the RTL's
literal arithmetic in the helix's schedule.

TEST/DESIGN INFRASTRUCTURE (tests/test_pencil_schedule.py checks it against
the oracle). The pull-form recurrence needs all 7 states of 7 predecessors
per cell (src/PE_1cyc.v:164-218); its PUSH form has the helix's data flow: a
cell knows its successors' symbols (a_{x+1}, b_{y+1}, c_{z+1}) and computes,
for each successor, the one state that successor takes from it -- the full
literal MAX7 of 7 wrapped candidates -- and sends that state. Every value
then arrives final, one per edge, exactly where the message form sends one.

Arithmetic: SCORE_BITS-bit words, every candidate wrapped before the max
(src/PE_1cyc.v:127-133). The kernel keeps each value shifted left by
16 - SCORE_BITS in an int16 half, so int16 adds wrap exactly at the RTL word
and signed int16 max is the RTL's signed compare; here plain Python ints and
an explicit wrap.

Faces (the zero states of x = 0, y = 0, z = 0):
  * x = 0: a column of the helix (P >= LA + 1); the position at x = 0 has its 7
    inputs forced to 0 and pushes the face values to x = 1 itself;
  * y = 0: the ring rows wave 0 reads during its first lap hold row 0's
    pushes into row 1 (receiver symbols a_{x+1}, b_1, c_{z+1});
  * z = 0: position 0's z-1 inputs are row-0-style pushes computed with its
    own symbols (a_x, b_y, c_1), one and two steps ahead.
"""
from __future__ import annotations

import numpy as np

NW, S, RING_EXTRA = 8, 2, 8


def penalties(go, ge):
    GO2, GE2, GOGE = 2 * go, 2 * ge, go + ge
    return np.array([[0, 0, 0, 0, 0, 0, 0],
                     [GO2, GE2, GOGE, GOGE, GOGE, GO2, GOGE],
                     [GO2, GOGE, GE2, GOGE, GOGE, GOGE, GO2],
                     [GO2, GOGE, GOGE, GE2, GO2, GOGE, GOGE],
                     [go, ge, ge, go, ge, go, go],
                     [go, go, ge, ge, go, ge, go],
                     [go, ge, go, ge, go, go, ge]], dtype=np.int64)


def emulate(a, b, c, match=1, mismatch=-1, go=2, ge=1, sop=False, bits=12):
    """(score, final7) of one triple by the literal helix schedule."""
    la, lb, lc = len(a), len(b), len(c)
    M = 1 if lc <= 128 else 2 if lc <= 256 else 4
    KS = 128 * M
    P = max(la + 1, KS)
    P = -(-P // M) * M
    if M <= 2:  # the kernel's TSA_LIT_STATIC: P a multiple of 4
        P = -(-P // 4) * 4
    R = P + RING_EXTRA
    Pen = penalties(go, ge)

    def wrap(v):
        if bits == 0:
            return v
        m = 1 << bits
        return ((v + (m >> 1)) % m) - (m >> 1)

    def code(seq, idx):  # symbol mod 4, -1 past the sequence
        seq = np.asarray(seq, np.int64)
        ok = (idx >= 0) & (idx < len(seq))
        return np.where(ok, seq[np.clip(idx, 0, len(seq) - 1)] & 3, -1)

    def s2(p, q):
        return np.where((p >= 0) & (p == q), match, mismatch)

    def s3(p, q, r):
        if sop:
            return s2(p, q) + s2(q, r) + s2(p, r)
        ab, bc = (p >= 0) & (p == q), (q >= 0) & (q == r)
        return np.where(ab, np.where(bc, 3 * match, 2 * (match + mismatch)), 3 * mismatch)

    lanes = np.arange(64)
    shape = (M, 64, 2)
    kpos = (64 * M * np.arange(2)[None, None, :] + M * lanes[None, :, None] + np.arange(M)[:, None, None])
    cnext = code(c, kpos + 1)          # c_{z+1} of position k (z = k+1)
    c1 = int(code(c, np.array(0)))

    def push(Sst, an, bn, cn):
        """The 7 successor states a cell with states Sst pushes (targets Ix,
        Iy, Iz, Ixy, Iyz, Ixz, M: src/PE_1cyc.v:164-218 in push order)."""
        add = {1: 0, 2: 0, 3: 0, 4: s2(an, bn), 5: s2(bn, cn), 6: s2(an, cn), 0: s3(an, bn, cn)}
        out = {}
        for T_ in range(7):
            cand = [wrap(Sst[s] - Pen[T_][s] + wrap(add[T_])) for s in range(7)]
            out[T_] = np.maximum.reduce(cand)
        return out

    zero7 = [np.zeros(shape, np.int64)] * 7
    B0 = code(b, np.array(0))

    def row0_rec(t_r):
        """Row 0's pushes into row 1 as wave 0 meets them at step t_r: position
        k has x' = t_r - k, so the receivers' symbols are a_{x'+1}, b_1, c_{z+1}."""
        an = code(a, t_r - kpos)
        o = push(zero7, an, np.full(shape, int(B0)), cnext)
        return np.stack([o[2], o[4], o[5], o[0]])  # {Iy, Ixy, Iyz, M}

    lag = P - S * (NW - 1)
    ring = np.stack([row0_rec((r + lag) % R) for r in range(R)])
    xr = np.zeros((NW, 4, 4) + shape, np.int64)
    st = []
    for w in range(NW):
        st.append(dict(oIx=np.zeros(shape, np.int64), shIz=np.zeros(shape, np.int64),
                       svIxy=np.zeros(shape, np.int64), svIyz=np.zeros(shape, np.int64),
                       shIxz=[np.zeros(shape, np.int64)] * 2, svM=[np.zeros(shape, np.int64)] * 2,
                       bn=np.full(shape, -1), xpos0=(P - (S * w) % P) % P, lap0=0 if w == 0 else -1))
    # wave 0, position 0 at x' = 1 in step 1: its z = 0 faces (x - 1, y, 0) and
    # (x - 1, y - 1, 0) would have been shifted in at step -1
    f = push(zero7, np.full(shape, int(code(a, np.array(0)))), np.full(shape, int(B0)), np.full(shape, c1))
    st[0]["shIxz"][1] = np.full(shape, int(f[6][0, 0, 0]))
    st[0]["svM"][1] = np.full(shape, int(f[0][0, 0, 0]))
    lap_f, w_f, k_f = (lb - 1) // NW, (lb - 1) % NW, lc - 1
    t_f = lap_f * P + la + S * w_f + k_f          # x' = la at u = la
    fin = None

    def shift(v, face):
        out = np.empty_like(v)
        out[1:] = v[:-1]
        out[0, 1:] = v[M - 1, :-1]
        out[0, 0, 0] = face
        out[0, 0, 1] = v[M - 1, 63, 0]
        return out

    for t in range(t_f + 1):
        PH = t & 1
        outs = [None] * NW
        for w in range(NW):
            d = st[w]
            rec = ring[(t - lag) % R] if w == 0 else xr[w - 1, (t - S) & 3]
            u = (t - S * w - kpos) % P                 # x' of each position
            an = code(a, u)                             # a_{x'+1}
            X, Y, Z = d["oIx"].copy(), rec[0].copy(), d["shIz"].copy()
            XY, YZ = d["svIxy"].copy(), d["svIyz"].copy()
            XZ, MM = d["shIxz"][PH].copy(), d["svM"][PH].copy()
            if d["xpos0"] < KS:  # x' = 0 at position xpos0: the face column, the next row's B
                inj = kpos == d["xpos0"]
                for v in (X, Y, Z, XY, YZ, XZ, MM):
                    v[inj] = 0
                row = d["lap0"] * NW + w                # 0-based row of this lap
                d["bn"] = np.where(inj, int(code(b, np.array(row + 1))), d["bn"])
            Sst = [MM, X, Y, Z, XY, YZ, XZ]
            if t == t_f and w == w_f:
                pos = tuple(np.argwhere(kpos == k_f)[0])
                fin = [int(v[pos]) for v in Sst]
            o = push(Sst, an, d["bn"], cnext)
            out = np.stack([o[2], o[4], o[5], o[0]])
            if w == NW - 1 and t < KS + S * NW:        # not-started positions: row 0's pushes
                unstarted = kpos > t - S * w
                fr = row0_rec(t + lag)
                out[:, unstarted] = fr[:, unstarted]
            outs[w] = out
            d["oIx"] = o[1]
            d["svIxy"] = rec[1]
            d["xpos0"] += 1
            if d["xpos0"] == P:
                d["xpos0"] = 0
                d["lap0"] += 1
            # z = 0 faces of position 0 (z = 1), its own symbols: at step t+1
            # x' = xpos0, at t+2 x' + 1; row y = lap0*NW + w + 1
            row = d["lap0"] * NW + w
            by = np.full(shape, int(code(b, np.array(row))))
            a2 = np.full(shape, int(code(a, np.array(d["xpos0"]))))   # a_x at t+2 (x' + 1)
            f = push(zero7, a2, by, np.full(shape, c1))       # (x, y, 0)-style pushes into z = 1
            d["shIxz"] = list(d["shIxz"])
            d["svM"] = list(d["svM"])
            d["shIxz"][PH] = shift(o[6], int(f[6][0, 0, 0]))
            d["shIz"] = shift(o[3], int(f[3][0, 0, 0]))
            d["svIyz"] = shift(rec[2], int(f[5][0, 0, 0]))
            d["svM"][PH] = shift(rec[3], int(f[0][0, 0, 0]))
        for w in range(NW):
            xr[w, t & 3] = outs[w]
        ring[t % R] = outs[NW - 1]
    return max(fin), fin
