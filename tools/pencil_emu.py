"""CPU replay of the helix kernel's schedule (csrc/pencil_kernel.hip).

TEST/DESIGN INFRASTRUCTURE: the helix's index and timing logic -- positions,
halves, the two-step wave skew, LDS record slots, the wave-0 ring with its
face rows, x = 1 injection, z-shifts with the z = 0 face, the final-cell
capture -- executed register by register with exact integer arithmetic, in
the message form (`vs=False`) or the V-space form of cell_messages_vs
(`vs=True`: values shifted by lam*(x+y+z), faces lam*q). tests/
test_pencil_schedule.py checks it against the oracle.

Layout as in the kernel: NW = 8 waves, wave w owns row y = lap*NW + w + 1;
lane l, register i, half h is position k = 64M h + M l + i (TWO mode, LC <= 64
and M = 1: k = l, and half h scores its own triple); position k of wave w
computes x = (t - S w - k) mod P + 1 at step t (S = 2).
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


def emulate(triples, match=1, mismatch=-1, go=2, ge=1, sop=False, vs=False):
    """Scores of one workgroup's unit: one triple, or two (TWO mode: LC <= 64).
    Returns a list of scores (one per triple)."""
    two = len(triples) == 2
    la_, lb_, lc_ = ([len(t[k]) for t in triples] for k in range(3))
    max_la, max_lb, max_lc = max(la_), max(lb_), max(lc_)
    M = 1 if max_lc <= 128 else 2
    assert not two or max_lc <= 64
    KS = 64 if two else 128 * M
    P = max(max_la, 64 if two else 128 * M)
    P = -(-P // M) * M
    if M == 2 and not two:  # the kernel's TSA_EV_STATIC: P a multiple of 4
        P = -(-P // 4) * 4
    R = P + RING_EXTRA
    lam = ge if vs else 0
    assert not vs or ge == -mismatch
    Pen = penalties(go, ge)
    f_single, f_pair = -int(Pen[1].min()), -int(Pen[4].min())
    dm = match - mismatch
    lanes = np.arange(64)
    shape = (M, 64, 2)
    i_ = np.arange(M)[:, None, None]
    l_ = lanes[None, :, None]
    h_ = np.arange(2)[None, None, :]
    kpos = (l_ + 0 * h_ + 0 * i_) if two else (64 * M * h_ + M * l_ + i_)   # [M, 64, 2]
    tri_of = (h_ + 0 * l_ + 0 * i_) if two else np.zeros(shape, np.int64)
    trip = triples if two else triples * 2

    def code(seq, idx):  # symbol (mod 4) or -1 past the sequence
        seq = np.asarray(seq, np.int64)
        ok = (idx >= 0) & (idx < len(seq))
        return np.where(ok, seq[np.clip(idx, 0, max(len(seq) - 1, 0))] & 3 if len(seq) else -1, -1)

    def per_half(fn):
        out = np.empty(shape, np.int64)
        for h in range(2):
            out[..., h] = fn(trip[h], h)[..., h]
        return out

    ccode = per_half(lambda t, h: code(t[2], kpos))
    # final cells: t_f per triple
    t_fs, w_fs, k_fs = [], [], []
    for (a, b, c) in (triples if two else triples[:1]):
        la, lb, lc = len(a), len(b), len(c)
        t_fs.append(((lb - 1) // NW) * P + (la - 1) + S * ((lb - 1) % NW) + (lc - 1))
        w_fs.append((lb - 1) % NW)
        k_fs.append(lc - 1)
    T = max(t_fs) + 1
    lag = P - S * (NW - 1)
    fin = [None] * len(t_fs)

    def face_rec(tr):  # the y = 0 row as wave 0 meets it at step tr
        if vs:
            return np.array([lam * (tr + 1), lam * (tr + 2), lam * (tr + 2), lam * (tr + 2)])
        return np.array([f_single, f_pair, f_pair, 0])

    ring = np.stack([face_rec((r + lag) % R)[:, None, None, None] * np.ones((1,) + shape, np.int64)
                     for r in range(R)])          # [R, 4, M, 64, 2]
    xr = np.zeros((NW, 4, 4) + shape, np.int64)    # [wave][slot][field]
    st = []
    for w in range(NW):
        xpos0 = (P - (S * w) % P) % P
        lap0 = 0 if w == 0 else -1
        d = dict(oIx=np.full(shape, f_single), shIz=np.full(shape, f_single),
                 svIxy=np.full(shape, f_pair), svIyz=np.full(shape, f_pair),
                 shIxz=[np.full(shape, f_pair), np.full(shape, f_pair)],
                 svM=[np.zeros(shape, np.int64), np.zeros(shape, np.int64)],
                 b=np.full(shape, -1), xpos0=xpos0, lap0=lap0)
        if vs:  # H(s) = lam (y + xpos0) at step s, H(-1) := H(0) - lam
            def h_at(s, w=w):
                u = s - S * w
                lp = u // P
                return lam * (lp * NW + w + 1 + (u - lp * P))
            d["H"] = {0: h_at(0), 1: h_at(1), -1: h_at(0) - lam}
            if w == 0:  # position 0's z = 0 faces at steps 0 and 1 ("shifted in" at steps -1, -2)
                d["shIz"][:] = d["svIyz"][:] = d["H"][0]
                d["shIxz"][1][:] = d["H"][1]
                d["svM"][1][:] = d["H"][0]
        st.append(d)

    def shift(v, face):
        # position k <- k-1; lane 0 register 0: low half the face, high half
        # lane 63's low half of register M-1 (TWO: both halves the face)
        out = np.empty_like(v)
        out[1:] = v[:-1]
        out[0, 1:] = v[M - 1, :-1]
        out[0, 0, 0] = face
        out[0, 0, 1] = face if two else v[M - 1, 63, 0]
        return out

    for t in range(T):
        PH = t & 1
        outs = [None] * NW
        for w in range(NW):
            d = st[w]
            rec = ring[(t - lag) % R] if w == 0 else xr[w - 1, (t - S) & 3]
            u = (t - S * w - kpos) % P
            acode = per_half(lambda tr, h: code(tr[0], u))
            inIx, inIy, inIz = d["oIx"].copy(), rec[0].copy(), d["shIz"].copy()
            inIxy, inIyz = d["svIxy"].copy(), d["svIyz"].copy()
            inIxz, inM = d["shIxz"][PH].copy(), d["svM"][PH].copy()
            b = d["b"]
            if d["xpos0"] < KS:  # x = 1 at position xpos0: the x = 0 face, the row's B
                inj = kpos == d["xpos0"]
                row = d["lap0"] * NW + w
                bn = per_half(lambda tr, h: code(tr[1], np.full(shape, row)))
                b = np.where(inj, bn, b)
                d["b"] = b
                if vs:
                    inIx[inj] = inIxy[inj] = inIxz[inj] = d["H"][t]
                    inM[inj] = d["H"][t - 1]
                else:
                    inIx[inj], inIxy[inj], inIxz[inj], inM[inj] = f_single, f_pair, f_pair, 0
            eab = (acode >= 0) & (acode == b)
            eac = (acode >= 0) & (acode == ccode)
            ebc = (b >= 0) & (b == ccode)
            if vs:
                sXY, sXZ, sYZ = inIxy + dm * eab, inIxz + dm * eac, inIyz + dm * ebc
                if sop:
                    sM = inM + dm * (eab.astype(np.int64) + ebc + eac) + 3 * mismatch + 3 * lam
                else:
                    sM = inM + np.where(eab, np.where(ebc, 3 * match, 2 * (match + mismatch)) - 3 * mismatch,
                                        0) + 3 * mismatch + 3 * lam
                sX, sY, sZ = inIx, inIy, inIz
                mx = np.maximum
                Gx, Gy, Gz = mx(mx(sY, sZ), sYZ), mx(mx(sX, sZ), sXZ), mx(mx(sX, sY), sXY)
                best = mx(mx(Gx, Gy), mx(sXY, sM))
                b1 = best - (go - ge)
                pXY, pYZ, pXZ = mx(Gz, b1), mx(Gx, b1), mx(Gy, b1)
                cP = go + mismatch + lam
                nIx = mx(sX - lam, mx(pXY, pXZ) - cP)
                oIy = mx(sY - lam, mx(pXY, pYZ) - cP)
                oIz = mx(sZ - lam, mx(pYZ, pXZ) - cP)
                oIxy, oIyz, oIxz = pXY, pYZ, pXZ
            else:  # message form, mismatch not folded (integer arithmetic)
                s2 = lambda e: np.where(e, match, mismatch)
                if sop:
                    s3 = s2(eab) + s2(ebc) + s2(eac)
                else:
                    s3 = np.where(eab, np.where(ebc, 3 * match, 2 * (match + mismatch)), 3 * mismatch)
                Sst = np.stack([inM + s3, inIx, inIy, inIz, inIxy + s2(eab), inIyz + s2(ebc),
                                inIxz + s2(eac)])
                msg = [(Sst - Pen[T_][:, None, None, None]).max(0) for T_ in range(7)]
                best, nIx, oIy, oIz, oIxy, oIyz, oIxz = msg
            for j, (tf, wf, kf) in enumerate(zip(t_fs, w_fs, k_fs)):
                if t == tf and w == wf:
                    pos = np.argwhere((kpos == kf) & (tri_of == j))[0]
                    fin[j] = int(best[tuple(pos)])
            out = np.stack([oIy, oIxy, oIyz, best])
            if w == NW - 1 and t < KS + S * NW:  # not-started positions publish the y = 0 face
                unstarted = kpos > t - S * w
                fr = face_rec(t + lag)
                for f in range(4):
                    out[f][unstarted] = fr[f]
            outs[w] = out
            # advance: position 0 moves on (wrap: a new row), then the z-shifts
            d["oIx"] = nIx
            d["svIxy"] = rec[1]
            if vs:
                d["H"][t + 2] = d["H"][t + 1] + lam
            d["xpos0"] += 1
            if d["xpos0"] == P:
                d["xpos0"] = 0
                d["lap0"] += 1
                if vs:
                    y = d["lap0"] * NW + w + 1
                    d["H"][t], d["H"][t + 1], d["H"][t + 2] = lam * (y - 1), lam * y, lam * (y + 1)
            if vs:
                h1, h2 = d["H"][t + 1], d["H"][t + 2]
                d["shIxz"][PH] = shift(oIxz, h2)
                d["shIz"] = shift(oIz, h1)
                d["svIyz"] = shift(rec[2], h1)
                d["svM"][PH] = shift(rec[3], h1)
            else:
                d["shIxz"][PH] = shift(oIxz, f_pair)
                d["shIz"] = shift(oIz, f_single)
                d["svIyz"] = shift(rec[2], f_pair)
                d["svM"][PH] = shift(rec[3], 0)
        for w in range(NW):
            xr[w, t & 3] = outs[w]
        ring[t % R] = outs[NW - 1]
    shifts = [lam * (len(a) + len(b) + len(c)) for (a, b, c) in (triples if two else triples[:1])]
    return [f - s for f, s in zip(fin, shifts)]
