"""CPU emulation of the pencil kernel's schedule (pencil_kernel.hip) -- a
debugging aid. Arrays are [wave][lane][pair][half] int32; every step mirrors
the kernel's receive / substitute / compute / send / shift sequence, with the
same helix position mapping k = 64*M*half + M*lane + pair."""
import sys
import numpy as np

PD, PMIN, NW = 8, 48, 16


def emulate(a, b, c, match=1, mismatch=-1, go=2, ge=1, sop=False, skew=1):
    # skew: steps between consecutive waves (TSA_SKEW; the kernel uses 2 for
    # M <= 2): wave w reads wave w-1's record of step t-skew from 2*skew slots
    la, lb, lc = len(a), len(b), len(c)
    M = 1 if lc <= 128 else 2
    ZT = 128 * M
    P = max(la, ZT, PMIN)
    R = P + 8
    E, O, E2, OE, O2 = ge, go, 2 * ge, go + ge, 2 * go
    f_single = -min(E2, OE, O2)
    f_pair = -min(E, O)
    oh = lambda s: 1 << (int(s) & 3)
    sA = np.array([oh(a[i]) if i < la else 0 for i in range(P)])
    sB = np.array([oh(b[i]) if i < lb else 0 for i in range(4096)])
    lane = np.arange(64)
    k = M * lane[:, None, None] + 64 * M * np.arange(2)[None, None, :] + np.arange(M)[None, :, None]  # [64][M][2]
    cpos = np.where(k < lc, np.array([oh(c[j]) if j < lc else 0 for j in range(ZT)])[np.minimum(k, ZT - 1)], 0)
    W = np.arange(NW)[:, None, None, None]
    shape = (NW, 64, M, 2)
    x0 = ((-W - k[None]) % P)
    areg = sA[x0]
    breg = np.zeros(shape, np.int64)
    breg[0, 0, 0, 0] = sB[0]
    oIx = np.full(shape, f_single); shIz = np.full(shape, f_single)
    shIxz1 = np.full(shape, f_pair); shIxz2 = np.full(shape, f_pair)
    svIxy = np.full(shape, f_pair); svIyz = np.full(shape, f_pair)
    svM1 = np.zeros(shape, np.int64); svM2 = np.zeros(shape, np.int64)
    xr = np.zeros((NW, 2 * skew, 64, M, 2, 4), np.int64)   # record slots written by wave w
    ring = np.zeros((R, 64, M, 2, 4), np.int64)
    ring[..., 0] = f_single; ring[..., 1] = f_pair; ring[..., 2] = f_pair; ring[..., 3] = 0
    lap = P - skew * (NW - 1)
    xpos0 = np.array([(P - (skew * w % P)) % P for w in range(NW)])
    lap0 = np.array([0 if w == 0 else -1 for w in range(NW)])
    lap_f, w_f, k_f = (lb - 1) // NW, (lb - 1) % NW, lc - 1
    t_f = lap_f * P + (la - 1) + skew * w_f + k_f
    h_f = k_f // (64 * M); l_f, i_f = divmod(k_f - 64 * M * h_f, M)
    order = np.argsort(k.reshape(-1))  # flat (lane, pair, half) index of position 0, 1, ...

    def shift(v, inj):
        # position k <- k-1 along the helix; position 0 gets inj (per wave)
        flat = v.reshape(v.shape[0], -1)
        out = np.empty_like(flat)
        out[:, order[1:]] = flat[:, order[:-1]]
        out[:, order[0]] = inj
        return out.reshape(v.shape)

    score = None
    for t in range(t_f + 1):
        rec = np.empty((NW, 64, M, 2, 4), np.int64)
        rec[0] = ring[(t - lap) % R]
        rec[1:] = xr[:-1, (t - skew) % (2 * skew)]
        inIx, inIy, inIz = oIx.copy(), rec[..., 0].copy(), shIz.copy()
        inIxy, inIyz, inIxz, inM = svIxy.copy(), svIyz.copy(), shIxz2.copy(), svM2.copy()
        for w in range(NW):
            ks = xpos0[w]
            if ks < ZT:
                h = ks // (64 * M); l, i = divmod(ks - 64 * M * h, M)
                inIx[w, l, i, h] = f_single; inIxy[w, l, i, h] = f_pair
                inIxz[w, l, i, h] = f_pair; inM[w, l, i, h] = 0
        eab = (areg & breg) != 0
        eac = (areg & cpos[None]) != 0
        ebc = (breg & cpos[None]) != 0
        s2 = lambda e: np.where(e, match, mismatch)
        s2ab, s2ac, s2bc = s2(eab), s2(eac), s2(ebc)
        if sop:
            s3 = s2ab + s2bc + s2ac
        else:
            s3 = np.where(eab, np.where(ebc, 3 * match, 2 * (match + mismatch)), 3 * mismatch)
        sM = inM + s3; sX, sY, sZ = inIx, inIy, inIz
        sXY, sYZ, sXZ = inIxy + s2ab, inIyz + s2bc, inIxz + s2ac
        mx = np.maximum
        # GO >= GE: each target's highest-penalty group widened to all 7 states
        best = mx.reduce([sM, sX, sY, sZ, sXY, sYZ, sXZ])
        nIx = mx.reduce([sX - E2, mx.reduce([sY, sZ, sXY, sXZ]) - OE, best - O2])
        oIy = mx.reduce([sY - E2, mx.reduce([sX, sZ, sXY, sYZ]) - OE, best - O2])
        oIz = mx.reduce([sZ - E2, mx.reduce([sX, sY, sYZ, sXZ]) - OE, best - O2])
        oIxy = mx(mx.reduce([sX, sY, sXY]) - E, best - O)
        oIyz = mx(mx.reduce([sY, sZ, sYZ]) - E, best - O)
        oIxz = mx(mx.reduce([sX, sZ, sXZ]) - E, best - O)
        recout = np.stack([oIy, oIxy, oIyz, best], -1)
        xr[:, t % (2 * skew)] = recout
        last = recout[NW - 1].copy()
        unstarted = (t - skew * (NW - 1) - k) < 0   # u < 0: row y0-1 of lap 0 is the y=0 face
        last[unstarted] = [f_single, f_pair, f_pair, 0]
        ring[t % R] = last
        if t == t_f:
            score = int(best[w_f, l_f, i_f, h_f])
        oIx = nIx
        shIxz2 = shIxz1
        shIxz1 = shift(oIxz, f_pair)
        shIz = shift(oIz, f_single)
        svIxy = rec[..., 1]
        svIyz = shift(rec[..., 2], f_pair)
        svM2 = svM1
        svM1 = shift(rec[..., 3], 0)
        xpos0 = xpos0 + 1
        wrap = xpos0 == P
        xpos0[wrap] = 0; lap0[wrap] += 1
        ainj = sA[xpos0]
        row0 = lap0 * NW + np.arange(NW)
        binj = np.where((lap0 >= 0) & (row0 < lb), sB[np.clip(row0, 0, 4095)], 0)
        ash = shift(areg, 0); ash[:, 0, 0, 0] = ainj; areg = ash
        bsh = shift(breg, 0); bsh[:, 0, 0, 0] = binj; breg = bsh
    return score


if __name__ == "__main__":
    sys.path.insert(0, "oracle")
    import oracle
    rng = np.random.default_rng(0)
    for la, lb, lc in [(64, 64, 64), (5, 40, 3), (47, 17, 128), (130, 31, 200), (20, 3, 1)]:
        A, B, C = (rng.integers(0, 4, n) for n in (la, lb, lc))
        e, r = emulate(A, B, C), oracle.score(A, B, C)
        print(la, lb, lc, e, r, "OK" if e == r else "MISMATCH")
