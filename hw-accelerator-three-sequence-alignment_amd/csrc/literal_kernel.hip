// literal_kernel.hip -- the RTL's literal arithmetic in the helix schedule
// (TSA_KERNEL_PLANE's batch path; tools/literal_emu.py replays it on the CPU).
//
// The literal recurrence (src/PE_1cyc.v:164-218) wraps every one of a target's
// 7 candidates to SCORE_BITS before the MAX7 (the `wordsize` candidate wires,
// src/PE_1cyc.v:127-133), so it cannot be factored into messages the way the
// pencil kernels do. In PULL form a cell needs all 7 states of 7 predecessors;
// in PUSH form it needs only its own 7 states and its successors' symbols
// (a_{x+1}, b_{y+1}, c_{z+1}): for each successor it computes the one state
// that successor takes from it -- the full literal MAX7 -- and sends it. The
// data flow is then exactly the helix's (pencil_kernel.hip): one value per
// edge, {Iy, Ixy, Iyz, M} records down the rows, {Ix} along x, {Iz, Ixz, Iyz,
// M} shifted along z, so the same schedule runs it:
//   * one workgroup per triple, NW = 8 waves = rows, two steps of skew per row,
//     one s_barrier per two steps, the wave-0 ring prefetched by LDS-DMA;
//   * lane l, register i, half h is position k = 64M h + M l + i (z = k + 1);
//   * position k of wave w is at x' = (t - 2w - k) mod P at step t: x' = 0 is a
//     column of the helix for the x = 0 face (P >= LA + 1) -- that position's 7
//     inputs are forced to 0, so its pushes are the face's;
//   * the y = 0 face: ring rows wave 0 reads in its first lap hold row 0's
//     pushes into row 1; the z = 0 face: position 0's z-1 inputs are pushes of
//     a zero cell with its own symbols (a_x, b_y, c_1), chosen in SALU.
// Arithmetic: every value shifted left by 16 - SCORE_BITS in an int16 half
// (two cells per VGPR), so v_pk_add_u16 wraps exactly at the RTL word and
// v_pk_max_i16 is its signed compare: no wrap instruction at all. Per cell pair
// 94 VALU: 28 for the three single targets (13 shared candidate adds), 15 for
// each pair target and M, 6 for the successor indicators.

#include "pencil_common.h"
#include "lap_kernel.h"

namespace tsa {

constexpr int LIT_NW = 8, LIT_S = 2, LIT_RING_EXTRA = 8;
// M <= 2: P a multiple of 4, so (as in the pencil helix, TSA_EV_STATIC) each
// wave meets the x' = 0 half-mask and lap-wrap events at one static step of
// its four-step group, the x' = 0 register is the step's parity (M = 2), and
// the injection is a tracked mask with no per-step branch
#ifndef TSA_LIT_STATIC
#define TSA_LIT_STATIC 1
#endif
// ring rows wave 0 prefetches (LDS-DMA): 8, 4 at M = 4 (LDS)
__host__ __device__ constexpr int lit_pd(int M) { return M >= 4 ? 4 : 8; }

struct LitGeom {
  int32_t M, P, R;
  int64_t ring_bytes_per_triple;
  size_t lds;
};
static LitGeom lit_geom(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  LitGeom g;
  g.M = max_lc <= 128 ? 1 : max_lc <= 256 ? 2 : 4;
  g.P = std::max(max_la + 1, 128 * g.M);  // x' = 0 .. LA: the face column first
  g.P = (g.P + g.M - 1) / g.M * g.M;       // M = 2: the x' = 0 register is (t - w) parity
  if (g.M <= 2 && TSA_LIT_STATIC) g.P = (g.P + 3) / 4 * 4;  // TSA_LIT_STATIC
  g.R = g.P + LIT_RING_EXTRA;
  g.ring_bytes_per_triple = (int64_t)g.R * g.M * 64 * REC_BYTES;
  g.lds = (size_t)(LIT_NW - 1) * 2 * LIT_S * g.M * 1024 + (size_t)lit_pd(g.M) * g.M * 1024 +
          4 * ((size_t)g.P + 128 * g.M) + 4 * (((size_t)max_lb + 4) & ~(size_t)3) + (size_t)7 * g.M * 256 + 32;
  return g;
}

bool literal_shape_ok(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  if (max_la < 1 || max_lb < 1 || max_lc < 1 || max_lc > 512 || max_la > 4095 || max_lb > 4096) return false;
  return lit_geom(max_la, max_lb, max_lc).lds <= LDS_MAX;
}
// Cost model fitted on MI355X (profiles/r3d_literal_vs_plane.jsonl): the
// literal helix runs T steps of 0.56 us (M = 1) / 0.95 us (M = 2) per
// workgroup, ~1.8x slower per step with two workgroups on every CU; PLANE
// runs LA+LB+LC plane launches of 4.4 us + 0.41 us per triple per 256^2
// (y,z) cells. A few large cubes sweep faster as planes over the chip.
static double literal_helix_us(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  const LitGeom g = lit_geom(max_la, max_lb, max_lc);
  const double T = (double)((max_lb + LIT_NW - 1) / LIT_NW) * g.P + LIT_S * (LIT_NW - 1) + max_lc;
  // M = 4 (208 VGPRs) runs one workgroup per CU: ~2x the M = 2 step (an estimate)
  const double waves = g.M == 4 ? (double)((n + 255) / 256)
                                : n > 256 ? 1.8 * (double)((n + 511) / 512) : 1.0;
  return T * (g.M == 1 ? 0.56 : g.M == 2 ? 0.95 : 1.9) * waves;
}
static double plane_us(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  return (double)(max_la + max_lb + max_lc) *
         (4.4 + 0.41 * (double)n * (double)max_lb * (double)max_lc / 65536.0);
}
// The literal lap schedule (lap_kernel LIT) for a few cubes: the geometry of
// least estimated latency, as lap_choice picks the factored form's.
static LapGeom literal_lap_choice(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop,
                                  int lap) {
  LapGeom best{};
  best.ok = false;
  // lap steps are counted in 13 bits (the progress words): T < 8192
  if (lap == LAP_OFF || max_la > 4096 || max_la + 2 * 8 + 64 * 2 + 1 >= 8192) return best;
  int m_lo = 1, m_hi = 2, nw_lo = 4, nw_hi = 8;
  if (const char *e = getenv("TSA_LAP_M")) m_lo = m_hi = std::max(1, std::min(2, atoi(e)));  // knobs
  if (const char *e = getenv("TSA_LAP_NW")) nw_lo = nw_hi = atoi(e) == 4 ? 4 : 8;
  for (int M = m_lo; M <= m_hi; M *= 2)
    for (int NW = nw_lo; NW <= nw_hi; NW *= 2) {
      const LapGeom g = lap_geom_chunked(n, max_la, max_lb, max_lc, M, NW, false, sop, true);  // as lap_choice
      if (!g.ok) continue;
      if (!best.ok || g.est_us < best.est_us) best = g;
    }
  return best;
}
// One cube split over np devices by laps in the literal arithmetic: the
// literal lap's geometry with full-length rings (pencil_split_geom's reasons),
// if it has at least np laps.
LapGeom literal_split_geom(int32_t la, int32_t lb, int32_t lc, bool sop, int np) {
  LapGeom g = literal_lap_choice(1, la, lb, lc, sop, LAP_RESIDENT);
  if (np < 1 || !g.ok || g.G < np) {
    g.ok = false;
    return g;
  }
  return lap_geom(1, la, lb, lc, g.M, g.NW, true, false, sop, true);
}
int literal_kind(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop, int lap) {
  const bool helix_ok = literal_shape_ok(max_la, max_lb, max_lc);
  if (const char *e = getenv("TSA_PENCIL_MODE")) {  // test knobs
    if (!strcmp(e, "plane")) return LIT_PLANE;
    if (!strcmp(e, "literal")) return helix_ok ? LIT_HELIX : LIT_PLANE;
    if (!strcmp(e, "litlap") && literal_lap_choice(n, max_la, max_lb, max_lc, sop, lap).ok) return LIT_LAP;
  }
  int kind = LIT_PLANE;
  double best = plane_us(n, max_la, max_lb, max_lc);
  if (helix_ok) {
    const double h = literal_helix_us(n, max_la, max_lb, max_lc);
    if (h <= best) { best = h; kind = LIT_HELIX; }
  }
  const LapGeom g = literal_lap_choice(n, max_la, max_lb, max_lc, sop, lap);
  if (g.ok && 1.25 * g.est_us < best) kind = LIT_LAP;  // by a margin, as lap_choice
  return kind;
}
bool literal_helix_chosen(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  return literal_kind(n, max_la, max_lb, max_lc, false, LAP_OFF) == LIT_HELIX;
}
size_t literal_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  return (size_t)std::min<int32_t>(n, 65535) * (size_t)lit_geom(max_la, max_lb, max_lc).ring_bytes_per_triple;
}

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) { return pk_add(a, b); }
__device__ __forceinline__ uint32_t mx2(uint32_t a, uint32_t b) { return pk_max(a, b); }

// The 7 states a cell with states (M, X, Y, Z, XY, YZ, XZ) pushes to its
// successors (src/PE_1cyc.v:164-218 with the successor's scores): nIx to
// (x+1,y,z), oIy (x,y+1,z), oIz (x,y,z+1), oIxy (x+1,y+1,z), oIyz (x,y+1,z+1),
// oIxz (x+1,y,z+1), oM (x+1,y+1,z+1). an/bn/cn: the successors' symbol codes.
template <bool SOP>
__device__ __forceinline__ void push_literal(const LitArgs &c, uint32_t ones, uint32_t MM, uint32_t X,
                                             uint32_t Y, uint32_t Z, uint32_t XY, uint32_t YZ,
                                             uint32_t XZ, uint32_t an, uint32_t bn, uint32_t cn,
                                             uint32_t &nIx, uint32_t &oIy, uint32_t &oIz, uint32_t &oIxy,
                                             uint32_t &oIyz, uint32_t &oIxz, uint32_t &oM) {
  // single targets: the 13 distinct wrapped candidates, shared
  const uint32_t m2O = add2(MM, c.n2O);
  const uint32_t x2E = add2(X, c.n2E), xOE = add2(X, c.nOE);
  const uint32_t y2E = add2(Y, c.n2E), yOE = add2(Y, c.nOE);
  const uint32_t z2E = add2(Z, c.n2E), zOE = add2(Z, c.nOE);
  const uint32_t xyOE = add2(XY, c.nOE), xy2O = add2(XY, c.n2O);
  const uint32_t yzOE = add2(YZ, c.nOE), yz2O = add2(YZ, c.n2O);
  const uint32_t xzOE = add2(XZ, c.nOE), xz2O = add2(XZ, c.n2O);
  const uint32_t A = mx2(mx2(m2O, zOE), xyOE), Bv = mx2(xOE, yzOE);
  nIx = mx2(mx2(A, x2E), mx2(mx2(yOE, yz2O), xzOE));            // :172-178
  oIy = mx2(mx2(A, Bv), mx2(y2E, xz2O));                         // :180-186
  oIz = mx2(mx2(Bv, m2O), mx2(mx2(yOE, z2E), mx2(xy2O, xzOE)));  // :188-194
  // the successors' pair scores (src/PE_1cyc.v:159-161), as (s2 - GE) and (s2 - GO)
  const uint32_t eab = pk_eq1(an, bn, ones), ebc = pk_eq1(bn, cn, ones), eac = pk_eq1(an, cn, ones);
  const uint32_t uxy = pk_mad(eab, c.dmS, c.mmE), vxy = add2(uxy, c.nDOE);
  const uint32_t uyz = pk_mad(ebc, c.dmS, c.mmE), vyz = add2(uyz, c.nDOE);
  const uint32_t uxz = pk_mad(eac, c.dmS, c.mmE), vxz = add2(uxz, c.nDOE);
  // pair targets: penalty GE from the states sharing the gap, GO from the rest
  oIxy = mx2(mx2(mx2(add2(X, uxy), add2(Y, uxy)), mx2(add2(XY, uxy), add2(MM, vxy))),   // :196-202
             mx2(mx2(add2(Z, vxy), add2(YZ, vxy)), add2(XZ, vxy)));
  oIyz = mx2(mx2(mx2(add2(Y, uyz), add2(Z, uyz)), mx2(add2(YZ, uyz), add2(MM, vyz))),   // :204-210
             mx2(mx2(add2(X, vyz), add2(XY, vyz)), add2(XZ, vyz)));
  oIxz = mx2(mx2(mx2(add2(X, uxz), add2(Z, uxz)), mx2(add2(XZ, uxz), add2(MM, vxz))),   // :212-218
             mx2(mx2(add2(Y, vxz), add2(XY, vxz)), add2(YZ, vxz)));
  // M: every state plus the successor's triple score (src/PE_1cyc.v:162-170)
  uint32_t s3;
  if constexpr (SOP) s3 = pk_mad(eab, c.dmS, pk_mad(ebc, c.dmS, pk_mad(eac, c.dmS, c.mm3S)));
  else s3 = pk_mad(eab, pk_mad(ebc, c.d1S, c.d0S), c.neS);
  oM = mx2(mx2(mx2(add2(MM, s3), add2(X, s3)), mx2(add2(Y, s3), add2(Z, s3))),
           mx2(mx2(add2(XY, s3), add2(YZ, s3)), add2(XZ, s3)));
}

// LDS: xr [NW-1][4][M][64][16] wave w -> w+1 records {Iy, Ixy, Iyz, M}
//      xr0 [PD][M][64][16]     ring rows prefetched for wave 0 (LDS-DMA)
//      sA2 [P+ZT] u32          A codes (1 << s) of positions k (lo) and k+64M (hi)
//      sB  [LB+1] u32          B code, both halves
//      fin [7][M][64] u32      the final cell's states (wave w_f)
template <int M, bool SOP>
__global__ __launch_bounds__(64 * LIT_NW) void literal_kernel(
    const uint8_t *__restrict__ seqs, const int64_t *__restrict__ offs, int32_t n, int32_t P, int32_t R,
    int32_t lds_a, int32_t lds_b, int64_t ring_stride, uint8_t *__restrict__ ring_base,
    int32_t *__restrict__ scores, int32_t *__restrict__ final7, LitArgs ca) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int NW = LIT_NW, S = LIT_S, PD = lit_pd(M), ZT = 128 * M;
  constexpr int PAIR_BYTES = 64 * REC_BYTES, SLOT_BYTES = M * PAIR_BYTES;
  uint8_t *xr = smem;
  uint8_t *xr0 = xr + (NW - 1) * 4 * SLOT_BYTES;
  uint32_t *sA2 = (uint32_t *)(xr0 + PD * SLOT_BYTES);
  uint32_t *sB = (uint32_t *)((uint8_t *)sA2 + lds_a);
  uint32_t *fin = (uint32_t *)((uint8_t *)sB + lds_b);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t sel = lane == 0 ? 0x05040302u : 0x07060504u;  // zshift: lane 0 low half = the face
  uint32_t ones = 0x00010001u, zero = 0u;
  asm volatile("" : "+v"(ones), "+v"(zero));
  const uint32_t a_lane = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)sA2 +
                          4u * (uint32_t)(ZT - M * lane - (M - 1));
  const int32_t lag = P - S * (NW - 1);

  for (int tri = blockIdx.x; tri < n; tri += gridDim.x) {
    const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
    const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
    const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
    uint8_t *ring = ring_base + (int64_t)blockIdx.x * ring_stride;
    auto sym = [&](int64_t base, int32_t i, int32_t len) -> uint32_t {
      return (i >= 0 && i < len) ? 1u << tsa_sym(seqs, base + i, ca.packed) : 0u;
    };
    // ---- A codes of x' (lo: position k, hi: k + 64M) and B codes
    for (int j = threadIdx.x; j < P + ZT; j += 64 * NW) {
      const int x0 = ((j - ZT) % P + P) % P, x1 = ((j - ZT - 64 * M) % P + P) % P;
      sA2[j] = sym(o0, x0, la) | (sym(o0, x1, la) << 16);
    }
    for (int i = threadIdx.x; i <= lb; i += 64 * NW) sB[i] = sym(o1, i, lb) * 0x00010001u;
    __syncthreads();
    // per-position c_{z+1} (successor) and the pushes of a zero cell
    uint32_t cn[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int k0 = M * lane + i, k1 = 64 * M + k0;
      cn[i] = sym(o2, k0 + 1, lc) | (sym(o2, k1 + 1, lc) << 16);
    }
    const uint32_t c1 = sym(o2, 0, lc), b1 = sB[0] & 0xFFFFu;
    // A code of x' (0-based symbol index), 0 outside [0, la): the table's low half
    auto acode = [&](int32_t xp) -> uint32_t { return (xp >= 0 && xp < la) ? sA2[xp + ZT] & 0xFFFFu : 0u; };
    // a zero cell's pushes into successors with codes (an, bn, cn): per half
    auto face_pair = [&](uint32_t p, uint32_t q) -> uint32_t {  // pair target, indicator per half
      const uint32_t lo = (p & q & 0xFFFFu) ? ca.fP[1] : ca.fP[0];
      const uint32_t hi = (p & q & 0xFFFF0000u) ? ca.fP[1] : ca.fP[0];
      return (lo & 0xFFFFu) | (hi & 0xFFFF0000u);
    };
    auto face_m = [&](uint32_t an, uint32_t bn, uint32_t cc) -> uint32_t {
      uint32_t r = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t m = 0xFFFFu << (16 * h);
        const int idx = ((an & bn & m) ? 4 : 0) | ((bn & cc & m) ? 2 : 0) | ((an & cc & m) ? 1 : 0);
        r |= ca.fM[idx] & m;
      }
      return r;
    };
    // ring rows of wave 0's first lap: row 0's pushes into row 1 at step
    // t_r = (r + lag) mod R, where position k sits at x' = t_r - k
    auto row0 = [&](int32_t t_r, int i, uint4 &rec) {
      const int k0 = M * lane + i, k1 = 64 * M + k0;
      const uint32_t an = acode(t_r - k0) | (acode(t_r - k1) << 16);
      const uint32_t bb = b1 * 0x00010001u;
      rec = make_uint4(ca.fS[1], face_pair(an, bb), face_pair(bb, cn[i]), face_m(an, bb, cn[i]));
    };
    for (int64_t j = threadIdx.x; j < (int64_t)R * M * 64; j += 64 * NW) {  // j % 64 == lane
      const int32_t r = (int32_t)(j / (M * 64)), i = (int32_t)((j / 64) % M);
      uint4 rec;
      row0((r + lag) % R, i, rec);
      ((uint4 *)ring)[j] = rec;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    uint32_t bn[M], oIx[M], shIz[M], svIxy[M], svIyz[M], shIxz[2][M], svM[2][M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      bn[i] = oIx[i] = shIz[i] = svIxy[i] = svIyz[i] = 0u;
      shIxz[0][i] = shIxz[1][i] = svM[0][i] = svM[1][i] = 0u;
    }
    if (w == 0) {  // position 0 at x' = 1 in step 1: its z = 0 faces, as if shifted in at step -1
      const uint32_t a0 = acode(0);
      const uint32_t fxz = ca.fP[(a0 & c1) ? 1 : 0];
      const uint32_t fm = ca.fM[((a0 & b1) ? 4 : 0) | ((b1 & c1) ? 2 : 0) | ((a0 & c1) ? 1 : 0)];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        shIxz[1][i] = fxz;
        svM[1][i] = fm;
      }
    }
    int32_t xpos0 = (P - ((S * w) % P)) % P;  // position at x' = 0 at step t
    int32_t lap0 = w == 0 ? 0 : -1;
    // TSA_LIT_STATIC: the x' = 0 half mask (low below 64M, high below ZT, none
    // from ZT to the wrap), switched at those events
    constexpr bool LSTAT = TSA_LIT_STATIC && M <= 2;
    auto hm_of = [&](int32_t xp) -> uint32_t {
      return xp >= ZT ? 0u : xp >= 64 * M ? 0xFFFF0000u : 0x0000FFFFu;
    };
    auto ev_of = [&](int32_t xp) -> int32_t { return xp < 64 * M ? 64 * M : xp < ZT ? ZT : P; };
    uint32_t hmCur = hm_of(xpos0);
    int32_t next_ev = ev_of(xpos0);
    auto bcode = [&](int32_t row) -> uint32_t { return (row >= 0 && row < lb) ? sB[row] : 0u; };
    uint32_t binj = bcode(lap0 * NW + w + 1);  // b_{y+1} of the row that starts at x' = 0
    uint32_t bcur = bcode(lap0 * NW + w);      // b_y of position 0's row (the z = 0 face)
    const int32_t lap_f = (lb - 1) / NW, w_f = (lb - 1) % NW, k_f = lc - 1;
    const int32_t t_f = lap_f * P + la + S * w_f + k_f;  // cell (la, lb, lc) at x' = la
    const int32_t T = t_f + 1;
    if (w == 0) {
#pragma unroll 1
      for (int s = 0; s < PD; ++s) {
        const int32_t row = ((s - lag) % R + R) % R;
#pragma unroll
        for (int i = 0; i < M; ++i)
          dma16(ring + ((int64_t)row * M + i) * PAIR_BYTES + lane * REC_BYTES,
                xr0 + (s % PD) * SLOT_BYTES + i * PAIR_BYTES);
      }
    }
    int32_t dma_row = ((PD - lag) % R + R) % R;
    int32_t st_row = 0;
    uint32_t a_nx[M];
    load_a<M>(a_lane + 4u * (uint32_t)xpos0, a_nx);
    // z = 0 face of position 0 (z = 1): a zero cell's pushes with its own
    // symbols, uniform per wave: to Iz a constant, to Iyz by [b_y = c_1] (per
    // row), to Ixz by [a_x = c_1] and to M by the three indicators
    auto zfaces = [&](uint32_t &fz, uint32_t &fyz, uint32_t &fxz, uint32_t &fm) {
      const uint32_t a2 = __builtin_amdgcn_readfirstlane(
          *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t)(
              (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)sA2 + 4u * (uint32_t)(xpos0 + ZT))) &
          0xFFFFu;
      const uint32_t by = bcur & 0xFFFFu;
      fz = ca.fS[2];
      fyz = ca.fP[(by & c1) ? 1 : 0];
      fxz = ca.fP[(a2 & c1) ? 1 : 0];
      fm = ca.fM[((a2 & by) ? 4 : 0) | ((by & c1) ? 2 : 0) | ((a2 & c1) ? 1 : 0)];
    };

    auto step = [&](auto ph, auto role, int32_t t) {
      constexpr int Q = decltype(ph)::value;  // t & 3
      constexpr int PH = Q & 1;
      constexpr int ROLE = decltype(role)::value & 3;
      constexpr int WPAR = (decltype(role)::value >> 2) - 1;  // wave parity (-1: unknown)
      // LSTAT: the x' = 0 register is (t - 2w) mod M = PH (P even); the events
      // fall on step (2w - 1) mod 4 of the group only
      constexpr int IS = M == 1 ? 0 : (LSTAT && M == 2) ? PH : -1;
      constexpr bool EV_HERE = !LSTAT || WPAR < 0 || Q == (WPAR == 0 ? 3 : 1);
      uint32_t a[M];
#pragma unroll
      for (int i = 0; i < M; ++i) a[i] = a_nx[i];
      uint4 rec[M];
      if constexpr (ROLE == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(M * (PD - 1)) : "memory");
        const uint8_t *src = xr0 + (t % PD) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
      } else {
        const uint8_t *src = xr + ((w - 1) * 4 + ((Q + 2) & 3)) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
      }
      uint32_t X[M], Y[M], Z[M], XY[M], YZ[M], XZ[M], MM[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        X[i] = oIx[i];
        Y[i] = rec[i].x;
        Z[i] = shIz[i];
        XY[i] = svIxy[i];
        YZ[i] = svIyz[i];
        XZ[i] = shIxz[PH][i];
        MM[i] = svM[PH][i];
      }
      // ---- x' = 0 at position xpos0: the face column (all 7 inputs 0) and the
      // next row's B code for its successors
      if (LSTAT || xpos0 < ZT) {  // (LSTAT: hmCur is 0 past ZT)
        int32_t ls, is, hs;
        pos_split<M>(xpos0, ls, is, hs);
        const uint32_t hm = LSTAT ? hmCur : hs ? 0xFFFF0000u : 0x0000FFFFu;
        uint32_t m1;
        asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m1) : "v"(hm), "s"(1ull << ls));
#pragma unroll
        for (int i = 0; i < M; ++i) {
          if (IS >= 0 ? i == IS : i == is) {
            X[i] = vbfi(m1, zero, X[i]);
            Y[i] = vbfi(m1, zero, Y[i]);
            Z[i] = vbfi(m1, zero, Z[i]);
            XY[i] = vbfi(m1, zero, XY[i]);
            YZ[i] = vbfi(m1, zero, YZ[i]);
            XZ[i] = vbfi(m1, zero, XZ[i]);
            MM[i] = vbfi(m1, zero, MM[i]);
            bn[i] = vbfi(m1, binj, bn[i]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < M; ++i) asm volatile("" : "+v"(bn[i]));
      // the final cell's states (src/TriAlign_1cyc.v:130,138,141-142)
      if (t == t_f && w == w_f) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          fin[(0 * M + i) * 64 + lane] = MM[i];
          fin[(1 * M + i) * 64 + lane] = X[i];
          fin[(2 * M + i) * 64 + lane] = Y[i];
          fin[(3 * M + i) * 64 + lane] = Z[i];
          fin[(4 * M + i) * 64 + lane] = XY[i];
          fin[(5 * M + i) * 64 + lane] = YZ[i];
          fin[(6 * M + i) * 64 + lane] = XZ[i];
        }
      }
      uint32_t nIx[M], oIy[M], oIz[M], oIxy[M], oIyz[M], oIxz[M], oM[M];
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < M; ++i)
        push_literal<SOP>(ca, ones, MM[i], X[i], Y[i], Z[i], XY[i], YZ[i], XZ[i], a[i], bn[i], cn[i], nIx[i],
                          oIy[i], oIz[i], oIxy[i], oIyz[i], oIxz[i], oM[i]);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      // ---- records: to the wave below, or (last wave) the ring
      if constexpr (ROLE != 2) {
        uint8_t *dst = xr + (w * 4 + Q) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) lds_write16(dst + i * PAIR_BYTES, make_uint4(oIy[i], oIxy[i], oIyz[i], oM[i]));
      } else {
        if (t < ZT + S * NW) {  // not-started positions: row 0's pushes (wave 0 meets them at t + lag)
          const int32_t lim = t - S * w;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            const uint32_t m = ((M * lane + i > lim) ? 0x0000FFFFu : 0u) |
                               ((64 * M + M * lane + i > lim) ? 0xFFFF0000u : 0u);
            uint4 f;
            row0(t + lag, i, f);
            oIy[i] = bfi(m, f.x, oIy[i]);
            oIxy[i] = bfi(m, f.y, oIxy[i]);
            oIyz[i] = bfi(m, f.z, oIyz[i]);
            oM[i] = bfi(m, f.w, oM[i]);
          }
        }
        uint4 *dst = (uint4 *)__builtin_assume_aligned(ring + (int64_t)st_row * SLOT_BYTES + lane * REC_BYTES, 16);
#pragma unroll
        for (int i = 0; i < M; ++i) dst[i * 64] = make_uint4(oIy[i], oIxy[i], oIyz[i], oM[i]);
      }
      // ---- advance: position 0 moves on (a wrap starts a new row), then the shifts
#pragma unroll
      for (int i = 0; i < M; ++i) {
        oIx[i] = nIx[i];
        svIxy[i] = rec[i].y;
      }
      if constexpr (LSTAT) {
        if constexpr (!EV_HERE) {
          ++xpos0;
        } else if (__builtin_expect(++xpos0 == next_ev, 0)) {
          if (xpos0 == P) {
            xpos0 = 0;
            ++lap0;
            binj = bcode(lap0 * NW + w + 1);
            bcur = bcode(lap0 * NW + w);
          }
          hmCur = hm_of(xpos0);
          next_ev = ev_of(xpos0);
        }
      } else if (++xpos0 == P) {
        xpos0 = 0;
        ++lap0;
        binj = bcode(lap0 * NW + w + 1);
        bcur = bcode(lap0 * NW + w);
      }
      uint32_t fz, fyz, fxz, fm;
      zfaces(fz, fyz, fxz, fm);
      uint32_t rz[M], rw[M];
#pragma unroll
      for (int i = 0; i < M; ++i) { rz[i] = rec[i].z; rw[i] = rec[i].w; }
      zshift<M>(shIxz[PH], oIxz, sel, fxz);  // (the faces sit in both halves)
      zshift<M>(shIz, oIz, sel, fz);
      zshift<M>(svIyz, rz, sel, fyz);
      zshift<M>(svM[PH], rw, sel, fm);
      load_a<M>(a_lane + 4u * (uint32_t)xpos0, a_nx);
      if constexpr (ROLE == 0) {
#pragma unroll
        for (int i = 0; i < M; ++i)
          dma16(ring + ((int64_t)dma_row * M + i) * PAIR_BYTES + lane * REC_BYTES,
                xr0 + (t % PD) * SLOT_BYTES + i * PAIR_BYTES);
        if (++dma_row == R) dma_row = 0;
      }
      if constexpr (ROLE == 2) {
        if (++st_row == R) st_row = 0;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(M * 4) : "memory");
      }
      if constexpr (PH == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    auto run = [&](auto role) {
      constexpr std::integral_constant<int, 0> Q0{};
      constexpr std::integral_constant<int, 1> Q1{};
      constexpr std::integral_constant<int, 2> Q2{};
      constexpr std::integral_constant<int, 3> Q3{};
#pragma unroll 1
      for (int32_t t = 0; t < T; t += 4) {  // whole groups of four (past T: harmless cells)
        step(Q0, role, t);
        step(Q1, role, t + 1);
        step(Q2, role, t + 2);
        step(Q3, role, t + 3);
      }
    };
    // role | (wave parity + 1) << 2 (LSTAT's static event step); NW is even
    static_assert(NW % 2 == 0, "the last wave is odd");
    if (w == 0) run(std::integral_constant<int, 0 + 4>{});
    else if (w == NW - 1) run(std::integral_constant<int, 2 + 8>{});
    else if (w & 1) run(std::integral_constant<int, 1 + 8>{});
    else run(std::integral_constant<int, 1 + 4>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 7) {  // unshift the final cell's states
      int32_t l_f, i_f, h_f;
      pos_split<M>(k_f, l_f, i_f, h_f);
      const uint32_t v = fin[(threadIdx.x * M + i_f) * 64 + l_f];
      const int32_t s = (int32_t)(int16_t)(uint16_t)(h_f ? (v >> 16) : (v & 0xFFFF)) >> ca.sh;
      fin[7 * M * 64 + threadIdx.x] = (uint32_t)s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int32_t best = (int32_t)fin[7 * M * 64];
#pragma unroll
      for (int s = 1; s < 7; ++s) best = max(best, (int32_t)fin[7 * M * 64 + s]);
      scores[tri] = best;  // FINAL MAX7, src/TriAlign_1cyc.v:141-142
      if (final7)
        for (int s = 0; s < 7; ++s) final7[7 * (int64_t)tri + s] = (int32_t)fin[7 * M * 64 + s];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
static inline int32_t wrap_bits(int64_t v, int bits) {
  const uint64_t u = (uint64_t)v << (64 - bits);
  return (int32_t)((int64_t)u >> (64 - bits));
}
LitArgs lit_args(const KParams &kp) {
  LitArgs c;
  memset(&c, 0, sizeof(c));
  const int bits = kp.bits ? kp.bits : 16;
  const int sh = 16 - bits;
  c.sh = sh;
  c.packed = kp.packed;
  auto S = [&](int64_t v) { return ((uint32_t)(uint16_t)(uint32_t)(wrap_bits(v, bits) << sh)) * 0x00010001u; };
  const int32_t GE = kp.pen[SIXY][SIX], GO = kp.pen[SIXY][SM];
  c.n2E = S(-2 * GE);
  c.nOE = S(-(GO + GE));
  c.n2O = S(-2 * GO);
  c.dmS = S((int64_t)kp.match - kp.mismatch);
  c.mmE = S((int64_t)kp.mismatch - GE);
  c.nDOE = S(-(GO - GE));
  c.d1S = S((int64_t)kp.s3_eq - kp.s3_ab);
  c.d0S = S((int64_t)kp.s3_ab - kp.s3_ne);
  c.neS = S(kp.s3_ne);
  c.mm3S = S(3LL * kp.mismatch);
  // a zero cell's pushes: the literal MAX7 of wrapped candidates 0 - P + add
  auto push0 = [&](int T, int64_t add) {
    int32_t m = INT32_MIN;
    for (int s = 0; s < 7; ++s) m = std::max(m, wrap_bits((int64_t)-kp.pen[T][s] + add, bits));
    return S(m);
  };
  c.fS[0] = push0(SIX, 0);
  c.fS[1] = push0(SIY, 0);
  c.fS[2] = push0(SIZ, 0);
  c.fP[0] = push0(SIXY, kp.mismatch);
  c.fP[1] = push0(SIXY, kp.match);
  for (int idx = 0; idx < 8; ++idx) {
    const bool eab = idx & 4, ebc = idx & 2, eac = idx & 1;
    int64_t s3;
    if (kp.s3_mode == TSA_S3_SOP)
      s3 = (eab ? kp.match : kp.mismatch) + (int64_t)(ebc ? kp.match : kp.mismatch) + (eac ? kp.match : kp.mismatch);
    else
      s3 = eab ? (ebc ? kp.s3_eq : kp.s3_ab) : kp.s3_ne;
    c.fM[idx] = push0(SM, wrap_bits(s3, bits));
  }
  return c;
}

template <int M, bool SOP>
static int launch_lit(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_lb,
                      const LitGeom &g, int32_t *d_scores, int32_t *d_final7, void *d_ws, const LitArgs &ca,
                      hipStream_t stream) {
  const int32_t lds_a = 4 * (g.P + 128 * M), lds_b = 4 * ((max_lb + 4) & ~3);
  auto kfn = literal_kernel<M, SOP>;
  const int grid = n < 65535 ? n : 65535;
  return launch_with_lds((const void *)kfn, g.lds, [&] {
           hipLaunchKernelGGL(kfn, dim3(grid), dim3(64 * LIT_NW), g.lds, stream, d_seqs, d_offsets, n, g.P, g.R,
                              lds_a, lds_b, g.ring_bytes_per_triple, (uint8_t *)d_ws, d_scores, d_final7, ca);
         }) == hipSuccess
             ? TSA_OK
             : TSA_EDEVICE;
}

int literal_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_la,
                         int32_t max_lb, int32_t max_lc, const KParams &kp, int32_t *d_scores,
                         int32_t *d_final7, void *d_ws, size_t ws_bytes, hipStream_t stream) {
  if (n <= 0) return TSA_OK;
  if (!literal_shape_ok(max_la, max_lb, max_lc)) return TSA_EINVAL;
  if (ws_bytes < literal_workspace_bytes(n, max_la, max_lb, max_lc)) return TSA_ENOMEM;
  const LitGeom g = lit_geom(max_la, max_lb, max_lc);
  const LitArgs ca = lit_args(kp);
  const bool sop = kp.s3_mode == TSA_S3_SOP;
  if (g.M == 1)
    return sop ? launch_lit<1, true>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_final7, d_ws, ca, stream)
               : launch_lit<1, false>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_final7, d_ws, ca, stream);
  if (g.M == 4)
    return sop ? launch_lit<4, true>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_final7, d_ws, ca, stream)
               : launch_lit<4, false>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_final7, d_ws, ca, stream);
  return sop ? launch_lit<2, true>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_final7, d_ws, ca, stream)
             : launch_lit<2, false>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_final7, d_ws, ca, stream);
}

// ---------------------------------------------------------------------------
// TSA_KERNEL_PLANE's plan: the literal lap, the literal helix or the PLANE sweep
// (literal_kind), its workspace and its launch.
size_t literal_plan_workspace(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop, int lap) {
  n = std::min<int32_t>(n, 65535);
  switch (literal_kind(n, max_la, max_lb, max_lc, sop, lap)) {
    case LIT_LAP: return lap_workspace_bytes(literal_lap_choice(n, max_la, max_lb, max_lc, sop, lap));
    case LIT_HELIX: return literal_workspace_bytes(n, max_la, max_lb, max_lc);
    default: return plane_workspace_bytes(n, max_la, max_lb, max_lc);
  }
}
int literal_plan_launch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_la, int32_t max_lb,
                        int32_t max_lc, const KParams &kp, int32_t *d_scores, int32_t *d_final7, void *d_ws,
                        size_t ws_bytes, hipStream_t stream, int lap, int32_t **d_err, int32_t choice_n) {
  if (d_err) *d_err = nullptr;
  const bool sop = kp.s3_mode == TSA_S3_SOP;
  const int32_t cn = std::min<int32_t>(choice_n < 0 ? n : choice_n, 65535);
  const int kind = literal_kind(cn, max_la, max_lb, max_lc, sop, lap);
  if (kind == LIT_LAP) {
    const LapGeom g = literal_lap_choice(cn, max_la, max_lb, max_lc, sop, lap);
    if (n > cn || ws_bytes < lap_workspace_bytes(g)) return TSA_ENOMEM;
    return lap_launch_lit(g, sop, d_seqs, d_offsets, n, d_scores, d_final7, d_ws, kp, stream, d_err);
  }
  if (kind == LIT_HELIX)
    return literal_launch_batch(d_seqs, d_offsets, n, max_la, max_lb, max_lc, kp, d_scores, d_final7, d_ws,
                                ws_bytes, stream);
  return plane_launch_batch(d_seqs, d_offsets, n, max_la, max_lb, max_lc, kp, d_scores, d_final7, d_ws, ws_bytes,
                            stream);
}
void literal_describe(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop, int lap, char *buf,
                      size_t len) {
  n = std::min<int32_t>(n, 65535);
  const int kind = literal_kind(n, max_la, max_lb, max_lc, sop, lap);
  if (kind == LIT_LAP) {
    const LapGeom g = literal_lap_choice(n, max_la, max_lb, max_lc, sop, lap);
    snprintf(buf, len, "plane literal-lap M=%d NW=%d laps=%d tiles=%d waves=%lld", g.M, g.NW, g.G, g.GZ,
             (long long)g.waves);
    if (g.chunk > 0) snprintf(buf + strlen(buf), len - strlen(buf), " chunk=%d", g.chunk);
    snprintf(buf + strlen(buf), len - strlen(buf), " est=%.0fus", g.est_us);
  } else if (kind == LIT_HELIX) {
    snprintf(buf, len, "plane literal-helix est=%.0fus", literal_helix_us(n, max_la, max_lb, max_lc));
  } else {
    snprintf(buf, len, "plane est=%.0fus", plane_us(n, max_la, max_lb, max_lc));
  }
}

}  // namespace tsa
