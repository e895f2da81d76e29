// pencil_kernel.hip -- TSA_KERNEL_PENCIL: register-systolic 3-D DP for CDNA4.
//
// The reference computes the cube with an 8x8 systolic PE array over (y,z)
// while A streams along x (src/TriAlign_1cyc.v:115-125, PE_1cyc.v:247-299),
// slicing the (y,z) plane into 8x8 pencils with face SRAMs between them
// (src/TriAlign_1cyc.v:78-98). This kernel keeps that idea -- every cell is
// computed from neighbour values that arrive by systolic shifts, never from a
// stored cube -- but shapes it for a 64-lane wave:
//
//  * one workgroup scores one triple; wave w of NW owns DP row y = lap*NW+w+1;
//  * the 64 lanes x M packed int16 pairs own Zt = 128*M consecutive z
//    positions k (lane l, register i, half h -> k = 64Mh + Ml + i), z = k+1:
//    a lane's consecutive positions sit in consecutive registers;
//  * position k of wave w computes cell x = u mod P + 1 of lap u div P at step
//    t, with u = t - w - k (one step of skew per y and per z). A lane that
//    finishes x = P of lap L continues with x = 1 of lap L+1 (row y+NW), so
//    there is no fill/drain between rows: the positions form a helix;
//  * z-1 neighbours arrive by register renaming (i >= 1) and one DPP
//    wave_ror:1 + v_perm for register 0, per message and step whatever M is,
//    y-1 neighbours through a 2-slot LDS record per wave pair, and the wave
//    above wave 0 (row y-1 of the previous lap) through a global ring that the
//    last wave writes and wave 0 prefetches PD steps ahead with LDS-DMA;
//  * A, B and the "x == 1" position flow through the same shifts; only lane
//    0 of pair 0 gets injected values (the z = 0 face, the next A symbol and
//    the current B symbol).
//
// Arithmetic is the factored ("message") form of src/PE_1cyc.v:164-218: a
// cell sends to each successor target T the value max_s(S[s] - P[T][s]) and
// the successor adds its pair/triple score. It equals the RTL's literal
// 49-candidate MAX7 whenever no candidate wraps at SCORE_BITS and every value
// fits int16, which the host proves a priori (trialign_api.hip:pencil_exact)
// before it ever selects this kernel.
//
// Supported shapes: LC <= 128*M (M = 1 or 2), LA <= 4096, LB <= 4096.

#include <vector>

#include "pencil_common.h"
#include "lap_kernel.h"

namespace tsa {


// waves (= DP rows) per lap: 8, two workgroups per CU, so one computes while
// the other waits at its barrier (16 rows in one 1024-thread workgroup measured
// slower in round 1 and dropped)
constexpr int PENCIL_NW = 8;
constexpr int STORE_SLACK = 4;     // last wave keeps <= this many steps of stores in flight
constexpr int MAX_LA = 4096, MAX_LB = 4096, MAX_LC = 1024;
// LDS-DMA prefetch distance (steps) of wave 0: helix (ring) and lap (hand-off);
// shorter for wide positions (M pairs per lane) so the record slots fit in LDS
__host__ __device__ constexpr int helix_pd(int M) { return M >= 8 ? 2 : M >= 4 ? 4 : 8; }
#ifndef TSA_SKEW  // helix: steps between waves; 2 = one barrier per two steps
#define TSA_SKEW 2
#endif
// skew and record slots per wave; M >= 4 keeps skew 1 (twice the slots would not fit LDS)
__host__ __device__ constexpr int helix_skew(int M) { return M <= 2 ? TSA_SKEW : 1; }
constexpr int RING_EXTRA = 8;
// V-space M = 2: the lap period P is a multiple of 4, so each wave meets its
// half-mask / lap-wrap events (xpos0 = 64M, 128M, P) at one static step of the
// four-step group (xpos0 is -2w mod 4 at the group start); the other three
// steps advance with no compare and no branch
#ifndef TSA_EV_STATIC
#define TSA_EV_STATIC 1
#endif
// V-space: the face values H(s) = lam q kept as wave-uniform integers and
// encoded to f16 bits in SALU (f16x2_int), so they live in SGPRs: no VALU add
// per step, and the bfi / perm that inject them read the SGPR directly
#ifndef TSA_H_SALU  // (measured slower: 1667 / 1645 vs 1697 / 1687 GCUPS, profiles/r5b_helix_ab.jsonl)
#define TSA_H_SALU 0
#endif
// V-space: step s's x = 1 injection applied to the state registers at the end
// of step s - 1 (before the step barrier), not to the inputs at the start of
// step s, where it stood between the barrier and the cell
#ifndef TSA_PREINJ  // (measured neutral with TSA_H_SALU: 1646 / 1646 vs 1667 / 1645, r5b)
#define TSA_PREINJ 0
#endif
// f16 bits of the integer v in both halves, exact for 0 <= v <= 2047 --
// integer ops only, so a wave-uniform v stays in SALU (~8 instructions). The
// face values lam q are >= 0, and < 2048 at every real cell (use_vs); a
// padding position (x > LA) may see a larger q, clamped to a finite value
// (its cells feed only padding cells and the x = 1 inputs the bfi replaces).
// With c = clz(v), v << (c - 21) puts the leading 1 at bit 10, which adds the
// one missing from the exponent field (45 - c - 1) + 1 = e + 15.
// Written in SALU asm: left to itself the compiler picks v_med3_i32 for the
// clamp and then keeps the whole encode in VALU (v is wave-uniform).
__device__ __forceinline__ uint32_t f16x2_int(int32_t v) {
  uint32_t r, a, c, t;
  asm("s_min_u32 %1, %4, 0x7ff\n\t"       // a = min(v, 2047) (v >= 0; unsigned: a negative v clamps too)
      "s_or_b32 %2, %1, 1\n\t"
      "s_flbit_i32_b32 %2, %2\n\t"         // c = clz(a | 1), 21..31
      "s_sub_u32 %3, %2, 21\n\t"
      "s_lshl_b32 %3, %1, %3\n\t"          // a << (c - 21): the leading 1 at bit 10
      "s_sub_u32 %2, 45, %2\n\t"
      "s_lshl_b32 %2, %2, 10\n\t"
      "s_add_u32 %3, %3, %2\n\t"           // + (45 - c) << 10
      "s_cmp_eq_u32 %1, 0\n\t"
      "s_cselect_b32 %3, 0, %3\n\t"
      "s_pack_ll_b32_b16 %0, %3, %3"
      : "=s"(r), "=&s"(a), "=&s"(c), "=&s"(t)
      : "s"(v)
      : "scc");
  return r;
}
// v_bfi_b32 with an SGPR source for the selected bits
__device__ __forceinline__ uint32_t vbfi_s(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "s"(a), "v"(b));
  return r;
}
// Ablation knobs (timing diagnostics only: the scores are WRONG when set):
// TSA_ABL_ZOWN / TSA_ABL_ZREC replace the DPP + v_perm z-shift of the own
// (Iz, Ixz) / the row-above (Iyz, M) messages by register moves, TSA_ABL_INJ
// drops the x = 1 injection -- how much of the step each costs.
#ifndef TSA_ABL_ZOWN
#define TSA_ABL_ZOWN 0
#endif
#ifndef TSA_ABL_ZREC
#define TSA_ABL_ZREC 0
#endif
#ifndef TSA_ABL_INJ
#define TSA_ABL_INJ 0
#endif
template <int M>
__device__ __forceinline__ void zmove_abl(uint32_t (&v)[M], const uint32_t (&src)[M]) {
#pragma unroll
  for (int i = M - 1; i >= 1; --i) v[i] = src[i - 1];
  v[0] = src[M - 1];
}
// A-table entries past P + 128M repeating its start (the table is periodic in
// P): the V-space loop reads a four-step group's A codes at constant offsets
// from one address computed at the group's start, across a lap wrap too
constexpr int A_PAD = 4;

struct PencilGeom {
  int32_t M;        // pairs per lane
  int32_t P;        // lap period (steps)
  int32_t R;        // ring rows
  bool two;         // two triples per workgroup (LC <= 64, M = 1)
  int64_t ring_bytes_per_triple;
};
// waves per CU the VGPR budget allows: 4 per SIMD up to M = 2, 2 beyond
static int waves_per_cu(int M) { return M >= 4 ? 8 : 16; }

static int helix_nw(int) { return PENCIL_NW; }
// TWO: for LC <= 64 a wave's two 16-bit halves hold two different triples at
// the same 64 positions (a lane = one z of both), instead of positions k and
// k+64 of one triple -- no idle half, and the lap period shrinks to max(LA, 64).
static bool helix_two(int32_t max_lc) {
  if (const char *e = getenv("TSA_PENCIL_TWO")) return atoi(e) != 0 && max_lc <= 64;  // A/B knob
  return max_lc <= 64;
}
static PencilGeom pencil_geom(int32_t max_la, int32_t max_lc) {
  PencilGeom g;
  g.M = pencil_pairs(max_lc);
  // >= 64 > NW + helix_pd + STORE_SLACK: ring lag
  g.two = helix_two(max_lc);
  g.P = std::max(max_la, g.two ? 64 : 128 * g.M);
  g.P = (g.P + g.M - 1) / g.M * g.M;  // even for M = 2: the x = 1 register is PH ^ (w & 1)
  if (g.M == 2 && !g.two && TSA_EV_STATIC) g.P = (g.P + 3) / 4 * 4;  // TSA_EV_STATIC
  g.R = g.P + RING_EXTRA;
  g.ring_bytes_per_triple = (int64_t)g.R * g.M * 64 * REC_BYTES;
  return g;
}
// vs: the V-space instantiation, whose M = 2 form (TSA_A_B64) also keeps the
// A table's copy shifted by one entry after fin; the other forms do not
static size_t helix_lds(int M, int NW, int32_t P, int32_t max_lb, bool vs) {
  const size_t a_tab = 4 * ((size_t)P + 128 * M + A_PAD);
  return (size_t)(NW - 1) * 2 * helix_skew(M) * M * 1024 + (size_t)helix_pd(M) * M * 1024 + a_tab +
         4 * (((size_t)max_lb + 3) & ~(size_t)3) + (size_t)M * 512 + (vs && M == 2 && TSA_A_B64 ? a_tab : 0);
}

// The factored messages widen each target's highest-penalty group to all seven
// states, exact only when gap_open >= gap_extend (cell_messages_f16).
bool pencil_supported(const tsa_params *p) { return p != nullptr && p->gap_open >= p->gap_extend; }

static bool pencil_shape_ok(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  if (!(max_la >= 1 && max_la <= MAX_LA && max_lb >= 1 && max_lb <= MAX_LB && max_lc >= 1 &&
        max_lc <= MAX_LC))
    return false;
  const PencilGeom g = pencil_geom(max_la, max_lc);
  // the helix is always runnable: the non-V-space form (use_vs admits the
  // V-space one only where its own footprint fits too)
  return helix_lds(g.M, helix_nw(g.M), g.P, max_lb, false) <= LDS_MAX;
}

static bool use_f16(const KParams &kp, const Range &r);
static bool use_vs(const KParams &kp, const Range &r, int32_t max_la, int32_t max_lb, int32_t max_lc);

// Estimated latency (us) of the helix kernel for a batch: dispatch waves x
// steps per triple x step time. Measured: a fully loaded chip (two 8-wave
// workgroups per CU) runs an M = 2 step in ~0.66 us (512 x 256^3 in 5.6 ms);
// a workgroup alone on its CU in 0.38 us (one 256^3 triple, 3.2 ms), M = 1
// (two triples per wave) in 0.31 us (one 64^3 triple, 0.18 ms).
static double helix_step_us(int M, bool loaded) {
  const double s = M == 1 ? 0.40 : M == 2 ? 0.66 : M == 4 ? 1.2 : 2.4;
  const double alone = M == 1 ? 0.31 : M == 2 ? 0.38 : M == 4 ? 0.7 : 1.4;
  return loaded ? s : alone;
}
static double helix_est(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  const PencilGeom g = pencil_geom(max_la, max_lc);
  const int nw = helix_nw(g.M);
  const int64_t per_cu = std::max<int64_t>(
      1, std::min<int64_t>(LDS_MAX / helix_lds(g.M, nw, g.P, max_lb, g.M == 2), waves_per_cu(g.M) / nw));
  const double T = (double)((max_lb - 1) / nw) * g.P + max_la + nw + max_lc;
  const int64_t units = g.two ? (n + 1) / 2 : n;
  return (double)((units + 256 * per_cu - 1) / (256 * per_cu)) * T *
         helix_step_us(g.M, units > 256);
}

// The lap kernel's geometry if it should run, else .ok = false (helix).
// Resident grids (waves == 1) are safe: every workgroup runs at once, so a
// consumer waiting for a record never holds a slot its producer needs. A cube
// beyond the resident slots runs in rounds inside one resident grid: each
// workgroup loops over its slot's laps in lap order (lap_kernel), so a
// consumer's producer is always running or done, and a producer never waits
// for a consumer of a later round (boundary rings, lap_geom); every wait is
// bounded.
static LapGeom lap_choice(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                          LapPolicy lap, bool f16, bool sop, bool need = false) {
  LapGeom none{};
  none.ok = false;
  if (lap == LAP_OFF || max_la > 4096 || max_la + 2 * 8 + 64 * 4 >= 8192) return none;
  const char *mode = getenv("TSA_PENCIL_MODE");
  if (mode && !strcmp(mode, "helix")) return none;
  const bool force = mode && !strcmp(mode, "lap");
  int m_lo = 1, m_hi = 4, nw_lo = 4, nw_hi = 8;
  if (const char *e = getenv("TSA_LAP_M")) m_lo = m_hi = std::max(1, std::min(4, atoi(e)));  // knobs
  if (const char *e = getenv("TSA_LAP_NW")) nw_lo = nw_hi = atoi(e) == 4 ? 4 : 8;
  LapGeom best = none;
  for (int M = m_lo; M <= m_hi; M *= 2) {
    for (int NW = nw_lo; NW <= nw_hi; NW *= 2) {
      // several rounds run as the resident workgroups' loops with boundary
      // rings (lap_geom), at any workgroups per CU (when the hardware
      // dispatcher ran round 2, two per CU started out of chain order and
      // timed out); a larger batch runs as chunks of triples, one launch
      // each (lap_geom_chunked)
      const LapGeom g = lap_geom_chunked(n, max_la, max_lb, max_lc, M, NW, f16, sop);
      if (!g.ok) continue;
      if (!best.ok || g.est_us < best.est_us) best = g;
    }
  }
  // `need` (the checked kernel): the lap schedule whatever the helix would cost;
  // otherwise the lap must win by a margin (its estimate is ~10-30 % uncertain,
  // and the helix has no cross-workgroup dependency)
  if (best.ok && !force && !need && 1.25 * best.est_us >= helix_est(n, max_la, max_lb, max_lc)) return none;
  return best;
}

bool pencil_checked_plan(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                         const KParams &kp, LapPolicy lap) {
  return pencil_shape_ok(max_la, max_lb, max_lc) &&
         lap_choice(n, max_la, max_lb, max_lc, lap, false, kp.s3_mode == TSA_S3_SOP, true).ok;
}

size_t pencil_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                              const KParams &kp, const Range &bound, LapPolicy lap, bool checked) {
  if (checked) {
    const LapGeom g = lap_choice(n, max_la, max_lb, max_lc, lap, false, kp.s3_mode == TSA_S3_SOP, true);
    return g.ok ? lap_workspace_bytes(g) : 0;
  }
  if (!pencil_shape_ok(max_la, max_lb, max_lc)) return 0;
  const size_t helix = (size_t)std::min<int32_t>(n, 65535) *
                       (size_t)pencil_geom(max_la, max_lc).ring_bytes_per_triple;
  const LapGeom g = lap_choice(n, max_la, max_lb, max_lc, lap, use_f16(kp, bound),
                               kp.s3_mode == TSA_S3_SOP);
  if (g.ok) return std::max(helix, lap_workspace_bytes(g));
  return helix;
}

bool pencil_shape_supported(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  return pencil_shape_ok(max_la, max_lb, max_lc);
}

// ---------------------------------------------------------------------------
// Helix kernel: one workgroup per triple (grid-stride over the batch).
//   LDS: xr  [NW-1][2][M][64][16]  wave w -> w+1 records {Iy, Ixy, Iyz, best}
//        xr0 [PD][M][64][16]       ring rows prefetched for wave 0 (LDS-DMA), PD = helix_pd(M)
//        sA2 [P+ZT] u32            A codes for positions k and k+64 of one pair
//        sB  [LB] u32              B code, both halves
//        fin [M][64] u32           best of the final step (wave w_f)
// F16 selects the exact-f16 arithmetic above, else the int16 form; VS the
// V-space f16 cell (cell_messages_vs): every value shifted by lam*(x+y+z), the
// zero faces injected as lam*q (x = 1: H(t), H(t-1); z = 0: H(t+1), H(t+2);
// y = 0: the ring's face records), the score shifted back at the end.
template <int M, int NW, bool F16, bool SOP, bool TWO, bool VS>
__global__ __launch_bounds__(64 * NW) void pencil_kernel(const uint8_t *__restrict__ seqs,
                                                         const int64_t *__restrict__ offs,
                                                         int32_t n, int32_t P, int32_t R,
                                                         int32_t lds_a, int32_t lds_b,
                                                         int64_t ring_stride,
                                                         uint8_t *__restrict__ ring_base,
                                                         int32_t *__restrict__ scores,
                                                         PencilArgs pa) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int PAIR_BYTES = 64 * REC_BYTES;  // one pair's record, 1 KiB
  constexpr int SLOT_BYTES = M * PAIR_BYTES;
  constexpr int ZT = 128 * M;
  constexpr int PD = helix_pd(M);
  constexpr int HSK = helix_skew(M), HNSL = 2 * HSK;
  uint8_t *xr = smem;
  uint8_t *xr0 = xr + (NW - 1) * HNSL * SLOT_BYTES;
  uint32_t *sA2 = (uint32_t *)(xr0 + PD * SLOT_BYTES);
  uint32_t *sB = (uint32_t *)((uint8_t *)sA2 + lds_a);
  uint32_t *fin = (uint32_t *)((uint8_t *)sB + lds_b);
  uint32_t *sA2s = (uint32_t *)((uint8_t *)fin + M * 512);  // A_B64: sA2 shifted by one entry
  constexpr bool A_B64 = VS && M == 2 && TSA_A_B64;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  static_assert(!TWO || M == 1, "two triples per wave: 64 positions, M = 1");
  static_assert(!VS || (F16 && M <= 2), "V-space: the f16 helix with the four-step loop");
  // f16 bits of an integer (|v| <= 2048: exact), in both halves
  auto h_bits = [](int32_t v) -> uint32_t {
    const _Float16 h = (_Float16)(float)v;
    return (uint32_t)__builtin_bit_cast(uint16_t, h) * 0x00010001u;
  };
  // TWO: the halves are two triples at the same position, so lane 0 takes its
  // whole word from the z = 0 face (no half crosses from lane 63)
  const uint32_t sel = lane == 0 ? (TWO ? 0x03020100u : 0x05040302u) : 0x07060504u;
  constexpr int KS = TWO ? 64 : 128 * M;  // positions (per half in TWO)
  uint32_t ones = F16 ? 0x08000800u : 0x00010001u;  // f16: match indicator 2^-13
  asm volatile("" : "+v"(ones));                     // keep it in a VGPR (VOP3P operand)
  const PencilArgs pv = F16 ? pa : pin_score_consts(pa);
  uint32_t fsv = pa.f_single, fpv = pa.f_pair;  // VGPR copies for v_bfi_b32 / v_pk_mad_u16
  uint32_t sbcv = pa.h_sbc, kdv = pa.h_kd, k0v = pa.h_k0, one1 = 0x00010001u;
  uint32_t hmLo = TWO ? 0xFFFFFFFFu : 0x0000FFFFu, hmHi = 0xFFFF0000u, zero = 0u;
  asm volatile("" : "+v"(fsv), "+v"(fpv), "+v"(sbcv), "+v"(kdv), "+v"(k0v), "+v"(one1));
  asm volatile("" : "+v"(hmLo), "+v"(hmHi), "+v"(zero));
  // a[i] of this lane at step t is sA2[(t-w) mod P + ZT - M lane - i]
  const uint32_t a_lane = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)sA2 +
                          4u * (uint32_t)(ZT - M * lane - (M - 1));

  // this lane's record slots: read from the wave above, written for the one
  // below (LDS pointers, so the slot offsets fold into the ds instructions)
  const lds_u8 *rd_base = to_lds(xr + (w > 0 ? (w - 1) * HNSL * SLOT_BYTES : 0) + lane * REC_BYTES);
  lds_u8 *wr_base = to_lds(xr + w * HNSL * SLOT_BYTES + lane * REC_BYTES);
  const int32_t nunit = TWO ? (n + 1) / 2 : n;  // workgroup units: triples, or pairs
  for (int unit = blockIdx.x; unit < nunit; unit += gridDim.x) {
    const int tri = TWO ? 2 * unit : unit;
    const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
    const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
    const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
    // TWO: the high halves score triple tri+1 (or repeat tri when n is odd)
    const bool has1 = TWO && tri + 1 < n;
    const int64_t *of1 = offs + 3 * (int64_t)(has1 ? tri + 1 : tri);
    const int64_t q0 = of1[0], q1 = of1[1], q2 = of1[2];
    const int32_t la1 = TWO ? (int32_t)(q1 - q0) : la, lb1 = TWO ? (int32_t)(q2 - q1) : lb;
    const int32_t lc1 = TWO ? (int32_t)(of1[3] - q2) : lc;
    const int32_t lbm = max(lb, lb1);
    uint8_t *ring = ring_base + (int64_t)blockIdx.x * ring_stride;

    // ---- stage A codes (padded to P, halves k/k+64M or, TWO, the two triples) and
    // B; face records in the ring
    auto a_entry = [&](int j) -> uint32_t {  // periodic in j: the pad repeats P
      const int x0 = ((j - ZT) % P + P) % P, x1 = TWO ? x0 : ((j - ZT - 64 * M) % P + P) % P;
      const uint32_t c0 = x0 < la ? SYM0 << tsa_sym(seqs, o0 + x0, pa.packed) : 0u;
      const uint32_t c1 = x1 < la1 ? SYM0 << tsa_sym(seqs, (TWO ? q0 : o0) + x1, pa.packed) : 0u;
      return c0 | (c1 << 16);
    };
    for (int j = threadIdx.x; j < P + ZT + A_PAD; j += 64 * NW) {
      sA2[j] = a_entry(j);
      if constexpr (A_B64) sA2s[j] = a_entry(j + 1);
    }
    for (int i = threadIdx.x; i < lbm; i += 64 * NW) {
      if constexpr (TWO)
        sB[i] = (i < lb ? SYM0 << tsa_sym(seqs, o1 + i, pa.packed) : 0u) |
                ((i < lb1 ? SYM0 << tsa_sym(seqs, q1 + i, pa.packed) : 0u) << 16);
      else
        sB[i] = (SYM0 << tsa_sym(seqs, o1 + i, pa.packed)) * 0x00010001u;
    }
    // ring rows of wave 0's lap 0 -> ring row (t - lag) mod R at step t
    const int32_t lag = P - HSK * (NW - 1);
    {
      const uint4 face = make_uint4(pa.f_single, pa.f_pair, pa.f_pair, 0u);
      const int64_t n16 = (int64_t)R * M * 64;
      for (int64_t i = threadIdx.x; i < n16; i += 64 * NW) {
        if constexpr (VS) {
          // row 0's face cells as wave 0 meets them at step tr: x + z = tr + 2 for
          // every position ({Iy, Ixy, Iyz, best} = lam q - lam, lam q x 3)
          const int32_t tr = (int32_t)((i / (M * 64) + lag) % R);
          const uint32_t f1 = h_bits(pa.lam * (tr + 1)), f2 = h_bits(pa.lam * (tr + 2));
          ((uint4 *)ring)[i] = make_uint4(f1, f2, f2, f2);
        } else {
          ((uint4 *)ring)[i] = face;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- per-position registers (arrays [2] alternate roles between even/odd steps)
    uint32_t b[M], c[M], SBC[M], K[M], DMC[M], DMB[M];
    uint32_t oIx[M], shIz[M], svIxy[M], svIyz[M], shIxz[2][M], svM[2][M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int k0 = M * lane + i, k1 = TWO ? k0 : 64 * M + M * lane + i;
      const uint32_t c0 = k0 < lc ? SYM0 << tsa_sym(seqs, o2 + k0, pa.packed) : 0u;
      const uint32_t c1 = k1 < lc1 ? SYM0 << tsa_sym(seqs, (TWO ? q2 : o2) + k1, pa.packed) : 0u;
      c[i] = c0 | (c1 << 16);
      DMC[i] = dm_over_code(pa.dmf, c[i]);
      b[i] = SBC[i] = K[i] = DMB[i] = 0;  // set when a position reaches x = 1 of its lap
      oIx[i] = pa.f_single;
      shIz[i] = pa.f_single;
      shIxz[0][i] = shIxz[1][i] = pa.f_pair;
      svIxy[i] = svIyz[i] = pa.f_pair;
      svM[0][i] = svM[1][i] = 0;
    }
    // position-0 bookkeeping (wave-uniform): u0 = t - w
    int32_t xpos0 = (P - ((HSK * w) % P)) % P;  // (t - HSK w) mod P at t = 0
    int32_t lap0 = w == 0 ? 0 : -1;     // floor((t - w) / P)
#if TSA_HM_TRACK
    // bfi half mask of the x = 1 position xpos0 -- low half below 64M, high
    // half below KS, none from KS up to the lap wrap (P > KS) -- switched at
    // those events (one compare per step) rather than tested every step
    auto hm_of = [&](int32_t xp) -> uint32_t {
      return xp >= KS ? zero : xp >= 64 * M ? hmHi : hmLo;
    };
    auto ev_of = [&](int32_t xp) -> int32_t { return xp < 64 * M ? 64 * M : xp < KS ? KS : P; };
    uint32_t hmCur = hm_of(xpos0);
    int32_t next_ev = ev_of(xpos0);
#endif
    // B code of row lap0*NW+w+1, taken by the position at x = 1 (0 past LB)
    auto b_of_lap = [&](int32_t lp) -> uint32_t {
      const int32_t r = lp * NW + w;
      return (lp >= 0 && r < lbm) ? sB[r] : 0u;
    };
    uint32_t binj = b_of_lap(lap0);
    // the per-row terms of the row whose B code is binj, for every position:
    // a position copies them when it reaches x = 1 (recomputed once per lap)
    uint32_t SBCn[M], Kn[M], DMBn = 0;
    auto row_terms = [&]() {
      if constexpr (F16 && TSA_ROW_NEXT) {
        // V-space: the [a=b] terms multiply the symbol code itself (a & b, no
        // min): DMB = dm / code(b) and, RTL, K = (d0 + [b=c] d1) / code(b)
        uint32_t kb0 = k0v, kbd = kdv;
        if constexpr (VS) {
          DMBn = dm_over_code(pa.dmf, binj);
          if constexpr (!SOP) {
            kb0 = dm_over_code(pa.d0f, binj);
            const uint32_t kb1 = dm_over_code(pa.d0f + pa.d1f, binj);
            kbd = (((kb1 & 0xFFFFu) - (kb0 & 0xFFFFu)) & 0xFFFFu) | ((((kb1 >> 16) - (kb0 >> 16)) & 0xFFFFu) << 16);
          }
        }
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const uint32_t e01 = pk_eq1(binj, c[i], one1);
          SBCn[i] = pk_mad(e01, sbcv, 0u);
          Kn[i] = pk_mad(e01, kbd, kb0);
        }
      }
    };
    row_terms();
    const int32_t lap_f = (lb - 1) / NW, w_f = (lb - 1) % NW, k_f = lc - 1;
    const int32_t t_f = lap_f * P + (la - 1) + HSK * w_f + k_f;  // final cell (la, lb, lc)
    // TWO: the high-half triple's final cell, captured by its own step test
    const int32_t w_f1 = (lb1 - 1) % NW, k_f1 = lc1 - 1;
    const int32_t t_f1 = ((lb1 - 1) / NW) * P + (la1 - 1) + HSK * w_f1 + k_f1;
    const int32_t T = (TWO ? max(t_f, t_f1) : t_f) + 1;

    // VS: Hr[s & 3] = H(s) = lam * (y + xpos0) at step s (y: position 0's row,
    // 1-based) -- the x = 0 face at the x = 1 position and, one and two steps
    // ahead, the z = 0 face of position 0; one v_pk_add per step, reset at a wrap
    uint32_t Hr[4] = {0u, 0u, 0u, 0u};
    int32_t Hq[4] = {0, 0, 0, 0};  // TSA_H_SALU: lam q as integers (Hr = their f16 bits)
    auto hq_at = [&](int32_t s) -> int32_t {
      const int32_t u = s - HSK * w;
      const int32_t lp = u >= 0 ? u / P : -((P - 1 - u) / P);
      return pa.lam * (lp * NW + w + 1 + (u - lp * P));
    };
    auto h_at = [&](int32_t s) -> uint32_t { return TSA_H_SALU ? f16x2_int(hq_at(s)) : h_bits(hq_at(s)); };
    if constexpr (VS) {
      Hq[0] = hq_at(0);
      Hq[1] = hq_at(1);
      Hq[3] = Hq[0] - pa.lam;
      Hr[0] = h_at(0);
      Hr[1] = h_at(1);
      // the step-0 injection's (0, y-1, z-1) face is H(0) - lam (wave 0 starts
      // its first row at step 0 with no wrap that would have set it)
      Hr[3] = TSA_H_SALU ? f16x2_int(Hq[3]) : U(H(Hr[0]) - H(pa.v_lam));
      if (w == 0) {  // position 0's z = 0 faces at steps 0 and 1 (as if shifted in at steps -1, -2)
#pragma unroll
        for (int i = 0; i < M; ++i) {
          shIz[i] = svIyz[i] = svM[1][i] = Hr[0];
          shIxz[1][i] = Hr[1];
        }
      }
    }
    // wave 0: prime the LDS-DMA pipeline (ring row of step s = s - P + NW - 1)
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
    int32_t dma_row = ((PD - lag) % R + R) % R;  // ring row for step t + PD
    uint32_t a_nx[M];                            // A codes of the coming step
    if constexpr (TSA_A_PREFETCH) load_a<M>(a_lane + 4u * (uint32_t)xpos0, a_nx);
    int32_t st_row = 0;                          // ring row written at step t (last wave)
    uint32_t abase = a_lane;                     // VS: A address of the group's first step
    // A_B64: the same entry in the shifted copy
    const uint32_t a_lane_s = a_lane + (uint32_t)((uint8_t *)sA2s - (uint8_t *)sA2);
    uint32_t abase_s = a_lane_s;

    // VS: the step whose cell is the final one, in this wave (-1: none)
    const int32_t t_fin = w == w_f ? T - 1 : -1;
    // the x = 1 mask kept from the even step of a pair (step, MASK_PAIRS)
    constexpr bool MASK_PAIRS = VS && M == 2 && HSK == 2 && TSA_HM_TRACK;
    uint32_t m1_pair = 0u;
    constexpr bool PRE = VS && TSA_PREINJ && !TSA_ABL_INJ && TSA_HM_TRACK;
    // PRE: the injection of the step of phase PQN (the next one), into the
    // registers that step reads: Ix (own), Ixy (the row above's record), Ixz and
    // M (the z-shifted double buffers of its parity), and the per-row terms
    auto vs_inject = [&](auto pqc) {
      constexpr int PQN = decltype(pqc)::value;
      constexpr int PHN = PQN & 1;
      constexpr int ISN = M == 2 ? PHN : -1;  // skew 2, even P: the x = 1 register is the step's parity
      int32_t ls, is, hs;
      pos_split<M>(xpos0, ls, is, hs);
      uint32_t m1;
      if constexpr (MASK_PAIRS && (PQN & 1)) {
        m1 = m1_pair;
      } else {
        asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m1) : "v"(hmCur), "s"(1ull << ls));
        if constexpr (MASK_PAIRS) m1_pair = m1;
      }
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (ISN >= 0 ? i == ISN : i == is) {
          if constexpr (TSA_H_SALU) {
            oIx[i] = vbfi_s(m1, Hr[PQN & 3], oIx[i]);
            svIxy[i] = vbfi_s(m1, Hr[PQN & 3], svIxy[i]);
            shIxz[PHN][i] = vbfi_s(m1, Hr[PQN & 3], shIxz[PHN][i]);
            svM[PHN][i] = vbfi_s(m1, Hr[(PQN + 3) & 3], svM[PHN][i]);
          } else {
            oIx[i] = vbfi(m1, Hr[PQN & 3], oIx[i]);
            svIxy[i] = vbfi(m1, Hr[PQN & 3], svIxy[i]);
            shIxz[PHN][i] = vbfi(m1, Hr[PQN & 3], shIxz[PHN][i]);
            svM[PHN][i] = vbfi(m1, Hr[(PQN + 3) & 3], svM[PHN][i]);
          }
          b[i] = vbfi(m1, binj, b[i]);
          SBC[i] = vbfi(m1, SBCn[i], SBC[i]);
          K[i] = vbfi(m1, Kn[i], K[i]);
          DMB[i] = vbfi(m1, DMBn, DMB[i]);
        }
      }
    };
    // One step; PH = t & 1 picks the register roles and the LDS record slots,
    // ROLE the wave's place in the lap (0: wave 0, reads the ring; 2: the last
    // wave, writes it; 1: the others), so the loop body has no role branches.
    auto step = [&](auto ph, auto role, int32_t t, auto fin_step) {
      // ph = t & 3 (or -1: slot phase at run time); PH = t & 1 picks the registers
      constexpr int PQ = decltype(ph)::value;
      constexpr int PH = PQ & 1;
      const int32_t q = PQ >= 0 && PQ < 4 ? PQ : (t & 3);  // record slot phase
      constexpr int ROLE = decltype(role)::value & 3;
      // M = 2 with even P: the x = 1 position's register (t - w) mod 2 is
      // PH ^ (w & 1), a compile-time constant for a wave of known parity
      constexpr int WPAR = (decltype(role)::value >> 2) - 1;  // -1: unknown
      constexpr int ISC = (M == 2 && WPAR >= 0) ? (HSK == 2 ? PH : PH ^ WPAR) : -1;
      constexpr bool FIN = decltype(fin_step)::value;  // the last step (t == T-1)
      // this step's A codes (LDS table) and the B code of position x = 1
      uint32_t a[M];
      if constexpr (TSA_A_PREFETCH) {
#pragma unroll
        for (int i = 0; i < M; ++i) a[i] = a_nx[i];
      } else {
        load_a<M>(a_lane + 4u * (uint32_t)xpos0, a);
      }
      // ---- receive the wave-above record of step t-1
      uint4 rec[M];
      if constexpr (ROLE == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(M * (PD - 1)) : "memory");
        const uint8_t *src = xr0 + (t % PD) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
      } else {
        const int off = (HSK == 2 ? (q + 2) & 3 : PH ^ 1) * SLOT_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16_at(rd_base, off + i * PAIR_BYTES);
      }
      uint32_t inIx[M], inIy[M], inIz[M], inIxy[M], inIyz[M], inIxz[M], inM[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        inIx[i] = oIx[i];
        inIy[i] = rec[i].x;
        inIz[i] = shIz[i];
        inIxy[i] = svIxy[i];
        inIyz[i] = svIyz[i];
        inIxz[i] = shIxz[PH][i];
        inM[i] = svM[PH][i];
      }
      // ---- x == 1 at position k* = (t - w) mod P: its x-1 inputs are the x = 0
      // face (EN_i==1&&EN==0 gating, src/PE_1cyc.v:164-178,196-202,212-218), and
      // it starts row lap0*NW+w+1, whose B symbol it takes here.
      if (!PRE && !TSA_ABL_INJ && (TSA_HM_TRACK || xpos0 < KS)) {  // (tracked: hmCur is 0 past KS)
        int32_t ls, is, hs;
        pos_split<M>(xpos0, ls, is, hs);
#if TSA_HM_TRACK
        uint32_t m1;
        // M = 2, skew 2: xpos0 has t's parity, so the odd step of a pair
        // injects the same lane and half as the even one (register 1 after
        // register 0; the half-mask events and the lap wrap fall on even
        // xpos0, between pairs): its mask is the even step's
        if constexpr (MASK_PAIRS && (PQ & 1)) {
          m1 = m1_pair;
        } else {
          asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m1) : "v"(hmCur), "s"(1ull << ls));
          if constexpr (MASK_PAIRS) m1_pair = m1;
        }
#elif TSA_LANE_MASK
        const uint32_t m1 = lane_half_mask(ls, hs, hmLo, hmHi);
#else
        const uint32_t m1 = lane == ls ? (TWO ? 0xFFFFFFFFu : hs ? 0xFFFF0000u : 0x0000FFFFu) : 0u;
#endif
#pragma unroll
        for (int i = 0; i < M; ++i) {
          if (ISC >= 0 ? i == ISC : i == is) {
            if constexpr (VS) {  // faces (0,y,z), (0,y-1,z), (0,y,z-1): lam(y+z-1); (0,y-1,z-1): one lam less
              if constexpr (TSA_H_SALU) {
                inIx[i] = vbfi_s(m1, Hr[PQ & 3], inIx[i]);
                inIxy[i] = vbfi_s(m1, Hr[PQ & 3], inIxy[i]);
                inIxz[i] = vbfi_s(m1, Hr[PQ & 3], inIxz[i]);
                inM[i] = vbfi_s(m1, Hr[(PQ + 3) & 3], inM[i]);
              } else {
                inIx[i] = vbfi(m1, Hr[PQ & 3], inIx[i]);
                inIxy[i] = vbfi(m1, Hr[PQ & 3], inIxy[i]);
                inIxz[i] = vbfi(m1, Hr[PQ & 3], inIxz[i]);
                inM[i] = vbfi(m1, Hr[(PQ + 3) & 3], inM[i]);
              }
            } else {
              inIx[i] = vbfi(m1, fsv, inIx[i]);
              inIxy[i] = vbfi(m1, fpv, inIxy[i]);
              inIxz[i] = vbfi(m1, fpv, inIxz[i]);
              inM[i] = vbfi(m1, zero, inM[i]);
            }
            b[i] = vbfi(m1, binj, b[i]);
            if constexpr (F16) {  // the new row's per-row terms
#if TSA_ROW_NEXT
              SBC[i] = vbfi(m1, SBCn[i], SBC[i]);
              K[i] = vbfi(m1, Kn[i], K[i]);
              if constexpr (VS) DMB[i] = vbfi(m1, DMBn, DMB[i]);
#else
              const uint32_t e01 = pk_eq1(b[i], c[i], one1);
              SBC[i] = pk_mad(e01, sbcv, 0u);
              K[i] = pk_mad(e01, kdv, k0v);
#endif
            }
          }
        }
      }
      // keep the per-row registers in place across the branches above (without
      // this the allocator copies b into a fresh pair every step)
#if TSA_PIN_ROW
#pragma unroll
      for (int i = 0; i < M; ++i) asm volatile("" : "+v"(b[i]), "+v"(SBC[i]), "+v"(K[i]), "+v"(DMB[i]));
#endif
      uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
      // Priority 0 for the cell arithmetic, 1 for the send/shift/barrier tail:
      // VALU issue goes by priority then age, so without this the oldest waves
      // of a SIMD finish each step first and idle at the barrier (+3-4 %).
      if constexpr (TSA_SETPRIO) __builtin_amdgcn_s_setprio(0);
      if constexpr (TSA_SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);  // keep the arithmetic between the two
      if constexpr (VS)
        cell_messages_vs<M, SOP>(a, b, c, SBC, K, DMC, DMB, pv, inIx, inIy, inIz, inIxy, inIyz, inIxz, inM, nIx,
                                 oIy, oIz, oIxy, oIyz, oIxz, oBest);
      else if constexpr (F16)
        cell_messages_f16<M, SOP>(a, b, c, SBC, K, DMC, ones, pv, inIx, inIy, inIz, inIxy, inIyz, inIxz, inM, nIx,
                             oIy, oIz, oIxy, oIyz, oIxz, oBest);
      else
        cell_messages<M, SOP ? 1 : 0>(a, b, c, ones, pv, inIx, inIy, inIz, inIxy, inIyz, inIxz,
                                      inM, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);

      if constexpr (TSA_SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);
      if constexpr (TSA_SETPRIO) __builtin_amdgcn_s_setprio(1);
      // ---- the final cell (src/TriAlign_1cyc.v:141-142,342-345) is in wave w_f's
      // last step; it is read back after the loop
      if constexpr (TWO) {  // two final cells, possibly at different steps
        if (t == t_f && w == w_f) fin[lane] = oBest[0];
        if (t == t_f1 && w == w_f1) fin[64 + lane] = oBest[0];
      } else if constexpr (VS) {  // the four-step loop runs past T: the final step is tested
        if (t == t_fin) {  // (peeling the last group instead trips a gfx950 backend bug)
#pragma unroll
          for (int i = 0; i < M; ++i) fin[i * 64 + lane] = oBest[i];
        }
      } else if constexpr (FIN) {
        if (w == w_f) {
#pragma unroll
          for (int i = 0; i < M; ++i) fin[i * 64 + lane] = oBest[i];
        }
      }

      // ---- send this step's record to the wave below (or the ring)
      if constexpr (ROLE != 2) {
        const int off = (HSK == 2 ? q : PH) * SLOT_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i)
          lds_write16_at(wr_base, off + i * PAIR_BYTES, make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
      } else {
        // Positions that have not started (u = t - w - k < 0) must publish the
        // y = 0 face: wave 0 reads this row as "row y0-1" during its lap 0.
        if (t < ZT + HSK * NW) {
          const int32_t lim = t - HSK * w;  // position k started iff k <= lim
          // VS: wave 0 meets this row at step t + lag, where x + z = t + lag + 2
          const uint32_t fy = VS ? h_bits(pa.lam * (t + lag + 1)) : pa.f_single;
          const uint32_t fp = VS ? h_bits(pa.lam * (t + lag + 2)) : pa.f_pair;
          const uint32_t fb = VS ? fp : 0u;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            const uint32_t m = ((M * lane + i > lim) ? 0x0000FFFFu : 0u) |
                               (((TWO ? 0 : 64 * M) + M * lane + i > lim) ? 0xFFFF0000u : 0u);
            oIy[i] = bfi(m, fy, oIy[i]);
            oIxy[i] = bfi(m, fp, oIxy[i]);
            oIyz[i] = bfi(m, fp, oIyz[i]);
            oBest[i] = bfi(m, fb, oBest[i]);
          }
        }
        uint4 *dst = (uint4 *)__builtin_assume_aligned(
            ring + (int64_t)st_row * SLOT_BYTES + lane * REC_BYTES, 16);
#pragma unroll
        for (int i = 0; i < M; ++i) dst[i * 64] = make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]);
      }
      // ---- advance the systolic registers
#pragma unroll
      for (int i = 0; i < M; ++i) {
        oIx[i] = nIx[i];
        svIxy[i] = rec[i].y;
      }
      uint32_t rz[M], rw[M];
#pragma unroll
      for (int i = 0; i < M; ++i) { rz[i] = rec[i].z; rw[i] = rec[i].w; }
      // position 0 advances to u0 + 1
      // (TSA_EV_STATIC: the events fall on step (2w - 1) mod 4 of a group only)
      constexpr bool EV_SKIP = VS && M == 2 && TSA_EV_STATIC && HSK == 2 && WPAR >= 0 && PQ >= 0 && PQ < 4 &&
                               (PQ & 3) != (WPAR == 0 ? 3 : 1);
      auto advance = [&]() {
#if TSA_HM_TRACK
        if constexpr (EV_SKIP) {
          ++xpos0;
          return;
        }
        if (__builtin_expect(++xpos0 == next_ev, 0)) {
          if (xpos0 == P) {
            xpos0 = 0;
            binj = b_of_lap(++lap0);
            row_terms();
            if constexpr (VS) {  // a new row at position 0: H(t .. t+2) restart
              const int32_t y = lap0 * NW + w + 1;
              if constexpr (TSA_H_SALU) {
                Hq[PQ & 3] = pa.lam * (y - 1);
                Hq[(PQ + 1) & 3] = pa.lam * y;
                Hq[(PQ + 2) & 3] = pa.lam * (y + 1);
                Hr[PQ & 3] = f16x2_int(Hq[PQ & 3]);
                Hr[(PQ + 1) & 3] = f16x2_int(Hq[(PQ + 1) & 3]);
                Hr[(PQ + 2) & 3] = f16x2_int(Hq[(PQ + 2) & 3]);
              } else {
                Hr[PQ & 3] = h_bits(pa.lam * (y - 1));
                Hr[(PQ + 1) & 3] = h_bits(pa.lam * y);
                Hr[(PQ + 2) & 3] = h_bits(pa.lam * (y + 1));
              }
            }
          }
          hmCur = hm_of(xpos0);
          next_ev = ev_of(xpos0);
        }
#else
        static_assert(!VS, "V-space tracks the lap wrap with the half-mask events");
        if (++xpos0 == P) {
          xpos0 = 0;
          binj = b_of_lap(++lap0);
          row_terms();
        }
#endif
      };
      if constexpr (VS) {
        if constexpr (TSA_H_SALU) {
          Hq[(PQ + 2) & 3] = Hq[(PQ + 1) & 3] + pa.lam;
          Hr[(PQ + 2) & 3] = f16x2_int(Hq[(PQ + 2) & 3]);
        } else {
          Hr[(PQ + 2) & 3] = U(H(Hr[(PQ + 1) & 3]) + H(pa.v_lam));
        }
        advance();
        // z = 0 faces of position 0: (x, y, 0) and (x, y-1, 0) at step t+1,
        // (x-1, y, 0) and (x-1, y-1, 0) at step t+2
        if constexpr (TSA_ABL_ZOWN) {
          zmove_abl<M>(shIxz[PH], oIxz);
          zmove_abl<M>(shIz, oIz);
        } else {
          zshift<M>(shIxz[PH], oIxz, sel, Hr[(PQ + 2) & 3]);
          zshift<M>(shIz, oIz, sel, Hr[(PQ + 1) & 3]);
        }
        if constexpr (TSA_ABL_ZREC) {
          zmove_abl<M>(svIyz, rz);
          zmove_abl<M>(svM[PH], rw);
        } else {
          zshift<M>(svIyz, rz, sel, Hr[(PQ + 1) & 3]);
          zshift<M>(svM[PH], rw, sel, Hr[(PQ + 1) & 3]);
        }
        if constexpr (PRE) vs_inject(std::integral_constant<int, (PQ + 1) & 3>{});  // the next step's x = 1
      } else {
        zshift<M>(shIxz[PH], oIxz, sel, pa.f_pair);  // z = 0 face for position 0
        zshift<M>(shIz, oIz, sel, pa.f_single);
        zshift<M>(svIyz, rz, sel, pa.f_pair);
        zshift<M>(svM[PH], rw, sel, 0u);
        advance();
      }
      if constexpr (A_B64) load_a_pair<(PQ & 3) + 1>(abase, abase_s, a_nx);  // x' of step t + 1
      else if constexpr (VS) load_a_off<M>(abase, (PQ & 3) + 1, a_nx);
      else if constexpr (TSA_A_PREFETCH) load_a<M>(a_lane + 4u * (uint32_t)xpos0, a_nx);

      // ---- wave 0: fetch the record of step t + PD into the slot just consumed
      if constexpr (ROLE == 0) {
#pragma unroll
        for (int i = 0; i < M; ++i)
          dma16(ring + ((int64_t)dma_row * M + i) * PAIR_BYTES + lane * REC_BYTES,
                xr0 + (t % PD) * SLOT_BYTES + i * PAIR_BYTES);
        if (++dma_row == R) dma_row = 0;
      }
      if constexpr (ROLE == 2) {
        if (++st_row == R) st_row = 0;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(M * STORE_SLACK) : "memory");
      }
      // skew 2: a wave reads records two steps old, so one barrier per pair of steps
      if constexpr (HSK == 1 || PH == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };

    // the last step is peeled off (it records the final cell), so the loop
    // body carries no final-step test; PH stays t & 1
    auto run = [&](auto role) {
      int32_t t = 0;
      const int32_t T1 = T - 1;
      // P0/P1: t & 1 known, the slot phase t & 3 read at run time (values 4, 5)
      constexpr std::integral_constant<int, 4> P0{};
      constexpr std::integral_constant<int, 5> P1{};
      constexpr std::integral_constant<int, 0> Q0{};
      constexpr std::integral_constant<int, 1> Q1{};
      constexpr std::integral_constant<int, 2> Q2{};
      constexpr std::integral_constant<int, 3> Q3{};
      constexpr std::false_type mid{};
      constexpr std::true_type last{};
      if constexpr (VS) {  // whole groups of four steps (H's phase is t & 3), the final cell tested
#pragma unroll 1
        for (; t < T; t += 4) {
          abase = a_lane + 4u * (uint32_t)xpos0;
          if constexpr (A_B64) abase_s = a_lane_s + 4u * (uint32_t)xpos0;
          TSA_INLINE_IF_WIDE(step(Q0, role, t, mid));
          TSA_INLINE_IF_WIDE(step(Q1, role, t + 1, mid));
          TSA_INLINE_IF_WIDE(step(Q2, role, t + 2, mid));
          TSA_INLINE_IF_WIDE(step(Q3, role, t + 3, mid));
        }
        return;
      }
#if TSA_UNROLL4
#pragma unroll 1
      for (; (M <= 2 || HSK == 2) && t + 3 < T1; t += 4) {
        TSA_INLINE_IF_WIDE(step(Q0, role, t, mid));
        TSA_INLINE_IF_WIDE(step(Q1, role, t + 1, mid));
        TSA_INLINE_IF_WIDE(step(Q2, role, t + 2, mid));
        TSA_INLINE_IF_WIDE(step(Q3, role, t + 3, mid));
      }
#endif
#pragma unroll 1
      for (; t + 1 < T1; t += 2) {
        TSA_INLINE_IF_WIDE(step(P0, role, t, mid));
        TSA_INLINE_IF_WIDE(step(P1, role, t + 1, mid));
      }
      if (t < T1) {
        TSA_INLINE_IF_WIDE(step(P0, role, t, mid));
        TSA_INLINE_IF_WIDE(step(P1, role, t + 1, last));
      } else {
        TSA_INLINE_IF_WIDE(step(P0, role, t, last));
      }
    };
    // role | (w & 1) + 1 << 2 (M = 2, see ISC in step)
    constexpr int W0 = (M == 2 && TSA_IS_STATIC) ? 4 : 0, W1 = (M == 2 && TSA_IS_STATIC) ? 8 : 0;
    static_assert(NW % 2 == 0, "the last wave is odd");
    if constexpr (PRE) vs_inject(std::integral_constant<int, 0>{});  // step 0's x = 1
    if (w == 0) TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 0 + W0>{}));
    else if (w == NW - 1) TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 2 + W1>{}));
    else if (W0 != 0 && (w & 1)) TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 1 + W1>{}));
    else TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 1 + W0>{}));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      auto decode = [&](uint16_t hb) -> int32_t {
        return F16 ? (int32_t)(float)__builtin_bit_cast(_Float16, hb) : (int32_t)(int16_t)hb;
      };
      // VS: the final cell's value sits lam (la + lb + lc) above its score
      const int32_t sh0 = VS ? pa.lam * (la + lb + lc) : 0, sh1 = VS ? pa.lam * (la1 + lb1 + lc1) : 0;
      if constexpr (TWO) {
        scores[tri] = decode((uint16_t)(fin[k_f] & 0xFFFF)) - sh0;
        if (has1) scores[tri + 1] = decode((uint16_t)(fin[64 + k_f1] >> 16)) - sh1;
      } else {
        int32_t l_f, i_f, h_f;
        pos_split<M>(k_f, l_f, i_f, h_f);
        const uint32_t v = fin[i_f * 64 + l_f];
        scores[tri] = decode((uint16_t)(h_f ? (v >> 16) : (v & 0xFFFF))) - sh0;
      }
    }
    __syncthreads();
  }
}

static uint32_t pk16(int32_t v) { return ((uint32_t)(uint16_t)(int16_t)v) * 0x00010001u; }
static uint32_t pkh(double v) {  // both halves = f16(v); v exactly representable
  const _Float16 h = (_Float16)v;
  uint16_t bits;
  memcpy(&bits, &h, 2);
  return (uint32_t)bits * 0x00010001u;
}

PencilArgs make_args(const KParams &kp, bool f16, bool vs) {
  const int32_t GE = kp.pen[SIXY][SIX], GO = kp.pen[SIXY][SM];  // Ixy row: Ix = GE, M = GO
  int32_t fs = -kp.pen[SIX][0], fp = -kp.pen[SIXY][0];
  for (int s = 0; s < 7; ++s) {
    fs = std::max(fs, -kp.pen[SIX][s]);
    fp = std::max(fp, -kp.pen[SIXY][s]);
  }
  PencilArgs a;
  memset(&a, 0, sizeof(a));
  a.sop = kp.s3_mode == TSA_S3_SOP;
  a.packed = kp.packed;
  if (!f16) {
    a.E = pk16(GE);
    a.O = pk16(GO);
    a.E2 = pk16(2 * GE);
    a.OE = pk16(GO + GE);
    a.O2 = pk16(2 * GO);
    a.f_single = pk16(fs);
    a.f_pair = pk16(fp);
    a.dm = pk16(kp.match - kp.mismatch);
    a.mm = pk16(kp.mismatch);
    a.s3_d1 = pk16(kp.s3_eq - kp.s3_ab);
    a.s3_d0 = pk16(kp.s3_ab - kp.s3_ne);
    a.s3_ne = pk16(kp.s3_ne);
    return a;
  }
  const int32_t mm = kp.mismatch;
  a.E = pkh(GE - mm);
  a.O = pkh(GO - mm);
  a.E2 = pkh(2 * GE);
  a.OE = pkh(GO + GE);
  a.O2 = pkh(2 * GO);
  a.f_single = pkh(fs);
  a.f_pair = pkh(fp + mm);
  const int32_t dm = kp.match - mm, d0 = kp.s3_ab - kp.s3_ne, d1 = kp.s3_eq - kp.s3_ab;
  a.h_dm = pkh(dm * 8192.0);
  a.dmf = (float)dm;
  a.h_c3 = pkh((double)kp.s3_ne);
  a.h_sbc = pkh((double)dm);  // SBC = e01 * bits(dm), e01 in {0, 1}
  const uint32_t k0 = a.sop ? pkh(3.0 * mm) : pkh(d0 * 8192.0);
  const uint32_t k1 = a.sop ? pkh(3.0 * mm + dm) : pkh((d0 + d1) * 8192.0);
  a.h_k0 = k0;                // K = k0 + e01 * (k1 - k0), per 16-bit half
  a.h_kd = (((k1 & 0xFFFF) - (k0 & 0xFFFF)) & 0xFFFF) * 0x00010001u;
  if (vs) {  // cell_messages_vs: lam = GE = -mismatch; SOP's K takes the 3 lam of M
    a.lam = GE;
    a.v_lam = pkh(GE);
    a.v_cP = pkh(GO + mm + GE);
    a.v_dO = pkh(GO - GE);
    a.d0f = (float)d0;
    a.d1f = (float)d1;
    if (a.sop) {
      const uint32_t k0v = pkh(3.0 * mm + 3.0 * GE), k1v = pkh(3.0 * mm + dm + 3.0 * GE);
      a.h_k0 = k0v;
      a.h_kd = (((k1v & 0xFFFF) - (k0v & 0xFFFF)) & 0xFFFF) * 0x00010001u;
    }
  }
  return a;
}

// Intermediates of the factored form vs the candidate/state bound: a message
// is a candidate minus its score (|s3| <= 4 sc), the f16 form adds the
// mismatch back (<= sc) and splits the triple score (<= 6 sc); face messages
// sit <= 2 GO below zero. 8 sc + 4 pe covers all of them.
int64_t pencil_slack(int32_t match, int32_t mismatch, int32_t gap_open, int32_t gap_extend) {
  const int64_t sc = std::max(std::llabs(match), std::llabs(mismatch));
  const int64_t pe = std::max(std::llabs(gap_open), std::llabs(gap_extend));
  return 8 * sc + 4 * pe;
}

// Exact-f16 arithmetic applies when every value and intermediate is an integer
// in [-2048, 2048] (value bound +- pencil_slack) and the scaled deltas fit f16.
// TSA_PENCIL_ARITH (A/B and test knob): "i16" forces the int16 form, "f16"
// the f16 form without V-space.
static bool use_f16(const KParams &kp, const Range &r) {
  if (const char *e = getenv("TSA_PENCIL_ARITH"))
    if (!strcmp(e, "i16")) return false;
  auto small = [](int64_t v) { return v >= -7 && v <= 7; };
  auto fits = [](int64_t v) { return v >= -2048 && v <= 2048; };
  const int64_t slack = pencil_slack(kp.match, kp.mismatch, kp.pen[SIXY][SM], kp.pen[SIXY][SIX]);
  return r.lo - slack >= -2048 && r.hi + slack <= 2048 &&
         small((int64_t)kp.match - kp.mismatch) && small((int64_t)kp.s3_ab - kp.s3_ne) &&
         small((int64_t)kp.s3_eq - kp.s3_ab) && small((int64_t)kp.s3_eq - kp.s3_ne) &&
         fits(kp.mismatch) && fits(kp.s3_ne) &&
         fits(3LL * kp.mismatch);
}

// The V-space f16 helix (cell_messages_vs) applies when lam = GE = -MISMATCH
// (the RTL constants: 1), the helix runs M <= 2, and the shifted values stay
// exact f16 integers: bound + lam (LA + LB + LC) + slack <= 2048.
static bool use_vs(const KParams &kp, const Range &r, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  if (const char *e = getenv("TSA_PENCIL_ARITH"))
    if (!strcmp(e, "i16") || !strcmp(e, "f16")) return false;
  const int32_t GE = kp.pen[SIXY][SIX], GO = kp.pen[SIXY][SM];
  if (!use_f16(kp, r) || pencil_pairs(max_lc) > 2 || GE < 1 || GE != -kp.mismatch || GO < GE) return false;
  const PencilGeom g = pencil_geom(max_la, max_lc);
  if (helix_lds(g.M, helix_nw(g.M), g.P, max_lb, true) > LDS_MAX) return false;  // the shifted A copy
  const int64_t slack = pencil_slack(kp.match, kp.mismatch, GO, GE);
  const int64_t hi = r.hi + (int64_t)GE * ((int64_t)max_la + max_lb + max_lc) + slack;
  return r.lo - slack >= -2048 && hi <= 2048 && (int64_t)GO + GE + kp.mismatch <= 2048;
}

// The lap kernel's V-space cell (lap_kernel VS) under the same conditions as
// the helix's, for any tile width: lam = GE = -MISMATCH and the shifted
// values exact f16 integers.
// Opt-in (TSA_LAP_VS=1): measured slower than the message form on MI355X
// (64^3 0.098 vs 0.087 ms, 256^3 0.412 vs 0.389 ms, same box,
// profiles/r4c_lapvs.jsonl) -- the chained lap step is bound by its loader's
// hand-off, not by the cell's instructions, and the V-space faces make lap 0's
// wave 0 wait on its loader, which the message form's constant faces do not.
static bool lap_vs_ok(const KParams &kp, const Range &r, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  const char *on = getenv("TSA_LAP_VS");
  if (!on || atoi(on) == 0) return false;
  if (const char *e = getenv("TSA_PENCIL_ARITH"))
    if (!strcmp(e, "i16") || !strcmp(e, "f16")) return false;
  const int32_t GE = kp.pen[SIXY][SIX], GO = kp.pen[SIXY][SM];
  if (!use_f16(kp, r) || GE < 1 || GE != -kp.mismatch || GO < GE) return false;
  const int64_t slack = pencil_slack(kp.match, kp.mismatch, GO, GE);
  const int64_t hi = r.hi + (int64_t)GE * ((int64_t)max_la + max_lb + max_lc) + slack;
  return r.lo - slack >= -2048 && hi <= 2048 && (int64_t)GO + GE + kp.mismatch <= 2048;
}

template <int M, int NW, bool F16, bool SOP>
static int launch_m(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                    int32_t max_lb, const PencilGeom &g, int32_t *d_scores, void *d_ws,
                    const PencilArgs &pa, hipStream_t stream) {
  constexpr bool VSOK = F16 && M <= 2;  // V-space instantiations
  const bool vs = VSOK && pa.lam != 0;
  const int32_t lds_a = 4 * (g.P + 128 * M + A_PAD), lds_b = 4 * ((max_lb + 3) & ~3);
  const size_t lds = helix_lds(M, NW, g.P, max_lb, vs);
  // TWO (two triples per workgroup) exactly when pencil_geom sized P for it
  const bool two = M == 1 && g.two;
  auto kfn = vs ? (two ? pencil_kernel<M, NW, F16, SOP, M == 1, VSOK> : pencil_kernel<M, NW, F16, SOP, false, VSOK>)
                : (two ? pencil_kernel<M, NW, F16, SOP, M == 1, false> : pencil_kernel<M, NW, F16, SOP, false, false>);
  if (lds > LDS_MAX) return TSA_EINVAL;
  const int32_t units = two ? (n + 1) / 2 : n;
  const int grid = units < 65535 ? units : 65535;
  return launch_with_lds((const void *)kfn, lds, [&] {
           hipLaunchKernelGGL(kfn, dim3(grid), dim3(64 * NW), lds, stream, d_seqs, d_offsets, n, g.P, g.R, lds_a,
                              lds_b, g.ring_bytes_per_triple, (uint8_t *)d_ws, d_scores, pa);
         }) == hipSuccess
             ? TSA_OK
             : TSA_EDEVICE;
}

void pencil_describe(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                     const Range &bound, LapPolicy lap, char *buf, size_t len, bool checked) {
  const bool f16 = checked ? false : use_f16(kp, bound);
  const char *arith = f16 ? "f16" : "i16";
  const char *s3 = kp.s3_mode == TSA_S3_SOP ? "sop" : "rtl";
  const LapGeom lg = lap_choice(n, max_la, max_lb, max_lc, lap, f16, kp.s3_mode == TSA_S3_SOP, checked);
  if (lg.ok) {
    if (f16 && lap_vs_ok(kp, bound, max_la, max_lb, max_lc)) arith = "f16v";  // the lap's V-space cell
    char chunk[32] = "";
    if (lg.chunk > 0) snprintf(chunk, sizeof chunk, " chunk=%d", lg.chunk);
    snprintf(buf, len, "pencil lap %s %s M=%d NW=%d laps=%d tiles=%d waves=%lld wpc=%d%s%s est=%.0fus", arith, s3,
             lg.M, lg.NW, lg.G, lg.GZ, (long long)lg.waves, lg.per_cu, chunk, checked ? " checked" : "", lg.est_us);
    return;
  }
  const PencilGeom g = pencil_geom(max_la, max_lc);
  if (use_vs(kp, bound, max_la, max_lb, max_lc)) arith = "f16v";  // the helix's V-space cell
  snprintf(buf, len, "pencil helix %s %s M=%d NW=%d P=%d%s est=%.0fus", arith, s3, g.M, helix_nw(g.M), g.P,
           g.two ? " two" : "", helix_est(n, max_la, max_lb, max_lc));
}

int pencil_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                        int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                        const Range &bound, int32_t *d_scores, void *d_ws, size_t ws_bytes,
                        hipStream_t stream, LapPolicy lap, int32_t **d_err,
                        const CheckLimits *chk) {
  if (d_err) *d_err = nullptr;
  if (n <= 0) return TSA_OK;
  if (!pencil_shape_ok(max_la, max_lb, max_lc)) return TSA_EINVAL;
  const bool f16 = chk ? false : use_f16(kp, bound);  // the checked kernel runs int16
  const bool sop = kp.s3_mode == TSA_S3_SOP;
  const LapGeom lg = lap_choice(n, max_la, max_lb, max_lc, lap, f16, sop, chk != nullptr);
  if (lg.ok) {
    if (ws_bytes < lap_workspace_bytes(lg)) return TSA_ENOMEM;
    const bool lvs = f16 && lap_vs_ok(kp, bound, max_la, max_lb, max_lc);
    return lap_launch(lg, f16, sop, d_seqs, d_offsets, n, d_scores, d_ws, make_args(kp, f16, lvs), stream,
                      d_err, chk);
  }
  const PencilArgs pa = make_args(kp, f16, !chk && use_vs(kp, bound, max_la, max_lb, max_lc));
  if (chk) return TSA_ERANGE;  // no lap schedule for this batch
  const PencilGeom g = pencil_geom(max_la, max_lc);
  const int32_t grid = n < 65535 ? n : 65535;
  if (ws_bytes < (size_t)grid * (size_t)g.ring_bytes_per_triple) return TSA_ENOMEM;
  return TSA_SHAPES(launch_m, g.M, f16, sop, d_seqs, d_offsets, n, max_lb, g,
                    d_scores, d_ws, pa, stream);
}

// A single cube split over np devices by laps: the lap schedule of this cube
// (whatever the helix would cost), if it has at least np laps.
LapGeom pencil_split_geom(int32_t la, int32_t lb, int32_t lc, const KParams &kp, const Range &bound,
                          int np) {
  LapGeom g{};
  g.ok = false;
  if (np < 1 || !pencil_shape_ok(la, lb, lc)) return g;
  const bool f16 = use_f16(kp, bound), sop = kp.s3_mode == TSA_S3_SOP;
  g = lap_choice(1, la, lb, lc, LAP_RESIDENT, f16, sop, true);
  if (!g.ok || g.G < np) {
    g.ok = false;
    return g;
  }
  // full-length rings: no producer ever waits for its consumer, so a part
  // whose launch queues behind an earlier part (parts sharing a hardware
  // queue) cannot deadlock it -- the only waits point from later parts to
  // earlier ones, which are launched first
  return lap_geom(1, la, lb, lc, g.M, g.NW, true, f16, sop);
}

int pencil_launch_split(const LapGeom &g, const KParams &kp, const Range &bound, const LapPart *parts,
                        int np, int32_t *d_score, uint32_t *d_err) {
  const bool f16 = use_f16(kp, bound);
  const PencilArgs pa = make_args(kp, f16, false);
  return lap_launch_split(g, f16, pa.sop != 0, pa, parts, np, d_score, d_err);
}
#undef TSA_SHAPES
#undef TSA_ARITH

}  // namespace tsa