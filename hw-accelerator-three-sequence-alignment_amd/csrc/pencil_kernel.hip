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

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "pencil_kernel.h"

namespace tsa {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// waves (= DP rows) per lap: 16 (one 1024-thread WG per CU) or 8 (two WGs
// per CU, so one computes while the other waits at its per-step barrier)
constexpr int PENCIL_NW_DEFAULT = 8;
constexpr int STORE_SLACK = 4;     // last wave keeps <= this many steps of stores in flight
constexpr int MAX_LA = 4096, MAX_LB = 4096, MAX_LC = 1024;
constexpr size_t LDS_MAX = 160 * 1024;
// LDS-DMA prefetch distance (steps) of wave 0: helix (ring) and lap (hand-off);
// shorter for wide positions (M pairs per lane) so the record slots fit in LDS
__host__ __device__ constexpr int helix_pd(int M) { return M >= 8 ? 2 : M >= 4 ? 4 : 8; }
#ifndef TSA_LAP_PD  // build-time tuning knobs of the lap hand-off
#define TSA_LAP_PD 4
#endif
#ifndef TSA_LAP_SLACK
#define TSA_LAP_SLACK 1
#endif
#ifndef TSA_LAP_PD1  // M = 1 (measured: 3 beats 2, 4, 6, 8 and 12 at 256^3 and 1024^3)
#define TSA_LAP_PD1 3
#endif
__host__ __device__ constexpr int lap_pd(int M) {
  return M >= 8 ? (TSA_LAP_PD < 3 ? TSA_LAP_PD : 3) : M == 1 ? TSA_LAP_PD1 : TSA_LAP_PD;
}
constexpr int LAP_SLACK = TSA_LAP_SLACK;  // producer steps of row stores in flight
constexpr int REC_BYTES = 16;      // {Iy, Ixy, Iyz, best} packed pairs per lane
#ifndef TSA_A_PREFETCH  // read the next step's A codes before the step barrier
#define TSA_A_PREFETCH 1
#endif
// A/B knobs of the f16 cell (build-time; see scripts/build_variant.sh)
#ifndef TSA_DMC        // a&c match term through a per-position scaled delta (no min)
#define TSA_DMC 1
#endif
#ifndef TSA_VMAX3_ASM  // message maxes as explicit v_pk_maximum3_f16 (measured slower:
#define TSA_VMAX3_ASM 0   // the asm blocks constrain the scheduler more than they save)
#endif
#ifndef TSA_GROUPS     // widened GO+GE groups sharing max(Ix,Iy,Iz)
#define TSA_GROUPS 1
#endif
#ifndef TSA_LANE_MASK  // x = 1 lane mask from a scalar shift (one v_cndmask)
#define TSA_LANE_MASK 1
#endif
#ifndef TSA_ROW_NEXT   // next row's per-row terms precomputed once per lap
#define TSA_ROW_NEXT 1
#endif
#ifndef TSA_PIN_ROW    // pin the per-row registers after the x = 1 block
#define TSA_PIN_ROW 1
#endif
#ifndef TSA_UNROLL4  // helix loop body of four steps instead of two (M <= 2)
#define TSA_UNROLL4 1
#endif
#ifndef TSA_HM_TRACK  // half mask kept in a register, switched at two events per lap
#define TSA_HM_TRACK 1
#endif
#ifndef TSA_SKEW  // helix: steps between waves; 2 = one barrier per two steps
#define TSA_SKEW 2
#endif
// skew and record slots per wave; M >= 4 keeps skew 1 (twice the slots would not fit LDS)
__host__ __device__ constexpr int helix_skew(int M) { return M <= 2 ? TSA_SKEW : 1; }
#ifndef TSA_SETPRIO  // helix: priority 0 for the cell arithmetic, 1 for the tail
#define TSA_SETPRIO 1
#endif
#ifndef TSA_IS_STATIC  // M = 2: the x = 1 register index from the wave parity
#define TSA_IS_STATIC 1
#endif
#ifndef TSA_SCHED_FENCE  // sched_barrier fences around the helix cell arithmetic
#define TSA_SCHED_FENCE 1
#endif
constexpr int RING_EXTRA = 8;

// Packed (both halves) constants. int16 form: two's complement; exact-f16 form
// (helix kernel, F16): f16 bits, pair penalties and f_pair with the mismatch
// folded in, h_* the 2^13-scaled score deltas and h_c3 the triple-score base.
struct PencilArgs {
  uint32_t E, O, E2, OE, O2;    // packed penalties GE, GO, 2GE, GO+GE, 2GO
  uint32_t f_single, f_pair;    // face messages of an all-zero cell
  uint32_t dm, mm;              // match-mismatch, mismatch
  uint32_t s3_d1, s3_d0, s3_ne; // RTL: s3 = ne + eab*(d0 + ebc*d1)
  uint32_t h_dm, h_c3;           // 2^13 (match-mismatch); RTL ne
  uint32_t h_sbc, h_k0, h_kd;     // per-row registers, see cell_messages_f16
  float dmf;                      // match - mismatch (per-position DMC, exact f16)
  int32_t sop;                  // TSA_S3_SOP
};

struct PencilGeom {
  int32_t M;        // pairs per lane
  int32_t P;        // lap period (steps)
  int32_t R;        // ring rows
  bool two;         // two triples per workgroup (LC <= 64, M = 1)
  int64_t ring_bytes_per_triple;
};

// positions per lane: M packed pairs cover LC <= 128*M (1, 2, 4 or 8)
static inline int32_t pencil_pairs(int32_t max_lc) {
  return max_lc <= 128 ? 1 : max_lc <= 256 ? 2 : max_lc <= 512 ? 4 : 8;
}
// waves per CU the VGPR budget allows: 4 per SIMD up to M = 2, 2 beyond
static int waves_per_cu(int M) { return M >= 4 ? 8 : 16; }

// Helix rows per workgroup: 8 (two WGs per CU) or 16; M >= 4 always 8.
static int helix_nw(int M) {
  if (M >= 4) return 8;
  if (const char *e = getenv("TSA_PENCIL_NW")) return atoi(e) == 16 ? 16 : 8;  // tuning knob
  return PENCIL_NW_DEFAULT;
}
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
  g.R = g.P + RING_EXTRA;
  g.ring_bytes_per_triple = (int64_t)g.R * g.M * 64 * REC_BYTES;
  return g;
}
static size_t helix_lds(int M, int NW, int32_t P, int32_t max_lb) {
  return (size_t)(NW - 1) * 2 * helix_skew(M) * M * 1024 + (size_t)helix_pd(M) * M * 1024 +
         4 * ((size_t)P + 128 * M) + 4 * (((size_t)max_lb + 3) & ~(size_t)3) + (size_t)M * 512;
}

// The factored messages widen each target's highest-penalty group to all seven
// states, exact only when gap_open >= gap_extend (cell_messages_f16).
bool pencil_supported(const tsa_params *p) { return p != nullptr && p->gap_open >= p->gap_extend; }

static bool pencil_shape_ok(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  if (!(max_la >= 1 && max_la <= MAX_LA && max_lb >= 1 && max_lb <= MAX_LB && max_lc >= 1 &&
        max_lc <= MAX_LC))
    return false;
  const PencilGeom g = pencil_geom(max_la, max_lc);
  return helix_lds(g.M, helix_nw(g.M), g.P, max_lb) <= LDS_MAX;  // the helix is always runnable
}

// Lap-parallel mode (pencil_lap_kernel) for small batches: every (lap, z-tile)
// of every triple gets its own resident workgroup.
// Rows per lap (waves per workgroup): fewer rows = shorter steps but more laps,
// each adding a hand-off lag. Tuning knob TSA_LAP_NW (8/16; M >= 4: 8).
constexpr int LAP_NW_DEFAULT = 16;
static int lap_nw(int M) {
  if (M >= 4) return 8;
  if (const char *e = getenv("TSA_LAP_NW")) return atoi(e) == 8 ? 8 : 16;
  return LAP_NW_DEFAULT;
}
constexpr int LAP_ZRING = 16;  // = ZRING in the kernel
static size_t lap_zrec(int NW) { return (((size_t)NW + 1) * 16 + 63) & ~(size_t)63; }
static size_t lap_lds(int M, int NW, int32_t max_la) {
  const int ZT = 128 * M;
  return (size_t)(NW - 1) * 2 * M * 1024 + (size_t)lap_pd(M) * M * 1024 +
         (4 + LAP_ZRING) * lap_zrec(NW) + 2 * (size_t)lap_pd(M) * 4 + (size_t)M * 256 +
         4 * (((size_t)max_la + NW + 2 * ZT + 3) & ~(size_t)3);
}
// waves per CU for the lap kernel (M = 1 stays under 64 VGPRs: 8 waves per SIMD)
static int lap_waves_per_cu(int M) { return M == 1 ? 32 : M == 2 ? 16 : 8; }
struct LapGeom {
  int32_t M, NW, G, GZ, YR;
  size_t lds, zrec, yf_bytes, zf_bytes, flag_bytes;
  int64_t waves;  // grid / resident slots: 1 = every workgroup resident at once
  bool ok;        // feasible (LDS) and more than one workgroup per triple
};
static LapGeom lap_geom_m(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, int M) {
  LapGeom g;
  g.M = M;
  g.NW = lap_nw(M);
  g.G = (max_lb + g.NW - 1) / g.NW;
  g.GZ = (max_lc + 128 * M - 1) / (128 * M);
  g.YR = max_la + 128 * M + g.NW + 16;
  g.lds = lap_lds(M, g.NW, max_la);
  g.zrec = lap_zrec(g.NW);
  const size_t wgs = (size_t)n * g.G * g.GZ;
  g.yf_bytes = wgs * g.YR * M * 64 * REC_BYTES;
  g.zf_bytes = g.GZ > 1 ? wgs * g.YR * g.zrec : 0;
  g.flag_bytes = ((wgs + 1) * sizeof(int32_t) + 255) & ~(size_t)255;
  const int64_t per_cu =
      g.lds > LDS_MAX ? 0 : std::min<int64_t>(LDS_MAX / g.lds, lap_waves_per_cu(M) / g.NW);
  g.waves = per_cu > 0 ? ((int64_t)wgs + 256 * per_cu - 1) / (256 * per_cu) : 0;
  g.ok = per_cu > 0 && (g.G >= 2 || g.GZ >= 2);
  return g;
}

// Cost model for the mode choice, in M = 2 step units. Measured single-workgroup
// step times: 0.56 us (M = 1), 0.88 us (M = 2); a lap or tile hand-off adds
// ~LAP_LAG steps of flag and DMA latency to the chain.
static double step_cost(int M) { return M == 1 ? 0.62 : M == 2 ? 1.0 : M == 4 ? 1.7 : 3.4; }
constexpr int LAP_LAG = 30;
// A grid beyond the resident slots runs in dispatch waves that barely overlap
// (a triple's later laps wait for slots its earlier laps free): calibrated at
// 256^3, 32 triples 3.0 ms vs helix 6.0 ms, 64 triples 6.2 vs 5.3 ms, so each
// wave costs ~2.8x its chain and streaming is limited to a few waves.
constexpr int64_t LAP_MAX_WAVES = 3;
static double lap_est(const LapGeom &g, int32_t max_la) {
  const double T = max_la + g.NW + 128 * g.M;
  const double chain = (double)(g.G - 1) * (g.NW + LAP_LAG) + (double)(g.GZ - 1) * (128 * g.M + LAP_LAG);
  return (g.waves <= 1 ? chain + T : 2.8 * g.waves * (chain + T)) * step_cost(g.M);
}
static double helix_est(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  const PencilGeom g = pencil_geom(max_la, max_lc);
  const int nw = helix_nw(g.M);
  const int64_t per_cu = std::max<int64_t>(
      1, std::min<int64_t>(LDS_MAX / helix_lds(g.M, nw, g.P, max_lb), waves_per_cu(g.M) / nw));
  const double T = (double)((max_lb - 1) / nw) * g.P + max_la + nw + max_lc;
  const int64_t units = g.two ? (n + 1) / 2 : n;
  return (double)((units + 256 * per_cu - 1) / (256 * per_cu)) * T * step_cost(g.M);
}

// The lap kernel's geometry if it should run, else .ok = false (helix).
// Resident grids (waves == 1) are always safe: a spinning consumer never blocks
// its producer. With stream_ok the grid may exceed the resident slots: producers
// always have lower block indices than their consumers, so with blocks dispatched
// in order (observed, not promised by HIP) a consumer's producer is running or
// done; spins are bounded and the caller checks the error word and falls back.
static LapGeom lap_choice(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                          bool stream_ok) {
  LapGeom none;
  none.ok = false;
  const char *mode = getenv("TSA_PENCIL_MODE");
  if (mode && !strcmp(mode, "helix")) return none;
  const bool force = mode && !strcmp(mode, "lap");
  const int m_lc = pencil_pairs(max_lc);  // one tile covers all of LC
  int m_lo = 1, m_hi = m_lc;
  if (const char *e = getenv("TSA_LAP_ZT")) {  // tuning knob: force the tile width
    const int zt = atoi(e);
    m_lo = m_hi = std::min(zt <= 128 ? 1 : zt <= 256 ? 2 : zt <= 512 ? 4 : 8, m_lc);
  }
  LapGeom best = none;
  double best_est = 0;
  for (int M = m_lo; M <= m_hi; M *= 2) {
    const LapGeom g = lap_geom_m(n, max_la, max_lb, max_lc, M);
    if (!g.ok || (g.waves > 1 && !stream_ok) || g.waves > LAP_MAX_WAVES) continue;
    const double e = lap_est(g, max_la);
    if (!best.ok || e < best_est) { best = g; best_est = e; }
  }
  if (best.ok && !force && best_est >= helix_est(n, max_la, max_lb, max_lc)) return none;
  return best;
}

size_t pencil_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                              bool stream_ok) {
  if (!pencil_shape_ok(max_la, max_lb, max_lc)) return 0;
  const size_t helix = (size_t)std::min<int32_t>(n, 65535) *
                       (size_t)pencil_geom(max_la, max_lc).ring_bytes_per_triple;
  const LapGeom g = lap_choice(n, max_la, max_lb, max_lc, stream_ok);
  if (g.ok) return std::max(helix, g.flag_bytes + g.yf_bytes + g.zf_bytes);
  return helix;
}

bool pencil_shape_supported(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  return pencil_shape_ok(max_la, max_lb, max_lc);
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, a),
                                                                __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
// v_pk_mad_u16 / v_pk_min_u16 written as asm: left to itself hipcc rewrites
// min(x,1)*d+c into per-half compares and selects (6 ops instead of 2).
__device__ __forceinline__ uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// per-half (a & b) != 0 -> 1 / 0 (one-hot symbols). `ones` = 0x00010001 in a
// VGPR: a VOP3P inline constant would feed 0 to the high half.
__device__ __forceinline__ uint32_t pk_eq1(uint32_t a, uint32_t b, uint32_t ones) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a & b), "v"(ones));
  return r;
}
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) {
  return (mask & a) | (~mask & b);
}
// one v_bfi_b32 (hipcc otherwise splits a group of bfi's with a shared mask
// into v_not + v_and + v_and_or)
__device__ __forceinline__ uint32_t vbfi(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
  return r;
}
// One LDS-DMA of 16 B per lane: LDS[m0 + lane*16] <- *gsrc (sc1: bypass L1).
// Issued from inline asm so that hipcc does not treat it as an in-flight LDS
// write and drain vmcnt(0) before every ds_read of the step loop; the
// consumer waits for it with an explicit counted s_waitcnt vmcnt
// (cdna_hip_programming.md 5.7: M0 must be set in the same statement).
__device__ __forceinline__ void dma16(const void *gsrc, const void *lds_dst) {
  unsigned keep;
  const unsigned dst = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)lds_dst;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off sc1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(dst))
      : "memory");
}
// 4-byte LDS-DMA from lane 0 only (the caller guards with lane == 0).
__device__ __forceinline__ void dma4(const void *gsrc, const void *lds_dst) {
  unsigned keep;
  const unsigned dst = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)lds_dst;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off sc1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(dst))
      : "memory");
}
// 16-byte LDS record read as one ds_read_b128 (lane-contiguous, conflict
// free). Through a generic pointer hipcc splits it into two ds_read2_b32
// with a 16 B lane stride, a 4-way bank conflict (SQ_LDS_BANK_CONFLICT).
typedef unsigned u32x4_lds __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 lds_read16(const uint8_t *p) {
  const __attribute__((address_space(3))) u32x4_lds *q =
      (const __attribute__((address_space(3))) u32x4_lds *)(const __attribute__((address_space(3))) void *)p;
  const u32x4_lds v = *q;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lds_write16(uint8_t *p, uint4 v) {
  __attribute__((address_space(3))) u32x4_lds *q =
      (__attribute__((address_space(3))) u32x4_lds *)(__attribute__((address_space(3))) void *)p;
  *q = (u32x4_lds){v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint32_t ror1(uint32_t v) {  // lane l <- lane l-1, lane 0 <- lane 63
  // mov_dpp (old = undef): wave_ror:1 reads a valid lane for every lane
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, false);
}

// One step of M packed cell pairs: scores (src/PE_1cyc.v:159-162) on one-hot
// symbols, the 7 states, and the 7 outgoing messages max_s(S[s] - P[T][s])
// (src/PE_1cyc.v:164-218) grouped by equal penalty; oBest = MAX7 of the states.
template <int M, int SOPM = -1>  // SOPM: 0 RTL, 1 SOP, -1 read pa.sop
__device__ __forceinline__ void cell_messages(
    const uint32_t (&a)[M], const uint32_t (&b)[M], const uint32_t (&c)[M], uint32_t ones,
    const PencilArgs &pa, const uint32_t (&inIx)[M], const uint32_t (&inIy)[M],
    const uint32_t (&inIz)[M], const uint32_t (&inIxy)[M], const uint32_t (&inIyz)[M],
    const uint32_t (&inIxz)[M], const uint32_t (&inM)[M], uint32_t (&nIx)[M], uint32_t (&oIy)[M],
    uint32_t (&oIz)[M], uint32_t (&oIxy)[M], uint32_t (&oIyz)[M], uint32_t (&oIxz)[M],
    uint32_t (&oBest)[M]) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const uint32_t eab = pk_eq1(a[i], b[i], ones);
    const uint32_t eac = pk_eq1(a[i], c[i], ones);
    const uint32_t ebc = pk_eq1(b[i], c[i], ones);
    const uint32_t s2ab = pk_mad(eab, pa.dm, pa.mm);
    const uint32_t s2ac = pk_mad(eac, pa.dm, pa.mm);
    const uint32_t s2bc = pk_mad(ebc, pa.dm, pa.mm);
    uint32_t s3;
    if (SOPM < 0 ? pa.sop != 0 : SOPM == 1) s3 = pk_add(pk_add(s2ab, s2bc), s2ac);
    else s3 = pk_mad(eab, pk_mad(ebc, pa.s3_d1, pa.s3_d0), pa.s3_ne);
    const uint32_t sM = pk_add(inM[i], s3);
    const uint32_t sX = inIx[i], sY = inIy[i], sZ = inIz[i];
    const uint32_t sXY = pk_add(inIxy[i], s2ab);
    const uint32_t sYZ = pk_add(inIyz[i], s2bc);
    const uint32_t sXZ = pk_add(inIxz[i], s2ac);
    // two-input maxes only (no packed int16 max3): pairs shared between groups
    const uint32_t pYZ = pk_max(sY, sZ), pXZ = pk_max(sX, sZ), pXY = pk_max(sX, sY);
    const uint32_t qXY_XZ = pk_max(sXY, sXZ), qXY_YZ = pk_max(sXY, sYZ), qYZ_XZ = pk_max(sYZ, sXZ);
    const uint32_t A1 = pk_max(pYZ, qXY_XZ);  // Ix  <- {Iy,Iz,Ixy,Ixz} at GO+GE
    const uint32_t A2 = pk_max(pXZ, qXY_YZ);  // Iy  <- {Ix,Iz,Ixy,Iyz}
    const uint32_t A3 = pk_max(pXY, qYZ_XZ);  // Iz  <- {Ix,Iy,Iyz,Ixz}
    const uint32_t C1 = pk_max(pXY, sXY);     // Ixy <- {Ix,Iy,Ixy} at GE
    const uint32_t C2 = pk_max(pYZ, sYZ);     // Iyz <- {Iy,Iz,Iyz}
    const uint32_t C3 = pk_max(pXZ, sXZ);     // Ixz <- {Ix,Iz,Ixz}
    // GO >= GE: the highest-penalty group of every target may be widened to
    // all 7 states (see cell_messages_f16), so it is the MAX7 minus one penalty
    const uint32_t best = pk_max(pk_max(A1, A2), sM);  // A1 | A2 = the six gap states
    const uint32_t bO = pk_sub(best, pa.O), bO2 = pk_sub(best, pa.O2);
    oBest[i] = best;
    nIx[i] = pk_max(pk_max(pk_sub(sX, pa.E2), pk_sub(A1, pa.OE)), bO2);
    oIy[i] = pk_max(pk_max(pk_sub(sY, pa.E2), pk_sub(A2, pa.OE)), bO2);
    oIz[i] = pk_max(pk_max(pk_sub(sZ, pa.E2), pk_sub(A3, pa.OE)), bO2);
    oIxy[i] = pk_max(pk_sub(C1, pa.E), bO);
    oIyz[i] = pk_max(pk_sub(C2, pa.E), bO);
    oIxz[i] = pk_max(pk_sub(C3, pa.E), bO);
  }
}

// The pk_mad operands must be VGPRs (inline asm "v"): pin them once, or hipcc
// re-materialises them from SGPRs with a v_mov before every use.
__device__ __forceinline__ PencilArgs pin_score_consts(const PencilArgs &pa) {
  PencilArgs r = pa;
  asm volatile("" : "+v"(r.dm), "+v"(r.mm), "+v"(r.s3_d1), "+v"(r.s3_d0), "+v"(r.s3_ne));
  return r;
}

// ---------------------------------------------------------------------------
// Exact-f16 arithmetic for the helix kernel. Every DP value is an integer; when
// the host proves all of them (and every candidate) lie in [-2048, 2048]
// (trialign_api.hip:pencil_exact), IEEE f16 add/fma/maximum on them are exact,
// and CDNA4's v_pk_maximum3_f16 folds two packed maxes into one instruction.
// Symbol codes are one-hot at bits 11..14 (0x800 << s), so min_u16(a & b, 0x800)
// is 0x0800 = f16 2^-13 on a match and 0 otherwise; the match-mismatch deltas
// are pre-scaled by 2^13 so a single v_pk_fma_f16 adds a pair score. The
// mismatch score of each pair target is folded into the penalties its
// messages carry (Ep = GE - mismatch, Op = GO - mismatch, and f_pair).
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 H(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ uint32_t U(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 hmax(h2 a, h2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ h2 hmax3(h2 a, h2 b, h2 c) { return hmax(hmax(a, b), c); }
// One v_pk_maximum3_f16 exactly: left to itself the compiler CSEs the shared
// two-input maxes of the message groups and then cannot fuse them into max3s.
__device__ __forceinline__ h2 vmax3(h2 a, h2 b, h2 c) {
#if TSA_VMAX3_ASM
  h2 r;
  asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return hmax3(a, b, c);
#endif
}
__device__ __forceinline__ h2 hfma(h2 a, h2 b, h2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ uint32_t umin2(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(us2, a),
                                                                 __builtin_bit_cast(us2, b)));
}
constexpr uint32_t SYM0 = 0x800u;  // helix symbol codes: SYM0 << s
// Per half: f16(dm / f16value(code)) for a one-hot code (a power of two:
// 2^-13, 2^-11, 2^-7 or 2), 0 for code 0 (padding); exact for |dm| <= 7.
__device__ __forceinline__ uint32_t dm_over_code(float dm, uint32_t codes) {
  uint32_t r = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint16_t c = (uint16_t)(codes >> (16 * h));
    if (c != 0) {
      const _Float16 v = (_Float16)(dm / (float)__builtin_bit_cast(_Float16, c));
      r |= (uint32_t)__builtin_bit_cast(uint16_t, v) << (16 * h);
    }
  }
  return r;
}

// Terms that depend only on (b, c) are per-position constants for a whole row
// (b changes when a position starts a new row at x = 1), kept in registers:
//   SBC = dm*[b=c]                       (f16) added to the Iyz input
//   K   = RTL: 2^13 (d0 + d1*[b=c])      fma multiplier of [a=b] for M
//         SOP: 3 mismatch + dm*[b=c]     added to the M input
template <int M, bool SOP>
__device__ __forceinline__ void cell_messages_f16(
    const uint32_t (&a)[M], const uint32_t (&b)[M], const uint32_t (&c)[M],
    const uint32_t (&SBC)[M], const uint32_t (&K)[M], const uint32_t (&DMC)[M], uint32_t Q,
    const PencilArgs &pa,
    const uint32_t (&inIx)[M], const uint32_t (&inIy)[M], const uint32_t (&inIz)[M],
    const uint32_t (&inIxy)[M], const uint32_t (&inIyz)[M], const uint32_t (&inIxz)[M],
    const uint32_t (&inM)[M], uint32_t (&nIx)[M], uint32_t (&oIy)[M], uint32_t (&oIz)[M],
    uint32_t (&oIxy)[M], uint32_t (&oIyz)[M], uint32_t (&oIxz)[M], uint32_t (&oBest)[M]) {
  const h2 DM = H(pa.h_dm), E = H(pa.E), O = H(pa.O), E2 = H(pa.E2), OE = H(pa.OE), O2 = H(pa.O2);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    // a & c is c's code (a power of two) on a match, 0 otherwise, and
    // DMC = (match - mismatch) / code(c) per position: the product is exact
#if TSA_DMC
    const h2 eab = H(umin2(a[i] & b[i], Q)), eac = H(a[i] & c[i]);
    const h2 DMCi = H(DMC[i]);
#else
    const h2 eab = H(umin2(a[i] & b[i], Q)), eac = H(umin2(a[i] & c[i], Q));
    const h2 DMCi = DM;
#endif
    const h2 sXY = hfma(eab, DM, H(inIxy[i]));  // src/PE_1cyc.v:159-161 (+mismatch folded)
    const h2 sXZ = hfma(eac, DMCi, H(inIxz[i]));
    const h2 sYZ = H(inIyz[i]) + H(SBC[i]);
    h2 sM;                                       // src/PE_1cyc.v:162
    if constexpr (SOP) sM = hfma(eab, DM, hfma(eac, DMCi, H(inM[i]))) + H(K[i]);
    else sM = hfma(eab, H(K[i]), H(inM[i])) + H(pa.h_c3);  // ne + [a=b](d0 + [b=c] d1)
    const h2 sX = H(inIx[i]), sY = H(inIy[i]), sZ = H(inIz[i]);
    // With GO >= GE (pencil_supported) a penalty group may take in any state
    // that already reaches the target at a penalty no larger (2GE <= GO+GE <=
    // 2GO, GE <= GO): each single target's GO+GE group takes in the target's
    // own state, so the three share max(Ix,Iy,Iz); each target's highest
    // group ({M,Iyz} at 2GO for Ix, {M,Iz,Iyz,Ixz} at GO for Ixy, ...) takes in
    // all 7, so it is MAX7 - penalty, shared by all six gap targets.
#if TSA_GROUPS
    // vmax3(a, b, c) = max(max(a, b), c): the inner pairs are all distinct, so
    // the compiler cannot CSE one and fuses every pair into one max3
    const h2 S3 = vmax3(sX, sY, sZ);
    const h2 A1 = vmax3(S3, sXY, sXZ);   // Ix  <- {Iy,Iz,Ixy,Ixz} (+Ix) at GO+GE
    const h2 A2 = vmax3(S3, sYZ, sXY);   // Iy  <- {Ix,Iz,Ixy,Iyz} (+Iy)
    const h2 A3 = vmax3(sYZ, sXZ, S3);   // Iz  <- {Ix,Iy,Iyz,Ixz} (+Iz)
    const h2 C1 = vmax3(sX, sXY, sY);    // Ixy <- {Ix,Iy,Ixy} at GE
    const h2 C2 = vmax3(sY, sYZ, sZ);
    const h2 C3 = vmax3(sZ, sXZ, sX);
    const h2 best = vmax3(A1, sYZ, sM);  // A1 | Iyz = the six gap states
#else
    const h2 pYZ = hmax(sY, sZ), pXZ = hmax(sX, sZ), pXY = hmax(sX, sY);
    const h2 A1 = hmax3(pYZ, sXY, sXZ), A2 = hmax3(pXZ, sXY, sYZ), A3 = hmax3(pXY, sYZ, sXZ);
    const h2 C1 = hmax(pXY, sXY), C2 = hmax(pYZ, sYZ), C3 = hmax(pXZ, sXZ);
    const h2 best = hmax3(A1, A2, sM);
#endif
    const h2 bO = best - O, bO2 = best - O2;
    oBest[i] = U(best);
    nIx[i] = U(vmax3(sX - E2, A1 - OE, bO2));
    oIy[i] = U(vmax3(sY - E2, A2 - OE, bO2));
    oIz[i] = U(vmax3(sZ - E2, A3 - OE, bO2));
    oIxy[i] = U(vmax3(C1 - E, bO, bO));
    oIyz[i] = U(vmax3(C2 - E, bO, bO));
    oIxz[i] = U(vmax3(C3 - E, bO, bO));
  }
}

// Shift a packed per-position value one position up the helix (k <- k-1).
// With k = 64M*h + M*lane + i, register i >= 1 takes register i-1 of the same
// lane (a rename, no instruction); register 0 takes register M-1 of lane-1
// (one DPP wave_ror:1), except lane 0: its low half is position 0 and gets the
// z = 0 face, its high half (position 64M) takes the low half of lane 63's
// register M-1 -- one v_perm with a per-lane selector does both.
// Only lane 0 reads the second v_perm source (its selector takes bytes 2..3 of
// it), so that source is `face`, whose high half is the z = 0 face (or, for a
// z-tile, the previous tile's last position) -- no extra v_bfi.
template <int M>
__device__ __forceinline__ void zshift(uint32_t (&v)[M], const uint32_t (&src)[M], uint32_t sel,
                                       uint32_t face) {
  const uint32_t r = ror1(src[M - 1]);
#pragma unroll
  for (int i = M - 1; i >= 1; --i) v[i] = src[i - 1];
  v[0] = __builtin_amdgcn_perm(r, face, sel);
}
// A codes of a lane's M registers: entries va, va-4, ... of the LDS table
// (register i holds position M*lane+i, one x behind register i-1).
template <int M>
__device__ __forceinline__ void load_a(uint32_t va, uint32_t (&a)[M]) {
#pragma unroll
  for (int i = 0; i < M; ++i)
    a[i] = *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t)(
        va + 4u * (uint32_t)(M - 1 - i));
}
// bfi mask selecting one half (hs) of one lane (ls): the lane bit comes from a
// scalar shift, so this is one VALU op (v_cndmask with an SGPR-pair mask);
// the two asm strings differ so the compiler does not merge them into one
// with a VALU-selected operand.
__device__ __forceinline__ uint32_t lane_half_mask(int32_t ls, int32_t hs, uint32_t hmLo,
                                                   uint32_t hmHi) {
  const uint64_t lm = 1ull << ls;
  uint32_t m;
  if (hs) asm("v_cndmask_b32_e64 %0, 0, %1, %2 ; hi" : "=v"(m) : "v"(hmHi), "s"(lm));
  else asm("v_cndmask_b32_e64 %0, 0, %1, %2 ; lo" : "=v"(m) : "v"(hmLo), "s"(lm));
  return m;
}
// Position k -> (lane, register, half) of the layout above.
template <int M>
__device__ __forceinline__ void pos_split(int32_t k, int32_t &l, int32_t &i, int32_t &h) {
  const uint32_t u = (uint32_t)k;  // k >= 0: shifts and masks only (M is a power of 2)
  h = (int32_t)(u / (64u * M));
  l = (int32_t)((u / M) & 63u);
  i = (int32_t)(u % M);
}

// The step lambdas are left to the regular inliner for M <= 2 (an early forced
// inline costs ~7 % there); for M >= 4 the inliner gives up on their size and
// the captured state would spill to scratch, so those calls are forced inline.
#define TSA_INLINE_IF_WIDE(call)                 \
  do {                                           \
    if constexpr (M >= 4) {                      \
      [[clang::always_inline]] call;             \
    } else {                                     \
      call;                                      \
    }                                            \
  } while (0)

// ---------------------------------------------------------------------------
// Helix kernel: one workgroup per triple (grid-stride over the batch).
//   LDS: xr  [NW-1][2][M][64][16]  wave w -> w+1 records {Iy, Ixy, Iyz, best}
//        xr0 [PD][M][64][16]       ring rows prefetched for wave 0 (LDS-DMA), PD = helix_pd(M)
//        sA2 [P+ZT] u32            A codes for positions k and k+64 of one pair
//        sB  [LB] u32              B code, both halves
//        fin [M][64] u32           best of the final step (wave w_f)
// F16 selects the exact-f16 arithmetic above, else the int16 form.
template <int M, int NW, bool F16, bool SOP, bool TWO>
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

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  static_assert(!TWO || M == 1, "two triples per wave: 64 positions, M = 1");
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
    for (int j = threadIdx.x; j < P + ZT; j += 64 * NW) {
      const int x0 = ((j - ZT) % P + P) % P, x1 = TWO ? x0 : ((j - ZT - 64 * M) % P + P) % P;
      const uint32_t c0 = x0 < la ? SYM0 << (seqs[o0 + x0] & 3) : 0u;
      const uint32_t c1 = x1 < la1 ? SYM0 << (seqs[(TWO ? q0 : o0) + x1] & 3) : 0u;
      sA2[j] = c0 | (c1 << 16);
    }
    for (int i = threadIdx.x; i < lbm; i += 64 * NW) {
      if constexpr (TWO)
        sB[i] = (i < lb ? SYM0 << (seqs[o1 + i] & 3) : 0u) |
                ((i < lb1 ? SYM0 << (seqs[q1 + i] & 3) : 0u) << 16);
      else
        sB[i] = (SYM0 << (seqs[o1 + i] & 3)) * 0x00010001u;
    }
    {
      const uint4 face = make_uint4(pa.f_single, pa.f_pair, pa.f_pair, 0u);
      const int64_t n16 = (int64_t)R * M * 64;
      for (int64_t i = threadIdx.x; i < n16; i += 64 * NW) ((uint4 *)ring)[i] = face;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- per-position registers (arrays [2] alternate roles between even/odd steps)
    uint32_t b[M], c[M], SBC[M], K[M], DMC[M];
    uint32_t oIx[M], shIz[M], svIxy[M], svIyz[M], shIxz[2][M], svM[2][M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int k0 = M * lane + i, k1 = TWO ? k0 : 64 * M + M * lane + i;
      const uint32_t c0 = k0 < lc ? SYM0 << (seqs[o2 + k0] & 3) : 0u;
      const uint32_t c1 = k1 < lc1 ? SYM0 << (seqs[(TWO ? q2 : o2) + k1] & 3) : 0u;
      c[i] = c0 | (c1 << 16);
      DMC[i] = dm_over_code(pa.dmf, c[i]);
      b[i] = SBC[i] = K[i] = 0;  // set when a position reaches x = 1 of its lap
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
    uint32_t SBCn[M], Kn[M];
    auto row_terms = [&]() {
      if constexpr (F16 && TSA_ROW_NEXT) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const uint32_t e01 = pk_eq1(binj, c[i], one1);
          SBCn[i] = pk_mad(e01, sbcv, 0u);
          Kn[i] = pk_mad(e01, kdv, k0v);
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

    // wave 0: prime the LDS-DMA pipeline (ring row of step s = s - P + NW - 1)
    const int32_t lag = P - HSK * (NW - 1);
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
        const uint8_t *src = xr + ((w - 1) * HNSL + (HSK == 2 ? (q + 2) & 3 : PH ^ 1)) * SLOT_BYTES +
                             lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
      }
      uint32_t inIx[M], inIy[M], inIz[M], inIxy[M], inIyz[M], inIxz[M], inM[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        inIx[i] = oIx[i];
#ifdef TSA_EXP_NOREC  // timing experiment only: wrong results
        inIy[i] = oIx[i] ^ 1u;
#else
        inIy[i] = rec[i].x;
#endif
        inIz[i] = shIz[i];
        inIxy[i] = svIxy[i];
        inIyz[i] = svIyz[i];
        inIxz[i] = shIxz[PH][i];
        inM[i] = svM[PH][i];
      }
      // ---- x == 1 at position k* = (t - w) mod P: its x-1 inputs are the x = 0
      // face (EN_i==1&&EN==0 gating, src/PE_1cyc.v:164-178,196-202,212-218), and
      // it starts row lap0*NW+w+1, whose B symbol it takes here.
      if (TSA_HM_TRACK || xpos0 < KS) {  // (tracked: hmCur is 0 past KS)
        int32_t ls, is, hs;
        pos_split<M>(xpos0, ls, is, hs);
#if TSA_HM_TRACK
        uint32_t m1;
        asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m1) : "v"(hmCur), "s"(1ull << ls));
#elif TSA_LANE_MASK
        const uint32_t m1 = lane_half_mask(ls, hs, hmLo, hmHi);
#else
        const uint32_t m1 = lane == ls ? (TWO ? 0xFFFFFFFFu : hs ? 0xFFFF0000u : 0x0000FFFFu) : 0u;
#endif
#pragma unroll
        for (int i = 0; i < M; ++i) {
          if (ISC >= 0 ? i == ISC : i == is) {
            inIx[i] = vbfi(m1, fsv, inIx[i]);
            inIxy[i] = vbfi(m1, fpv, inIxy[i]);
            inIxz[i] = vbfi(m1, fpv, inIxz[i]);
            inM[i] = vbfi(m1, zero, inM[i]);
            b[i] = vbfi(m1, binj, b[i]);
            if constexpr (F16) {  // the new row's per-row terms
#if TSA_ROW_NEXT
              SBC[i] = vbfi(m1, SBCn[i], SBC[i]);
              K[i] = vbfi(m1, Kn[i], K[i]);
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
      for (int i = 0; i < M; ++i) asm volatile("" : "+v"(b[i]), "+v"(SBC[i]), "+v"(K[i]));
#endif
      uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
      // Priority 0 for the cell arithmetic, 1 for the send/shift/barrier tail:
      // VALU issue goes by priority then age, so without this the oldest waves
      // of a SIMD finish each step first and idle at the barrier (+3-4 %).
      if constexpr (TSA_SETPRIO) __builtin_amdgcn_s_setprio(0);
      if constexpr (TSA_SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);  // keep the arithmetic between the two
      if constexpr (F16)
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
      } else if constexpr (FIN) {
        if (w == w_f) {
#pragma unroll
          for (int i = 0; i < M; ++i) fin[i * 64 + lane] = oBest[i];
        }
      }

      // ---- send this step's record to the wave below (or the ring)
      if constexpr (ROLE != 2) {
        uint8_t *dst = xr + (w * HNSL + (HSK == 2 ? q : PH)) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i)
          lds_write16(dst + i * PAIR_BYTES, make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
      } else {
        // Positions that have not started (u = t - w - k < 0) must publish the
        // y = 0 face: wave 0 reads this row as "row y0-1" during its lap 0.
        if (t < ZT + HSK * NW) {
          const int32_t lim = t - HSK * w;  // position k started iff k <= lim
#pragma unroll
          for (int i = 0; i < M; ++i) {
            const uint32_t m = ((M * lane + i > lim) ? 0x0000FFFFu : 0u) |
                               (((TWO ? 0 : 64 * M) + M * lane + i > lim) ? 0xFFFF0000u : 0u);
            oIy[i] = bfi(m, pa.f_single, oIy[i]);
            oIxy[i] = bfi(m, pa.f_pair, oIxy[i]);
            oIyz[i] = bfi(m, pa.f_pair, oIyz[i]);
            oBest[i] = bfi(m, 0u, oBest[i]);
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
      zshift<M>(shIxz[PH], oIxz, sel, pa.f_pair);  // z = 0 face for position 0
      zshift<M>(shIz, oIz, sel, pa.f_single);
      zshift<M>(svIyz, rz, sel, pa.f_pair);
      zshift<M>(svM[PH], rw, sel, 0u);
      // position 0 advances to u0 + 1
#if TSA_HM_TRACK
      if (__builtin_expect(++xpos0 == next_ev, 0)) {
        if (xpos0 == P) {
          xpos0 = 0;
          binj = b_of_lap(++lap0);
          row_terms();
        }
        hmCur = hm_of(xpos0);
        next_ev = ev_of(xpos0);
      }
#else
      if (++xpos0 == P) {
        xpos0 = 0;
        binj = b_of_lap(++lap0);
        row_terms();
      }
#endif
      if constexpr (TSA_A_PREFETCH) load_a<M>(a_lane + 4u * (uint32_t)xpos0, a_nx);

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
#ifdef TSA_EXP_NOBAR  // timing experiment only: wrong results
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
      // skew 2: a wave reads records two steps old, so one barrier per pair of steps
      if constexpr (HSK == 1 || PH == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
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
      if constexpr (TWO) {
        scores[tri] = decode((uint16_t)(fin[k_f] & 0xFFFF));
        if (has1) scores[tri + 1] = decode((uint16_t)(fin[64 + k_f1] >> 16));
      } else {
        int32_t l_f, i_f, h_f;
        pos_split<M>(k_f, l_f, i_f, h_f);
        const uint32_t v = fin[i_f * 64 + l_f];
        scores[tri] = decode((uint16_t)(h_f ? (v >> 16) : (v & 0xFFFF)));
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Single-cube variant: the cube is cut into NW-row laps (y) and ZT-position
// tiles (z, ZT = 128*M); every (lap, tile) gets its own workgroup and all of
// them run at once (blockIdx.x = (tri * G + L) * GZ + q). Each workgroup runs
// the helix step in its own local time t (position k of wave w at x = t-w-k+1).
//   y hand-off: lap L's last wave stores its per-step record rows; lap L+1's
//     wave 0 LDS-DMAs them LPD steps ahead (rows of step r feed step r-(NW-1)).
//   z hand-off: every wave's last position (lane 63, pair M-1, hi half) leaves
//     its {Iz, Ixz, Iyz, best} words in an LDS staging record, with wave 0
//     adding the row above's {Iyz, best}; the last wave stores that record per
//     step, and tile q+1's wave 0 LDS-DMAs record t+ZT for its position 0
//     (tile q+1 runs ZT steps behind tile q, the z skew of the wavefront).
//   producer: write-through (sc1) stores; each step a counted vmcnt proves
//     rows <= t-LAP_SLACK (and z records two steps older) complete, then one
//     agent-scope flag store publishes t-LAP_SLACK+1 (MI355X_MICROARCH.md
//     "Valid forms", row 1);
//   consumer: the flag words travel with the data (LDS-DMA, LPD steps ahead);
//     only when they do not yet cover what it needs does wave 0 drain its
//     queue and poll (bounded: on timeout *err is set and scores are invalid).
// Producers have lower block indices than their consumers; the host keeps the
// grid resident or relies on in-order dispatch (lap_choice), so a spinning
// consumer never blocks its producer.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_sc1(void *gptr, uint4 v) {
  const u32x4 d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(gptr), "v"(d) : "memory");
}
constexpr int ZRING = 16;  // z records resident in LDS (power of 2, >= lap_pd + 3)

template <int M, int NW, bool F16, bool SOP>
__global__ __launch_bounds__(64 * NW) void pencil_lap_kernel(
    const uint8_t *__restrict__ seqs, const int64_t *__restrict__ offs, int32_t G, int32_t GZ,
    int32_t YR, int32_t lds_a, uint8_t *__restrict__ yf_base, uint8_t *__restrict__ zf_base,
    int32_t *__restrict__ flags, int32_t *__restrict__ err, int32_t *__restrict__ scores,
    PencilArgs pa, unsigned long long *__restrict__ trace) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int PAIR_BYTES = 64 * REC_BYTES;
  constexpr int SLOT_BYTES = M * PAIR_BYTES;
  constexpr int ZT = 128 * M;
  constexpr int LPD = lap_pd(M);
  // diagnostic trace (TSA_LAP_TRACE): per workgroup {start, loop begin, loop end, XCC id}
  auto stamp = [&](int slot) {
    if (trace != nullptr && threadIdx.x == 0) {
      unsigned long long v;
      if (slot == 3) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        v = x;
      }
      else asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
      trace[(int64_t)blockIdx.x * 8 + slot] = v;
    }
  };
  stamp(0);
  stamp(3);
  constexpr int ZREC = ((NW + 1) * 16 + 63) & ~63;  // z record: rows -1..NW-1 x 16 B
  static_assert(ZRING >= LPD + 3, "z ring");
  uint8_t *xr = smem;                                    // [NW-1][2][M][64][16]
  uint8_t *xr0 = xr + (NW - 1) * 2 * SLOT_BYTES;         // [LPD][M][64][16]
  uint8_t *zst = xr0 + LPD * SLOT_BYTES;                 // [4][ZREC] z staging (producer)
  uint8_t *zring = zst + 4 * ZREC;                       // [ZRING][ZREC] z records (consumer)
  // producer flags, LDS-DMA'd every step and read every step without a wait: the
  // word holds whichever DMA landed last (flags only grow), a lower bound that
  // lags by the DMA latency rather than by the prefetch distance
  int32_t *fslot = (int32_t *)(zring + ZRING * ZREC);    // [1] y-producer flag
  int32_t *zfslot = fslot + LPD;                         // [1] z-producer flag
  uint32_t *fin = (uint32_t *)(zfslot + LPD);            // [M][64] final-step best
  uint32_t *sA2 = fin + M * 64;                          // [la + ZT + NW + ZT] A code pairs

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t sel = lane == 0 ? 0x05040302u : 0x07060504u;
  uint32_t Q = F16 ? 0x08000800u : 0x00010001u, fsv = pa.f_single, fpv = pa.f_pair;
  asm volatile("" : "+v"(Q), "+v"(fsv), "+v"(fpv));
  const PencilArgs pv = F16 ? pa : pin_score_consts(pa);

  const int32_t wg = blockIdx.x, q = wg % GZ, tri = wg / (G * GZ), L = (wg / GZ) % G;
  const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
  const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
  const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
  const int32_t nlap = (lb + NW - 1) / NW, ntile = (lc + ZT - 1) / ZT;
  if (L >= nlap || q >= ntile) return;  // whole workgroup
  const bool zin = q > 0, zout = q + 1 < ntile;
  const int32_t zt_q = min(ZT, lc - q * ZT);  // positions of this tile
  const bool final_wg = L == nlap - 1 && q == ntile - 1;
  const int32_t w_f = (lb - 1) % NW, k_f = lc - 1 - q * ZT;
  // steps of this workgroup; the final one stops at the final cell (la, lb, lc)
  const int32_t T_full = la + (NW - 1) + (zt_q - 1);
  const int32_t T = final_wg ? (la - 1) + w_f + k_f + 1 : T_full;
  const int32_t T_zprev = la + (NW - 1) + (ZT - 1);  // steps of tile q-1 (full width)
  uint8_t *yf_mine = yf_base + (int64_t)wg * YR * SLOT_BYTES;
  const uint8_t *yf_prev = yf_mine - (int64_t)GZ * YR * SLOT_BYTES;  // (L-1, q)
  uint8_t *zf_mine = zf_base + (int64_t)wg * YR * ZREC;
  const uint8_t *zf_prev = zf_mine - (int64_t)YR * ZREC;             // (L, q-1)
  int32_t *flag_mine = flags + wg;
  const int32_t *flag_prev = flag_mine - GZ, *flag_zprev = flag_mine - 1;

  // A code pairs: entry j holds x = j-ZT (lo) and x = j-ZT-64M (hi), 0 outside [0, la)
  const int32_t na = lds_a / 4;
  for (int j = threadIdx.x; j < na; j += 64 * NW) {
    const int x0 = j - ZT, x1 = j - ZT - 64 * M;
    const uint32_t c0 = (x0 >= 0 && x0 < la) ? SYM0 << (seqs[o0 + x0] & 3) : 0u;
    const uint32_t c1 = (x1 >= 0 && x1 < la) ? SYM0 << (seqs[o0 + x1] & 3) : 0u;
    sA2[j] = c0 | (c1 << 16);
  }
  // position k of this wave is at x-1 = t - w - k: a[i] = sA2[t - w + ZT - M lane - i]
  const uint32_t a_lane = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)sA2 +
                          4u * (uint32_t)(ZT - w - M * lane - (M - 1));

  const int32_t y = L * NW + w + 1;  // this wave's DP row
  const uint32_t bw = y <= lb ? (SYM0 << (seqs[o1 + y - 1] & 3)) * 0x00010001u : 0u;
  uint32_t b[M], c[M], SBC[M], K[M], DMC[M];
  uint32_t oIx[M], shIz[M], svIxy[M], svIyz[M], shIxz[2][M], svM[2][M];
  {
    uint32_t one1 = 0x00010001u, sbcv = pa.h_sbc, kdv = pa.h_kd, k0v = pa.h_k0;
    asm volatile("" : "+v"(one1), "+v"(sbcv), "+v"(kdv), "+v"(k0v));
    const int64_t oc = o2 + (int64_t)q * ZT;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int k0 = M * lane + i, k1 = 64 * M + M * lane + i;
      const uint32_t c0 = k0 < zt_q ? SYM0 << (seqs[oc + k0] & 3) : 0u;
      const uint32_t c1 = k1 < zt_q ? SYM0 << (seqs[oc + k1] & 3) : 0u;
      c[i] = c0 | (c1 << 16);
      DMC[i] = dm_over_code(pa.dmf, c[i]);
      b[i] = bw;  // one row per wave
      const uint32_t e01 = pk_eq1(bw, c[i], one1);
      SBC[i] = pk_mad(e01, sbcv, 0u);
      K[i] = pk_mad(e01, kdv, k0v);
      oIx[i] = shIz[i] = pa.f_single;
      shIxz[0][i] = shIxz[1][i] = svIxy[i] = svIyz[i] = pa.f_pair;
      svM[0][i] = svM[1][i] = 0;
    }
  }

  // ---- consumer side (wave 0): progress of the y and z producers
  int32_t seen = 0, seen_z = 0;  // producer flags seen (rows < seen, z records < seen_z - 2)
  uint32_t n_poll = 0, n_spin = 0;  // diagnostics (trace only)
  // Wait until need < producer flag, reading the flag through its LDS word and
  // refreshing that word by LDS-DMA: no vmcnt drain, so the row and record DMAs
  // already in flight keep going (a drained poll cost ~2-4 us each)
  auto poll = [&](const int32_t *fl, int32_t *word, int32_t &sn, int32_t need) {
    ++n_poll;
    for (uint32_t spin = 0;; ++spin, ++n_spin) {
      sn = max(sn, __builtin_amdgcn_readfirstlane(
                       *(volatile const __attribute__((address_space(3))) int32_t *)(
                           const __attribute__((address_space(3))) void *)word));
      if (need < sn) break;
      if (spin > (1u << 22)) {
        if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sn = 1 << 30;
        break;
      }
      if ((spin & 15) == 0 && lane == 0) dma4(fl, word);
      __builtin_amdgcn_s_sleep(2);
    }
  };
  const int32_t T_prev = T_full;  // rows lap L-1 publishes (same tile width)
  auto fetch_y = [&](int32_t s2) {  // rows of step s2 -> xr0 slot s2 % LPD (+ flag word)
    const int32_t r = s2 + NW - 1;
    if (r < T_prev && r >= seen) poll(flag_prev, fslot, seen, r);
    const int32_t rr = r < T_prev ? r : T_prev - 1;  // past the end: any valid row
#pragma unroll
    for (int i = 0; i < M; ++i)
      dma16(yf_prev + ((int64_t)rr * M + i) * PAIR_BYTES + lane * REC_BYTES,
            xr0 + (s2 % LPD) * SLOT_BYTES + i * PAIR_BYTES);
    if (lane == 0) dma4(flag_prev, fslot);
  };
  auto fetch_z = [&](int32_t i) {  // z record i -> zring (+ the flag word)
    if (i < T_zprev && i >= seen_z - 2) poll(flag_zprev, zfslot, seen_z, i + 2);
    const int32_t ii = i < T_zprev ? i : T_zprev - 1;
    if (lane < ZREC / 16)
      dma16(zf_prev + (int64_t)ii * ZREC + lane * 16, zring + (i & (ZRING - 1)) * ZREC);
    if (lane == 0) dma4(flag_zprev, zfslot);
  };
  if (w == 0) {
    // flag slots not DMA'd by the prologue must read as "nothing published"
    if (lane < 2 * LPD) fslot[lane] = 0;  // fslot and zfslot
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // before any DMA lands there
    if (L > 0)
      for (int s2 = 0; s2 < LPD; ++s2) fetch_y(s2);
    if (zin) {  // records ZT-1 .. ZT+LPD serve the first LPD+1 steps
      for (int i = ZT - 1; i <= ZT + LPD; ++i) fetch_z(i);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      seen_z = max(seen_z, __builtin_amdgcn_readfirstlane(zfslot[0]));
    }
  }
  __syncthreads();
  stamp(1);
  const uint4 face = make_uint4(pa.f_single, pa.f_pair, pa.f_pair, 0u);
  uint32_t a_nx[M];  // A codes of the coming step
  if constexpr (TSA_A_PREFETCH) load_a<M>(a_lane, a_nx);

  // ROLE (wave 0): bit 0 = rows of lap L-1 arrive (L > 0), bit 2 = z records of
  // tile q-1 arrive (q > 0); 2 = middle waves; 3 = the last wave
  auto step = [&](auto ph, auto role, int32_t t, auto fin_step) {
    constexpr int PH = decltype(ph)::value;
    constexpr int ROLE = decltype(role)::value;
    constexpr bool FIN = decltype(fin_step)::value;  // the last step (t == T-1)
    constexpr bool W0 = ROLE == 0 || ROLE == 1 || ROLE == 4 || ROLE == 5;
    constexpr bool YIN = ROLE == 1 || ROLE == 5, ZIN0 = ROLE == 4 || ROLE == 5;
    uint32_t a[M];
    if constexpr (TSA_A_PREFETCH) {
#pragma unroll
      for (int i = 0; i < M; ++i) a[i] = a_nx[i];
      load_a<M>(a_lane + 4u * (uint32_t)(t + 1), a_nx);  // lands by the step barrier
    } else {
      load_a<M>(a_lane + 4u * (uint32_t)t, a);
    }
    uint4 rec[M];
    if constexpr (W0) {
      // rows (+ flag) and the z record (+ flag) of step t were DMA'd LPD steps ago
      constexpr int OPS = (YIN ? M + 1 : 0) + (ZIN0 ? 2 : 0);
      if constexpr (OPS > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS * (LPD - 1)) : "memory");
      if constexpr (YIN) {
        const uint8_t *src = xr0 + (t % LPD) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
        // producer progress as of the last landed flag DMA (no wait, no round trip)
        seen = max(seen, __builtin_amdgcn_readfirstlane(
                             *(volatile const __attribute__((address_space(3))) int32_t *)(
                                 const __attribute__((address_space(3))) void *)fslot));
      } else {
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = face;  // y = 0 face
      }
      if constexpr (ZIN0)
        seen_z = max(seen_z, __builtin_amdgcn_readfirstlane(
                                 *(volatile const __attribute__((address_space(3))) int32_t *)(
                                     const __attribute__((address_space(3))) void *)zfslot));
    } else {
      const uint8_t *src = xr + ((w - 1) * 2 + (PH ^ 1)) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
      for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
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
    // x == 1 at position k* = t - w: x = 0 face inputs (src/PE_1cyc.v:164-178,196-218)
    const int32_t ks = t - w;
    if (ks >= 0 && ks < ZT) {
      int32_t ls, is, hs;
      pos_split<M>(ks, ls, is, hs);
      const uint32_t hm = hs ? 0xFFFF0000u : 0x0000FFFFu;
      const uint32_t m1 = lane == ls ? hm : 0u;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (i == is) {
          inIx[i] = vbfi(m1, fsv, inIx[i]);
          inIxy[i] = vbfi(m1, fpv, inIxy[i]);
          inIxz[i] = vbfi(m1, fpv, inIxz[i]);
          inM[i] = vbfi(m1, 0u, inM[i]);
        }
      }
    }
    uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);  // keep the arithmetic between the two
    if constexpr (F16)
      cell_messages_f16<M, SOP>(a, b, c, SBC, K, DMC, Q, pa, inIx, inIy, inIz, inIxy, inIyz, inIxz,
                                inM, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
    else
      cell_messages<M, SOP ? 1 : 0>(a, b, c, Q, pv, inIx, inIy, inIz, inIxy, inIyz, inIxz, inM,
                                    nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
    __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
    if constexpr (FIN) {
      if (final_wg && w == w_f) {
#pragma unroll
        for (int i = 0; i < M; ++i) fin[i * 64 + lane] = oBest[i];
      }
    }
    // z staging: this wave's last position, and (wave 0) the row above's
    if (zout && lane == 63) {
      lds_write16(zst + (t & 3) * ZREC + (w + 1) * 16,
                  make_uint4(oIz[M - 1], oIxz[M - 1], oIyz[M - 1], oBest[M - 1]));
      if constexpr (W0) {  // rec of step t = the row above at step t-1
        if (t >= 1)
          lds_write16(zst + ((t - 1) & 3) * ZREC, make_uint4(0u, 0u, rec[M - 1].z, rec[M - 1].w));
      }
    }
    if constexpr (ROLE != 3) {
      uint8_t *dst = xr + (w * 2 + PH) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
      for (int i = 0; i < M; ++i)
        lds_write16(dst + i * PAIR_BYTES, make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
    } else {
#pragma unroll
      for (int i = 0; i < M; ++i)
        store16_sc1(yf_mine + ((int64_t)t * M + i) * PAIR_BYTES + lane * REC_BYTES,
                    make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
      if (zout && t >= 2 && lane <= NW) {  // z record of step t-2 is complete in LDS
        const uint4 v = lds_read16(zst + ((t - 2) & 3) * ZREC + lane * 16);
        store16_sc1(zf_mine + (int64_t)(t - 2) * ZREC + lane * 16, v);
      }
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      oIx[i] = nIx[i];
      svIxy[i] = rec[i].y;
    }
    uint32_t rz[M], rw[M];
#pragma unroll
    for (int i = 0; i < M; ++i) { rz[i] = rec[i].z; rw[i] = rec[i].w; }
    // position 0's z-1 neighbour: the z = 0 face, or tile q-1's last position
    uint32_t fIxz = pa.f_pair, fIz = pa.f_single, fIyz = pa.f_pair, fM = 0u;
    if (zin) {
      const uint8_t *ra = zring + ((t + ZT) & (ZRING - 1)) * ZREC + (w + 1) * 16;
      const uint8_t *rb = zring + ((t + ZT - 1) & (ZRING - 1)) * ZREC + w * 16 + 8;
      typedef unsigned u32x2_lds __attribute__((ext_vector_type(2)));
      const u32x2_lds za = *(const __attribute__((address_space(3))) u32x2_lds *)(
          const __attribute__((address_space(3))) void *)ra;
      const u32x2_lds zb = *(const __attribute__((address_space(3))) u32x2_lds *)(
          const __attribute__((address_space(3))) void *)rb;
      fIz = za.x;
      fIxz = za.y;
      fIyz = zb.x;
      fM = zb.y;
    }
    zshift<M>(shIxz[PH], oIxz, sel, fIxz);
    zshift<M>(shIz, oIz, sel, fIz);
    zshift<M>(svIyz, rz, sel, fIyz);
    zshift<M>(svM[PH], rw, sel, fM);
    if constexpr (W0) {
      if constexpr (YIN) fetch_y(t + LPD);  // usually covered by the prefetched flag
      if constexpr (ZIN0) fetch_z(t + ZT + LPD + 1);
    }
    if constexpr (ROLE == 3) {
      // rows <= t - LAP_SLACK (z records two steps older) complete: per step M row
      // stores, 1 flag store and at most one z store -- the count assumes none,
      // so with a z store it waits for slightly more than it needs
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LAP_SLACK * (M + 1)) : "memory");
      if (lane == 0)
        __hip_atomic_store(flag_mine, t >= LAP_SLACK ? t - LAP_SLACK + 1 : 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto run = [&](auto role) {  // last step peeled, as in the helix kernel
    int32_t t = 0;
    const int32_t T1 = T - 1;
    constexpr std::integral_constant<int, 0> P0{};
    constexpr std::integral_constant<int, 1> P1{};
    constexpr std::false_type mid{};
    constexpr std::true_type last{};
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
  if (w == 0) {
    if (L == 0) {
      if (zin) TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 4>{}));
      else TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 0>{}));
    } else {
      if (zin) TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 5>{}));
      else TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 1>{}));
    }
  } else if (w == NW - 1) {
    TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 3>{}));
  } else {
    TSA_INLINE_IF_WIDE(run(std::integral_constant<int, 2>{}));
  }
  stamp(2);
  if (trace != nullptr && threadIdx.x == 0) {
    trace[(int64_t)blockIdx.x * 8 + 4] = n_poll;
    trace[(int64_t)blockIdx.x * 8 + 5] = n_spin;
  }
  // the last two z records: every wave's staging writes are done after this barrier
  __syncthreads();
  if (w == NW - 1) {
    if (zout && lane <= NW)
      for (int32_t s2 = max(T - 2, 0); s2 < T; ++s2)
        store16_sc1(zf_mine + (int64_t)s2 * ZREC + lane * 16,
                    lds_read16(zst + (s2 & 3) * ZREC + lane * 16));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(flag_mine, T + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (final_wg) {
    if (threadIdx.x == 0) {
      int32_t l_f, i_f, h_f;
      pos_split<M>(k_f, l_f, i_f, h_f);
      const uint32_t v = fin[i_f * 64 + l_f];
      const uint16_t hb = (uint16_t)(h_f ? (v >> 16) : (v & 0xFFFF));
      scores[tri] = F16 ? (int32_t)(float)__builtin_bit_cast(_Float16, hb) : (int32_t)(int16_t)hb;
    }
  }
}


static uint32_t pk16(int32_t v) { return ((uint32_t)(uint16_t)(int16_t)v) * 0x00010001u; }
static uint32_t pkh(double v) {  // both halves = f16(v); v exactly representable
  const _Float16 h = (_Float16)v;
  uint16_t bits;
  memcpy(&bits, &h, 2);
  return (uint32_t)bits * 0x00010001u;
}

static PencilArgs make_args(const KParams &kp, bool f16) {
  const int32_t GE = kp.pen[SIXY][SIX], GO = kp.pen[SIXY][SM];  // Ixy row: Ix = GE, M = GO
  int32_t fs = -kp.pen[SIX][0], fp = -kp.pen[SIXY][0];
  for (int s = 0; s < 7; ++s) {
    fs = std::max(fs, -kp.pen[SIX][s]);
    fp = std::max(fp, -kp.pen[SIXY][s]);
  }
  PencilArgs a;
  memset(&a, 0, sizeof(a));
  a.sop = kp.s3_mode == TSA_S3_SOP;
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
  return a;
}

// Exact-f16 arithmetic applies when every value and candidate is an integer in
// [-2048, 2048] (value bound + PENCIL_MARGIN) and the scaled deltas fit f16.
static bool use_f16(const KParams &kp, const Range &r) {
  if (const char *e = getenv("TSA_PENCIL_ARITH"))  // tuning / test knob
    if (!strcmp(e, "i16")) return false;
  auto small = [](int64_t v) { return v >= -7 && v <= 7; };
  auto fits = [](int64_t v) { return v >= -2048 && v <= 2048; };
  return r.lo - PENCIL_MARGIN >= -2048 && r.hi + PENCIL_MARGIN <= 2048 &&
         small((int64_t)kp.match - kp.mismatch) && small((int64_t)kp.s3_ab - kp.s3_ne) &&
         small((int64_t)kp.s3_eq - kp.s3_ab) && small((int64_t)kp.s3_eq - kp.s3_ne) &&
         fits(kp.mismatch) && fits(kp.s3_ne) &&
         fits(3LL * kp.mismatch);
}

template <int M, int NW, bool F16, bool SOP>
static int launch_m(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                    int32_t max_lb, const PencilGeom &g, int32_t *d_scores, void *d_ws,
                    const PencilArgs &pa, hipStream_t stream) {
  const int32_t lds_a = 4 * (g.P + 128 * M), lds_b = 4 * ((max_lb + 3) & ~3);
  const size_t lds = helix_lds(M, NW, g.P, max_lb);
  // TWO (two triples per workgroup) exactly when pencil_geom sized P for it
  const bool two = M == 1 && g.two;
  auto kfn = two ? pencil_kernel<M, NW, F16, SOP, M == 1> : pencil_kernel<M, NW, F16, SOP, false>;
  if (lds > LDS_MAX) return TSA_EINVAL;
  if (hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return TSA_EDEVICE;
  const int32_t units = two ? (n + 1) / 2 : n;
  const int grid = units < 65535 ? units : 65535;
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(64 * NW), lds, stream, d_seqs, d_offsets, n, g.P,
                     g.R, lds_a, lds_b, g.ring_bytes_per_triple, (uint8_t *)d_ws, d_scores,
                     pa);
  return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
}

template <int M, int NW, bool F16, bool SOP>
static int launch_lap(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_la,
                      const LapGeom &g, int32_t *d_scores, void *d_ws, const PencilArgs &pa,
                      hipStream_t stream) {
  const int32_t lds_a = 4 * ((max_la + NW + 2 * 128 * M + 3) & ~3);
  auto kfn = pencil_lap_kernel<M, NW, F16, SOP>;
  if (g.lds > LDS_MAX) return TSA_EINVAL;
  if (hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)g.lds) != hipSuccess)
    return TSA_EDEVICE;
  const int64_t wgs = (int64_t)n * g.G * g.GZ;
  int32_t *flags = (int32_t *)d_ws;  // [wgs] progress + [1] error word
  if (hipMemsetAsync(flags, 0, g.flag_bytes, stream) != hipSuccess) return TSA_EDEVICE;
  uint8_t *yf = (uint8_t *)d_ws + g.flag_bytes;
  uint8_t *zf = yf + g.yf_bytes;
  unsigned long long *trace = nullptr;
  const char *tpath = getenv("TSA_LAP_TRACE");  // diagnostic: per-WG timestamps to a CSV file
  if (tpath && hipMalloc(&trace, (size_t)wgs * 8 * 8) != hipSuccess) return TSA_ENOMEM;
  if (trace && hipMemsetAsync(trace, 0, (size_t)wgs * 8 * 8, stream) != hipSuccess) return TSA_EDEVICE;
  hipLaunchKernelGGL(kfn, dim3((uint32_t)wgs), dim3(64 * NW), g.lds, stream, d_seqs, d_offsets,
                     g.G, g.GZ, g.YR, lds_a, yf, zf, flags, flags + wgs, d_scores, pa, trace);
  if (trace) {
    std::vector<unsigned long long> h((size_t)wgs * 8);
    if (hipMemcpyAsync(h.data(), trace, h.size() * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return TSA_EDEVICE;
    (void)hipFree(trace);
    if (FILE *fp = fopen(tpath, "w")) {
      fprintf(fp, "wg,tri,lap,tile,start,loop_begin,loop_end,xcc,polls,spins\n");
      for (int64_t i = 0; i < wgs; ++i)
        fprintf(fp, "%lld,%lld,%lld,%lld,%llu,%llu,%llu,%llu,%llu,%llu\n", (long long)i,
                (long long)(i / ((int64_t)g.G * g.GZ)), (long long)((i / g.GZ) % g.G),
                (long long)(i % g.GZ), h[i * 8], h[i * 8 + 1], h[i * 8 + 2], h[i * 8 + 3],
                h[i * 8 + 4], h[i * 8 + 5]);
      fclose(fp);
    }
  }
  return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
}

// Instantiated shapes: M = 1, 2 with 8 or 16 rows per workgroup; M = 4, 8
// (LC up to 512 / 1024) with 8; each in f16 / int16 arithmetic and RTL / SOP s3.
#define TSA_SHAPES(LAUNCH, M_, NW_, F16_, SOP_, ...)                                      \
  ((M_) == 1 ? ((NW_) == 16 ? TSA_ARITH(LAUNCH, 1, 16, F16_, SOP_, __VA_ARGS__)            \
                            : TSA_ARITH(LAUNCH, 1, 8, F16_, SOP_, __VA_ARGS__))            \
   : (M_) == 2 ? ((NW_) == 16 ? TSA_ARITH(LAUNCH, 2, 16, F16_, SOP_, __VA_ARGS__)          \
                              : TSA_ARITH(LAUNCH, 2, 8, F16_, SOP_, __VA_ARGS__))          \
   : (M_) == 4 ? TSA_ARITH(LAUNCH, 4, 8, F16_, SOP_, __VA_ARGS__)                          \
               : TSA_ARITH(LAUNCH, 8, 8, F16_, SOP_, __VA_ARGS__))
#define TSA_ARITH(LAUNCH, MM, NN, F16_, SOP_, ...)                                        \
  ((F16_) ? ((SOP_) ? LAUNCH<MM, NN, true, true>(__VA_ARGS__)                              \
                    : LAUNCH<MM, NN, true, false>(__VA_ARGS__))                            \
          : ((SOP_) ? LAUNCH<MM, NN, false, true>(__VA_ARGS__)                             \
                    : LAUNCH<MM, NN, false, false>(__VA_ARGS__)))

void pencil_describe(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                     const Range &bound, bool stream_ok, char *buf, size_t len) {
  const char *arith = use_f16(kp, bound) ? "f16" : "i16";
  const char *s3 = kp.s3_mode == TSA_S3_SOP ? "sop" : "rtl";
  const LapGeom lg = lap_choice(n, max_la, max_lb, max_lc, stream_ok);
  if (lg.ok) {
    snprintf(buf, len, "pencil lap %s %s M=%d NW=%d laps=%d tiles=%d waves=%lld", arith, s3, lg.M,
             lg.NW, lg.G, lg.GZ, (long long)lg.waves);
    return;
  }
  const PencilGeom g = pencil_geom(max_la, max_lc);
  snprintf(buf, len, "pencil helix %s %s M=%d NW=%d P=%d%s", arith, s3, g.M, helix_nw(g.M), g.P,
           g.two ? " two" : "");
}

int pencil_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                        int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                        const Range &bound, int32_t *d_scores, void *d_ws, size_t ws_bytes,
                        hipStream_t stream, bool stream_ok, int32_t **d_err) {
  if (d_err) *d_err = nullptr;
  if (n <= 0) return TSA_OK;
  if (!pencil_shape_ok(max_la, max_lb, max_lc)) return TSA_EINVAL;
  const bool f16 = use_f16(kp, bound);
  const PencilArgs pa = make_args(kp, f16);
  const bool sop = pa.sop != 0;
  const LapGeom lg = lap_choice(n, max_la, max_lb, max_lc, stream_ok);
  if (lg.ok) {
    if (ws_bytes < lg.flag_bytes + lg.yf_bytes + lg.zf_bytes) return TSA_ENOMEM;
    if (d_err) *d_err = (int32_t *)d_ws + (size_t)n * lg.G * lg.GZ;
    return TSA_SHAPES(launch_lap, lg.M, lg.NW, f16, sop, d_seqs, d_offsets, n, max_la, lg,
                      d_scores, d_ws, pa, stream);
  }
  const PencilGeom g = pencil_geom(max_la, max_lc);
  const int32_t grid = n < 65535 ? n : 65535;
  if (ws_bytes < (size_t)grid * (size_t)g.ring_bytes_per_triple) return TSA_ENOMEM;
  return TSA_SHAPES(launch_m, g.M, helix_nw(g.M), f16, sop, d_seqs, d_offsets, n, max_lb, g,
                    d_scores, d_ws, pa, stream);
}
#undef TSA_SHAPES
#undef TSA_ARITH

}  // namespace tsa
