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
//    positions k (lane l, pair i, half h -> k = l + 64h + 128i), z = k+1;
//  * position k of wave w computes cell x = u mod P + 1 of lap u div P at step
//    t, with u = t - w - k (one step of skew per y and per z). A lane that
//    finishes x = P of lap L continues with x = 1 of lap L+1 (row y+NW), so
//    there is no fill/drain between rows: the positions form a helix;
//  * z-1 neighbours arrive by one DPP wave_ror:1 + v_perm per packed value,
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

#include "pencil_kernel.h"

namespace tsa {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// waves (= DP rows) per lap: 16 (one 1024-thread WG per CU) or 8 (two WGs
// per CU, so one computes while the other waits at its per-step barrier)
constexpr int PENCIL_NW_DEFAULT = 16;
constexpr int PD = 8;              // LDS-DMA prefetch distance of wave 0, steps
constexpr int LPD = 4;             // prefetch distance of the lap kernel (cross-CU hand-off)
constexpr int STORE_SLACK = 4;     // last wave keeps <= this many steps of stores in flight
constexpr int PMIN = 48;           // >= PD + NW + STORE_SLACK + margin
constexpr int MAX_LA = 4096, MAX_LB = 4096;
constexpr int REC_BYTES = 16;      // {Iy, Ixy, Iyz, best} packed pairs per lane
constexpr int RING_EXTRA = 8;

struct PencilArgs {
  uint32_t E, O, E2, OE, O2;    // packed penalties GE, GO, 2GE, GO+GE, 2GO
  uint32_t f_single, f_pair;    // face messages of an all-zero cell
  uint32_t dm, mm;              // match-mismatch, mismatch
  uint32_t s3_d1, s3_d0, s3_ne; // RTL: s3 = ne + eab*(d0 + ebc*d1)
  int32_t sop;                  // TSA_S3_SOP
};

struct PencilGeom {
  int32_t M;        // pairs per lane
  int32_t P;        // lap period (steps)
  int32_t R;        // ring rows
  int64_t ring_bytes_per_triple;
};

static inline int32_t pencil_pairs(int32_t max_lc) { return max_lc <= 128 ? 1 : 2; }

static PencilGeom pencil_geom(int32_t max_la, int32_t max_lc) {
  PencilGeom g;
  g.M = pencil_pairs(max_lc);
  const int32_t zt = 128 * g.M;
  g.P = std::max(std::max(max_la, zt), PMIN);
  g.R = g.P + RING_EXTRA;
  g.ring_bytes_per_triple = (int64_t)g.R * g.M * 64 * REC_BYTES;
  return g;
}

bool pencil_supported(const tsa_params *p) { return p != nullptr; }

static bool pencil_shape_ok(int32_t max_la, int32_t max_lb, int32_t max_lc) {
  return max_la >= 1 && max_la <= MAX_LA && max_lb >= 1 && max_lb <= MAX_LB && max_lc >= 1 &&
         max_lc <= 256;
}

// Lap-parallel mode (pencil_lap_kernel) for small batches of tall cubes: every
// lap of every triple gets its own resident workgroup.
// Rows per lap (waves per workgroup) of the lap kernel: fewer rows = shorter
// steps but more laps, each adding a hand-off lag. Tuning knob TSA_LAP_NW.
constexpr int LAP_NW_DEFAULT = 16;
static int lap_nw() {
  if (const char *e = getenv("TSA_LAP_NW")) {
    const int v = atoi(e);
    if (v == 4 || v == 8 || v == 16) return v;
  }
  return LAP_NW_DEFAULT;
}
// workgroups guaranteed co-resident: one per CU for 16 waves, two for 8, four for 4
static int max_resident_wg(int nw) { return 256 * (16 / nw); }
struct LapGeom {
  int32_t NW, G, YR;
  size_t yf_bytes, flag_bytes;
};
static LapGeom lap_geom(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  LapGeom g;
  const int32_t M = pencil_pairs(max_lc);
  g.NW = lap_nw();
  g.G = (max_lb + g.NW - 1) / g.NW;
  g.YR = max_la + max_lc + 2 * g.NW + PD + 8;
  g.yf_bytes = (size_t)n * g.G * g.YR * M * 64 * REC_BYTES;
  g.flag_bytes = (((size_t)n * g.G + 1) * sizeof(int32_t) + 255) & ~(size_t)255;
  return g;
}
static bool use_lap_mode(int32_t n, int32_t max_lb) {
  if (const char *e = getenv("TSA_PENCIL_MODE")) {
    if (!strcmp(e, "helix")) return false;
  }
  const int nw = lap_nw();
  const int32_t G = (max_lb + nw - 1) / nw;
  return G >= 2 && (int64_t)n * G <= max_resident_wg(nw);
}

size_t pencil_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  if (!pencil_shape_ok(max_la, max_lb, max_lc)) return 0;
  if (use_lap_mode(n, max_lb)) {
    const LapGeom g = lap_geom(n, max_la, max_lb, max_lc);
    return g.flag_bytes + g.yf_bytes;
  }
  return (size_t)n * (size_t)pencil_geom(max_la, max_lc).ring_bytes_per_triple;
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

// Shift a packed per-position value one position up the helix (k <- k-1):
// lanes >= 1 take lane-1's pair as is; lane 0 takes (pair i-1).hi and
// (pair i).lo of lane 63; position 0 (lane 0, pair 0, lo) gets `inj`.
template <int M>
__device__ __forceinline__ void shift_pos(uint32_t (&v)[M], uint32_t sel, uint32_t mask0,
                                          uint32_t inj) {
  uint32_t r[M];
#pragma unroll
  for (int i = 0; i < M; ++i) r[i] = ror1(v[i]);
#pragma unroll
  for (int i = 0; i < M; ++i) v[i] = __builtin_amdgcn_perm(r[i], r[(i + M - 1) % M], sel);
  v[0] = bfi(mask0, inj, v[0]);
}

// The x == 1 position k* (if inside this lane span) takes the x = 0 face for
// its x-1 inputs (EN_i==1&&EN==0 gating, src/PE_1cyc.v:164-178,196-202,212-218).
template <int M>
__device__ __forceinline__ void x1_substitute(int ks, int lane, const PencilArgs &pa,
                                              uint32_t (&inIx)[M], uint32_t (&inIxy)[M],
                                              uint32_t (&inIxz)[M], uint32_t (&inM)[M]) {
  if (ks >= 0 && ks < 128 * M) {
    const uint32_t hm = (ks >> 6) & 1 ? 0xFFFF0000u : 0x0000FFFFu;
    const uint32_t m1 = lane == (ks & 63) ? hm : 0u;
    const int is = ks >> 7;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i == is) {
        inIx[i] = bfi(m1, pa.f_single, inIx[i]);
        inIxy[i] = bfi(m1, pa.f_pair, inIxy[i]);
        inIxz[i] = bfi(m1, pa.f_pair, inIxz[i]);
        inM[i] = bfi(m1, 0u, inM[i]);
      }
    }
  }
}

// One step of M packed cell pairs: scores (src/PE_1cyc.v:159-162) on one-hot
// symbols, the 7 states, and the 7 outgoing messages max_s(S[s] - P[T][s])
// (src/PE_1cyc.v:164-218) grouped by equal penalty; oBest = MAX7 of the states.
template <int M>
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
    if (pa.sop) s3 = pk_add(pk_add(s2ab, s2bc), s2ac);
    else s3 = pk_mad(eab, pk_mad(ebc, pa.s3_d1, pa.s3_d0), pa.s3_ne);
    const uint32_t sM = pk_add(inM[i], s3);
    const uint32_t sX = inIx[i], sY = inIy[i], sZ = inIz[i];
    const uint32_t sXY = pk_add(inIxy[i], s2ab);
    const uint32_t sYZ = pk_add(inIyz[i], s2bc);
    const uint32_t sXZ = pk_add(inIxz[i], s2ac);
    const uint32_t pYZ = pk_max(sY, sZ), pXZ = pk_max(sX, sZ), pXY = pk_max(sX, sY);
    const uint32_t qXY_XZ = pk_max(sXY, sXZ), qXY_YZ = pk_max(sXY, sYZ), qYZ_XZ = pk_max(sYZ, sXZ);
    const uint32_t A1 = pk_max(pYZ, qXY_XZ);  // Ix  <- {Iy,Iz,Ixy,Ixz} at GO+GE
    const uint32_t A2 = pk_max(pXZ, qXY_YZ);  // Iy  <- {Ix,Iz,Ixy,Iyz}
    const uint32_t A3 = pk_max(pXY, qYZ_XZ);  // Iz  <- {Ix,Iy,Iyz,Ixz}
    const uint32_t B1 = pk_max(sM, sYZ);      // Ix  <- {M,Iyz} at 2GO
    const uint32_t B2 = pk_max(sM, sXZ);      // Iy  <- {M,Ixz}
    const uint32_t B3 = pk_max(sM, sXY);      // Iz  <- {M,Ixy}
    const uint32_t C1 = pk_max(pXY, sXY);     // Ixy <- {Ix,Iy,Ixy} at GE
    const uint32_t C2 = pk_max(pYZ, sYZ);     // Iyz <- {Iy,Iz,Iyz}
    const uint32_t C3 = pk_max(pXZ, sXZ);     // Ixz <- {Ix,Iz,Ixz}
    const uint32_t D1 = pk_max(B1, pk_max(sZ, sXZ));  // Ixy <- {M,Iz,Iyz,Ixz} at GO
    const uint32_t D2 = pk_max(B2, pk_max(sX, sXY));  // Iyz <- {M,Ix,Ixy,Ixz}
    const uint32_t D3 = pk_max(B3, pk_max(sY, sYZ));  // Ixz <- {M,Iy,Ixy,Iyz}
    oBest[i] = pk_max(pk_max(A1, B1), sX);            // MAX7 of the states
    nIx[i] = pk_max(pk_max(pk_sub(sX, pa.E2), pk_sub(A1, pa.OE)), pk_sub(B1, pa.O2));
    oIy[i] = pk_max(pk_max(pk_sub(sY, pa.E2), pk_sub(A2, pa.OE)), pk_sub(B2, pa.O2));
    oIz[i] = pk_max(pk_max(pk_sub(sZ, pa.E2), pk_sub(A3, pa.OE)), pk_sub(B3, pa.O2));
    oIxy[i] = pk_max(pk_sub(C1, pa.E), pk_sub(D1, pa.O));
    oIyz[i] = pk_max(pk_sub(C2, pa.E), pk_sub(D2, pa.O));
    oIxz[i] = pk_max(pk_sub(C3, pa.E), pk_sub(D3, pa.O));
  }
}

// Diagnostic stamps (separate build, never timed): per-wave sums of s_memtime
// deltas over the step phases [receive, compute+send, shifts, barrier].
#define TSA_STAMP(var)                                                             \
  do {                                                                             \
    if constexpr (STAMPS) {                                                        \
      __builtin_amdgcn_sched_barrier(0);                                           \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                           \
    }                                                                              \
  } while (0)

template <int M, int NW, bool STAMPS = false>
__global__ __launch_bounds__(64 * NW) void pencil_kernel(const uint8_t *__restrict__ seqs,
                                                         const int64_t *__restrict__ offs,
                                                         int32_t n, int32_t P, int32_t R,
                                                         int32_t lds_a, int32_t stagger,
                                                         int64_t ring_stride,
                                                         uint8_t *__restrict__ ring_base,
                                                         int32_t *__restrict__ scores,
                                                         PencilArgs pa,
                                                         unsigned long long *__restrict__ dbg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0, st4 = 0;
  unsigned long long acc[4] = {0, 0, 0, 0};
  constexpr int PAIR_BYTES = 64 * REC_BYTES;              // one pair's record, 1 KiB
  constexpr int SLOT_BYTES = M * PAIR_BYTES;
  uint8_t *xr = smem;                                     // [NW-1][2][M][64][16]
  uint8_t *xr0 = xr + (NW - 1) * 2 * SLOT_BYTES;          // [PD][M][64][16]
  uint8_t *sA = xr0 + PD * SLOT_BYTES;                    // [lds_a >= P] one-hot A
  uint8_t *sB = sA + lds_a;                               // [>= max LB] one-hot B

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t sel = lane == 0 ? 0x05040302u : 0x07060504u;
  const uint32_t mask0 = lane == 0 ? 0x0000FFFFu : 0u;
  uint32_t ones = 0x00010001u;
  asm volatile("" : "+v"(ones));  // keep it in a VGPR (VOP3P operand)
  constexpr int ZT = 128 * M;

  for (int tri = blockIdx.x; tri < n; tri += gridDim.x) {
    const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
    const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
    const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
    uint8_t *ring = ring_base + (int64_t)blockIdx.x * ring_stride;

    // ---- stage one-hot A (padded to P) and B; fill the ring with face records
    for (int i = threadIdx.x; i < P; i += 64 * NW)
      sA[i] = i < la ? (uint8_t)(1u << (seqs[o0 + i] & 3)) : 0;
    for (int i = threadIdx.x; i < lb; i += 64 * NW) sB[i] = (uint8_t)(1u << (seqs[o1 + i] & 3));
    {
      const uint4 face = make_uint4(pa.f_single, pa.f_pair, pa.f_pair, 0u);
      const int64_t n16 = (int64_t)R * M * 64;
      for (int64_t i = threadIdx.x; i < n16; i += 64 * NW) ((uint4 *)ring)[i] = face;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- per-position registers
    uint32_t a[M], b[M], c[M];
    uint32_t oIx[M], shIz[M], shIxz1[M], shIxz2[M], svIxy[M], svIyz[M], svM1[M], svM2[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int k0 = lane + 128 * i, k1 = lane + 64 + 128 * i;
      const uint32_t c0 = k0 < lc ? 1u << (seqs[o2 + k0] & 3) : 0u;
      const uint32_t c1 = k1 < lc ? 1u << (seqs[o2 + k1] & 3) : 0u;
      c[i] = c0 | (c1 << 16);
      // symbols at step 0: position k is at u = -w-k (x index (u mod P))
      const int x0 = ((-w - k0) % P + P) % P, x1 = ((-w - k1) % P + P) % P;
      a[i] = (uint32_t)sA[x0] | ((uint32_t)sA[x1] << 16);
      // only position 0 of wave 0 has started (u = 0, row 1); others are u < 0
      b[i] = (i == 0 && w == 0 && lane == 0) ? (uint32_t)sB[0] : 0u;
      oIx[i] = pa.f_single;
      shIz[i] = pa.f_single;
      shIxz1[i] = shIxz2[i] = pa.f_pair;
      svIxy[i] = svIyz[i] = pa.f_pair;
      svM1[i] = svM2[i] = 0;
    }
    // position-0 bookkeeping (wave-uniform): u0 = t - w
    int32_t xpos0 = (P - (w % P)) % P;      // (t - w) mod P at t = 0
    int32_t lap0 = w == 0 ? 0 : -1;         // floor((t - w) / P)
    // final cell (la, lb, lc)
    const int32_t lap_f = (lb - 1) / NW, w_f = (lb - 1) % NW, k_f = lc - 1;
    const int32_t t_f = lap_f * P + (la - 1) + w_f + k_f;
    const int32_t l_f = k_f & 63, i_f = k_f >> 7, h_f = (k_f >> 6) & 1;
    const int32_t T = t_f + 1;

    // wave 0: prime the LDS-DMA pipeline (ring row of step s = s - P + NW - 1)
    const int32_t lag = P - (NW - 1);
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
    int32_t st_row = 0;                          // ring row written at step t (last wave)

    // optional phase offset between co-resident workgroups (tuning knob)
    if (stagger > 0 && (blockIdx.x & 1))
      for (int z = 0; z < stagger; ++z) __builtin_amdgcn_s_sleep(1);

    TSA_STAMP(st0);
#pragma unroll 1
    for (int32_t t = 0; t < T; ++t) {
      // position 0's next symbols, read at the top of the step: sA/sB are
      // read-only in the loop, so their LDS latency hides under the compute
      int32_t nx0 = xpos0 + 1, nlap0 = lap0;
      if (nx0 == P) { nx0 = 0; ++nlap0; }
      const uint32_t ainj = sA[nx0];
      const int32_t row0 = nlap0 * NW + w;
      const uint32_t binj = (nlap0 >= 0 && row0 < lb) ? (uint32_t)sB[row0] : 0u;
      // ---- receive the wave-above record of step t-1
      uint4 rec[M];
      if (w == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(M * (PD - 1)) : "memory");
        const uint8_t *src = xr0 + (t % PD) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
      } else {
        const uint8_t *src = xr + ((w - 1) * 2 + ((t - 1) & 1)) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
      }

      // ---- inputs (messages into this cell)
      uint32_t inIx[M], inIy[M], inIz[M], inIxy[M], inIyz[M], inIxz[M], inM[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        inIx[i] = oIx[i];
        inIy[i] = rec[i].x;
        inIz[i] = shIz[i];
        inIxy[i] = svIxy[i];
        inIyz[i] = svIyz[i];
        inIxz[i] = shIxz2[i];
        inM[i] = svM2[i];
      }
      // x == 1 at position k* = (t - w) mod P: its x-1 inputs are the x = 0 face
      // (EN_i==1&&EN==0 gating, src/PE_1cyc.v:164-178,196-202,212-218)
      if constexpr (STAMPS) asm volatile("" ::"v"(rec[0].x), "v"(rec[M - 1].w));
      TSA_STAMP(st1);
      x1_substitute<M>(xpos0, lane, pa, inIx, inIxy, inIxz, inM);
      uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
      cell_messages<M>(a, b, c, ones, pa, inIx, inIy, inIz, inIxy, inIyz, inIxz, inM, nIx, oIy, oIz,
                       oIxy, oIyz, oIxz, oBest);

      // ---- send this step's record to the wave below (or the ring)
      if (w < NW - 1) {
        uint8_t *dst = xr + (w * 2 + (t & 1)) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i)
          lds_write16(dst + i * PAIR_BYTES, make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
      } else {
        // Positions that have not started (u = t - w - k < 0) must publish the
        // y = 0 face: wave 0 reads this row as "row y0-1" during its lap 0.
        if (t < ZT + NW) {
          const int32_t lim = t - w;  // position k started iff k <= lim
#pragma unroll
          for (int i = 0; i < M; ++i) {
            const uint32_t m = ((lane + 128 * i > lim) ? 0x0000FFFFu : 0u) |
                               ((lane + 64 + 128 * i > lim) ? 0xFFFF0000u : 0u);
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

      // ---- final cell (src/TriAlign_1cyc.v:141-142,342-345)
      if (t == t_f && w == w_f) {
        uint32_t v = oBest[0];
#pragma unroll
        for (int i = 1; i < M; ++i) if (i == i_f) v = oBest[i];
        if (lane == l_f) scores[tri] = (int32_t)(int16_t)(h_f ? (v >> 16) : (v & 0xFFFF));
      }

      // ---- advance the systolic registers
#pragma unroll
      for (int i = 0; i < M; ++i) {
        oIx[i] = nIx[i];
        shIxz2[i] = shIxz1[i];
        shIxz1[i] = oIxz[i];
        shIz[i] = oIz[i];
        svIxy[i] = rec[i].y;
        svIyz[i] = rec[i].z;
        svM2[i] = svM1[i];
        svM1[i] = rec[i].w;
      }
      TSA_STAMP(st2);
      shift_pos<M>(shIxz1, sel, mask0, pa.f_pair);   // z = 0 face for position 0
      shift_pos<M>(shIz, sel, mask0, pa.f_single);
      shift_pos<M>(svIyz, sel, mask0, pa.f_pair);
      shift_pos<M>(svM1, sel, mask0, 0u);
      // position 0 advances to u0 + 1
      xpos0 = nx0;
      lap0 = nlap0;
      shift_pos<M>(a, sel, mask0, ainj);
      shift_pos<M>(b, sel, mask0, binj);

      // ---- wave 0: fetch the record of step t + PD into the slot just consumed
      if (w == 0) {
#pragma unroll
        for (int i = 0; i < M; ++i)
          dma16(ring + ((int64_t)dma_row * M + i) * PAIR_BYTES + lane * REC_BYTES,
                xr0 + (t % PD) * SLOT_BYTES + i * PAIR_BYTES);
        if (++dma_row == R) dma_row = 0;
      }
      if (w == NW - 1) {
        if (++st_row == R) st_row = 0;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(M * STORE_SLACK) : "memory");
      }
      TSA_STAMP(st3);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      TSA_STAMP(st4);
      if constexpr (STAMPS) {
        acc[0] += st1 - st0; acc[1] += st2 - st1; acc[2] += st3 - st2; acc[3] += st4 - st3;
        st0 = st4;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if constexpr (STAMPS) {
    if (blockIdx.x == 0 && lane == 0)
      for (int q = 0; q < 4; ++q) dbg[w * 4 + q] = acc[q];
  }
}

// ---------------------------------------------------------------------------
// Single-cube variant: one 16-row lap per workgroup, all laps of a triple in
// flight at once (blockIdx.x = tri * G + L). Lap L's last wave hands its
// per-step record rows down to lap L+1's wave 0 through global memory:
//   producer: write-through (sc1) row stores; each step a counted vmcnt proves
//             rows <= tau-STORE_SLACK complete, then one agent-scope flag store
//             publishes that count (MI355X_MICROARCH.md "Valid forms", row 1);
//   consumer: before LDS-DMA'ing (sc1) a row it has not yet seen published, it
//             drains its own queue and polls the flag with agent-scope loads.
// Every workgroup of the grid must be resident (host: n*G <= resident WGs), so
// a spinning consumer never blocks its producer. Spins are bounded: on
// timeout the kernel sets *err and carries on (scores then invalid).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_sc1(void *gptr, uint4 v) {
  const u32x4 d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(gptr), "v"(d) : "memory");
}

template <int M, int NW>
__global__ __launch_bounds__(64 * NW) void pencil_lap_kernel(
    const uint8_t *__restrict__ seqs, const int64_t *__restrict__ offs, int32_t G, int32_t YR,
    uint8_t *__restrict__ yf_base, int32_t *__restrict__ flags, int32_t *__restrict__ err,
    int32_t *__restrict__ scores, PencilArgs pa) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int PAIR_BYTES = 64 * REC_BYTES;
  constexpr int SLOT_BYTES = M * PAIR_BYTES;
  uint8_t *xr = smem;                             // [NW-1][2][M][64][16]
  uint8_t *xr0 = xr + (NW - 1) * 2 * SLOT_BYTES;  // [LPD][M][64][16]
  int32_t *fslot = (int32_t *)(xr0 + LPD * SLOT_BYTES);  // [LPD] prefetched producer flags
  uint8_t *sA = (uint8_t *)(fslot + LPD);          // one-hot A

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t sel = lane == 0 ? 0x05040302u : 0x07060504u;
  const uint32_t mask0 = lane == 0 ? 0x0000FFFFu : 0u;
  uint32_t ones = 0x00010001u;
  asm volatile("" : "+v"(ones));

  const int32_t tri = blockIdx.x / G, L = blockIdx.x % G;
  const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
  const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
  const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
  const int32_t nlap = (lb + NW - 1) / NW;
  if (L >= nlap) return;  // whole workgroup
  const int32_t T = la + (NW - 1) + (lc - 1);      // steps of this lap
  uint8_t *yf_mine = yf_base + ((int64_t)tri * G + L) * YR * SLOT_BYTES;
  const uint8_t *yf_prev = yf_mine - (int64_t)YR * SLOT_BYTES;
  int32_t *flag_mine = flags + (int64_t)tri * G + L;
  const int32_t *flag_prev = flag_mine - 1;

  for (int i = threadIdx.x; i < la; i += 64 * NW) sA[i] = (uint8_t)(1u << (seqs[o0 + i] & 3));
  __syncthreads();

  const int32_t y = L * NW + w + 1;                 // this wave's DP row
  const uint32_t bw = y <= lb ? (1u << (seqs[o1 + y - 1] & 3)) * 0x00010001u : 0u;
  uint32_t a[M], b[M], c[M];
  uint32_t oIx[M], shIz[M], shIxz1[M], shIxz2[M], svIxy[M], svIyz[M], svM1[M], svM2[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int k0 = lane + 128 * i, k1 = lane + 64 + 128 * i;
    const uint32_t c0 = k0 < lc ? 1u << (seqs[o2 + k0] & 3) : 0u;
    const uint32_t c1 = k1 < lc ? 1u << (seqs[o2 + k1] & 3) : 0u;
    c[i] = c0 | (c1 << 16);
    b[i] = bw;  // one row per wave: B is constant
    a[i] = (i == 0 && w == 0 && lane == 0) ? (uint32_t)sA[0] : 0u;  // only (x=1,k=0) started
    oIx[i] = pa.f_single;
    shIz[i] = pa.f_single;
    shIxz1[i] = shIxz2[i] = pa.f_pair;
    svIxy[i] = svIyz[i] = pa.f_pair;
    svM1[i] = svM2[i] = 0;
  }
  const int32_t w_f = (lb - 1) % NW, k_f = lc - 1;
  const bool final_lap = L == (lb - 1) / NW;
  const int32_t t_f = (la - 1) + w_f + k_f;
  const int32_t l_f = k_f & 63, i_f = k_f >> 7, h_f = (k_f >> 6) & 1;

  // wave 0 of lap L>0: row r of yf_prev feeds step r - (NW-1); prime LPD steps
  int32_t seen = 0;  // rows of yf_prev known complete
  auto ensure = [&](int32_t r) {  // r < T: row r must be published
    if (r < seen || r >= T) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t spin = 0;; ++spin) {
      seen = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(flag_prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (r < seen) break;
      if (spin > (1u << 22)) {
        if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        seen = T;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  if (w == 0 && L > 0) {
    for (int s2 = 0; s2 < LPD; ++s2) {
      const int32_t r = s2 + NW - 1;
      ensure(r);
#pragma unroll
      for (int i = 0; i < M; ++i)
        dma16(yf_prev + ((int64_t)r * M + i) * PAIR_BYTES + lane * REC_BYTES,
              xr0 + (s2 % LPD) * SLOT_BYTES + i * PAIR_BYTES);
      if (lane == 0) dma4(flag_prev, fslot + (s2 % LPD));
    }
  }
  const uint4 face = make_uint4(pa.f_single, pa.f_pair, pa.f_pair, 0u);

#pragma unroll 1
  for (int32_t t = 0; t < T; ++t) {
    uint4 rec[M];
    if (w == 0) {
      if (L == 0) {
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = face;  // y = 0 face
      } else {
        // rows + flag of step t were DMA'd LPD steps ago: M+1 ops per step
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((M + 1) * (LPD - 1)) : "memory");
        const uint8_t *src = xr0 + (t % LPD) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rec[i] = lds_read16(src + i * PAIR_BYTES);
        // producer progress as of ~LPD steps ago, free of any round trip
        seen = max(seen, __builtin_amdgcn_readfirstlane(fslot[t % LPD]));
      }
    } else {
      const uint8_t *src = xr + ((w - 1) * 2 + ((t - 1) & 1)) * SLOT_BYTES + lane * REC_BYTES;
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
      inIxz[i] = shIxz2[i];
      inM[i] = svM2[i];
    }
    x1_substitute<M>(t - w, lane, pa, inIx, inIxy, inIxz, inM);
    uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
    cell_messages<M>(a, b, c, ones, pa, inIx, inIy, inIz, inIxy, inIyz, inIxz, inM, nIx, oIy, oIz,
                     oIxy, oIyz, oIxz, oBest);

    if (w < NW - 1) {
      uint8_t *dst = xr + (w * 2 + (t & 1)) * SLOT_BYTES + lane * REC_BYTES;
#pragma unroll
      for (int i = 0; i < M; ++i)
        lds_write16(dst + i * PAIR_BYTES, make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
    } else {
#pragma unroll
      for (int i = 0; i < M; ++i)
        store16_sc1(yf_mine + ((int64_t)t * M + i) * PAIR_BYTES + lane * REC_BYTES,
                    make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
    }
    if (final_lap && t == t_f && w == w_f) {
      uint32_t v = oBest[0];
#pragma unroll
      for (int i = 1; i < M; ++i) if (i == i_f) v = oBest[i];
      if (lane == l_f) scores[tri] = (int32_t)(int16_t)(h_f ? (v >> 16) : (v & 0xFFFF));
    }
#pragma unroll
    for (int i = 0; i < M; ++i) {
      oIx[i] = nIx[i];
      shIxz2[i] = shIxz1[i];
      shIxz1[i] = oIxz[i];
      shIz[i] = oIz[i];
      svIxy[i] = rec[i].y;
      svIyz[i] = rec[i].z;
      svM2[i] = svM1[i];
      svM1[i] = rec[i].w;
    }
    shift_pos<M>(shIxz1, sel, mask0, pa.f_pair);
    shift_pos<M>(shIz, sel, mask0, pa.f_single);
    shift_pos<M>(svIyz, sel, mask0, pa.f_pair);
    shift_pos<M>(svM1, sel, mask0, 0u);
    {
      const int32_t xi = t + 1 - w;  // position 0's x-1 at step t+1
      const uint32_t ainj = (xi >= 0 && xi < la) ? (uint32_t)sA[xi] : 0u;
      shift_pos<M>(a, sel, mask0, ainj);
    }
    if (w == 0 && L > 0) {
      const int32_t r = t + LPD + NW - 1;  // row for step t + LPD
      ensure(r);  // usually satisfied by the prefetched flag: no round trip
#pragma unroll
      for (int i = 0; i < M; ++i)
        dma16(yf_prev + ((int64_t)r * M + i) * PAIR_BYTES + lane * REC_BYTES,
              xr0 + (t % LPD) * SLOT_BYTES + i * PAIR_BYTES);
      if (lane == 0) dma4(flag_prev, fslot + (t % LPD));
    }
    if (w == NW - 1) {
      // rows <= t - STORE_SLACK complete (M stores + 1 flag store per step)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STORE_SLACK * (M + 1)) : "memory");
      // exactly M + 1 vector-memory ops per step keep that count exact
      if (lane == 0)
        __hip_atomic_store(flag_mine, t >= STORE_SLACK ? t - STORE_SLACK + 1 : 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (w == NW - 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(flag_mine, T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


static PencilArgs make_args(const KParams &kp) {
  auto pk = [](int32_t v) { return ((uint32_t)(uint16_t)(int16_t)v) * 0x00010001u; };
  const int32_t GE = kp.pen[SIXY][SIX], GO = kp.pen[SIXY][SM];  // Ixy row: Ix = GE, M = GO
  PencilArgs a;
  a.E = pk(GE);
  a.O = pk(GO);
  a.E2 = pk(2 * GE);
  a.OE = pk(GO + GE);
  a.O2 = pk(2 * GO);
  int32_t fs = -kp.pen[SIX][0], fp = -kp.pen[SIXY][0];
  for (int s = 0; s < 7; ++s) {
    fs = std::max(fs, -kp.pen[SIX][s]);
    fp = std::max(fp, -kp.pen[SIXY][s]);
  }
  a.f_single = pk(fs);
  a.f_pair = pk(fp);
  a.dm = pk(kp.match - kp.mismatch);
  a.mm = pk(kp.mismatch);
  a.s3_d1 = pk(kp.s3_eq - kp.s3_ab);
  a.s3_d0 = pk(kp.s3_ab - kp.s3_ne);
  a.s3_ne = pk(kp.s3_ne);
  a.sop = kp.s3_mode == TSA_S3_SOP;
  return a;
}

template <int M, int NW>
static int launch_m(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                    int32_t max_lb, const PencilGeom &g, int32_t *d_scores, void *d_ws,
                    const PencilArgs &pa, hipStream_t stream) {
  const int32_t lds_a = (g.P + 15) & ~15, lds_b = (max_lb + 15) & ~15;
  const size_t lds = (size_t)(NW - 1) * 2 * M * 1024 + (size_t)PD * M * 1024 + lds_a + lds_b;
  auto kfn = pencil_kernel<M, NW>;
  if (hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return TSA_EDEVICE;
  const int grid = n < 65535 ? n : 65535;
  int stagger = 0;
  if (const char *e = getenv("TSA_PENCIL_STAGGER")) stagger = atoi(e);  // tuning knob
  if (getenv("TSA_PENCIL_STAMPS")) {  // diagnostic build: phase shares, printed to stderr
    auto kst = pencil_kernel<M, NW, true>;
    if (hipFuncSetAttribute((const void *)kst, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return TSA_EDEVICE;
    unsigned long long *dbg = nullptr, h[NW * 4];
    if (hipMalloc(&dbg, sizeof(h)) != hipSuccess) return TSA_ENOMEM;
    hipLaunchKernelGGL(kst, dim3(grid), dim3(64 * NW), lds, stream, d_seqs, d_offsets, n, g.P,
                       g.R, lds_a, stagger, g.ring_bytes_per_triple, (uint8_t *)d_ws, d_scores,
                       pa, dbg);
    if (hipMemcpyAsync(h, dbg, sizeof(h), hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return TSA_EDEVICE;
    (void)hipFree(dbg);
    for (int w = 0; w < NW; ++w)
      fprintf(stderr, "STAMPS wave %2d recv %llu compute+send %llu shifts+dma %llu barrier %llu\n",
              w, h[w * 4], h[w * 4 + 1], h[w * 4 + 2], h[w * 4 + 3]);
    return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(64 * NW), lds, stream, d_seqs, d_offsets, n, g.P,
                     g.R, lds_a, stagger, g.ring_bytes_per_triple, (uint8_t *)d_ws, d_scores, pa,
                     nullptr);
  return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
}

template <int M, int NW>
static int launch_lap(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_la,
                      const LapGeom &g, int32_t *d_scores, void *d_ws, const PencilArgs &pa,
                      hipStream_t stream) {
  const size_t lds = (size_t)(NW - 1) * 2 * M * 1024 + (size_t)LPD * M * 1024 + LPD * 4 +
                     ((max_la + 15) & ~15);
  auto kfn = pencil_lap_kernel<M, NW>;
  if (hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return TSA_EDEVICE;
  int32_t *flags = (int32_t *)d_ws;           // [n*G] progress + [1] error word
  if (hipMemsetAsync(flags, 0, g.flag_bytes, stream) != hipSuccess) return TSA_EDEVICE;
  uint8_t *yf = (uint8_t *)d_ws + g.flag_bytes;
  hipLaunchKernelGGL(kfn, dim3(n * g.G), dim3(64 * NW), lds, stream, d_seqs, d_offsets, g.G, g.YR,
                     yf, flags, flags + (size_t)n * g.G, d_scores, pa);
  return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
}

int pencil_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                        int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                        int32_t *d_scores, void *d_ws, size_t ws_bytes, hipStream_t stream) {
  if (n <= 0) return TSA_OK;
  if (!pencil_shape_ok(max_la, max_lb, max_lc)) return TSA_EINVAL;
  if (use_lap_mode(n, max_lb)) {
    const LapGeom lg = lap_geom(n, max_la, max_lb, max_lc);
    if (ws_bytes < lg.flag_bytes + lg.yf_bytes) return TSA_ENOMEM;
    const PencilArgs pa = make_args(kp);
#define TSA_LAP(MM, NN) launch_lap<MM, NN>(d_seqs, d_offsets, n, max_la, lg, d_scores, d_ws, pa, stream)
    if (pencil_pairs(max_lc) == 1)
      return lg.NW == 4 ? TSA_LAP(1, 4) : lg.NW == 8 ? TSA_LAP(1, 8) : TSA_LAP(1, 16);
    return lg.NW == 4 ? TSA_LAP(2, 4) : lg.NW == 8 ? TSA_LAP(2, 8) : TSA_LAP(2, 16);
#undef TSA_LAP
  }
  const PencilGeom g = pencil_geom(max_la, max_lc);
  const int32_t grid = n < 65535 ? n : 65535;
  if (ws_bytes < (size_t)grid * (size_t)g.ring_bytes_per_triple) return TSA_ENOMEM;
  const PencilArgs pa = make_args(kp);
  int nw = PENCIL_NW_DEFAULT;
  if (const char *e = getenv("TSA_PENCIL_NW")) nw = atoi(e) == 8 ? 8 : 16;  // tuning knob
  if (g.M == 1)
    return nw == 8 ? launch_m<1, 8>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_ws, pa, stream)
                   : launch_m<1, 16>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_ws, pa, stream);
  return nw == 8 ? launch_m<2, 8>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_ws, pa, stream)
                 : launch_m<2, 16>(d_seqs, d_offsets, n, max_lb, g, d_scores, d_ws, pa, stream);
}

}  // namespace tsa
