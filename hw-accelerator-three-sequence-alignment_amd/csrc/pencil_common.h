// pencil_common.h -- device helpers, packed constants and build knobs shared
// by the register-systolic kernels: the batch helix (pencil_kernel.hip) and the
// single-cube lap kernel (lap_kernel.hip). See pencil_kernel.hip for the design.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "pencil_kernel.h"

namespace tsa {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

constexpr size_t LDS_MAX = 160 * 1024;
constexpr int REC_BYTES = 16;      // {Iy, Ixy, Iyz, best} packed pairs per lane
#ifndef TSA_A_B64  // V-space M = 2: a step's A codes as one ds_read_b64 (pencil_kernel)
#define TSA_A_B64 1
#endif
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
#ifndef TSA_SETPRIO  // helix: priority 0 for the cell arithmetic, 1 for the tail
#define TSA_SETPRIO 1
#endif
#ifndef TSA_IS_STATIC  // M = 2: the x = 1 register index from the wave parity
#define TSA_IS_STATIC 1
#endif
#ifndef TSA_SCHED_FENCE  // sched_barrier fences around the helix cell arithmetic
#define TSA_SCHED_FENCE 1
#endif

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
  int32_t packed;               // 2-bit packed input symbols (tsa_sym)
  // V-space helix (cell_messages_vs): values of cell (x,y,z) shifted by
  // lam*(x+y+z); lam = GE = -MISMATCH, f16 bits in both halves
  int32_t lam;                  // lam as an integer (0: not V-space)
  uint32_t v_lam, v_cP, v_dO;   // lam, GO + MISMATCH + lam, GO - GE
  float d0f, d1f;               // RTL s3 deltas (V-space K = (d0 + [b=c] d1) / code(b))
};


// Literal RTL arithmetic (literal_kernel.hip, the lap kernel's LIT form):
// constants as int16 values shifted left by sh = 16 - SCORE_BITS, both halves,
// so packed u16 adds wrap exactly at the RTL word.
struct LitArgs {
  uint32_t n2E, nOE, n2O;   // -2GE, -(GO+GE), -2GO
  uint32_t dmS, mmE, nDOE;  // match - mismatch, mismatch - GE, -(GO - GE)
  uint32_t d1S, d0S, neS;   // RTL s3 = ne + [a=b](d0 + [b=c] d1)
  uint32_t mm3S;            // SOP s3 = 3 mismatch + dm ([a=b] + [b=c] + [a=c])
  // pushes of a zero cell (the faces): to Ix / Iy / Iz, to a pair target with
  // its pair score a match (1) or not (0), to M by the successor's indicators
  uint32_t fS[3], fP[2], fM[8];
  int32_t sh, packed;
};
LitArgs lit_args(const KParams &kp);

// positions per lane: M packed pairs cover LC <= 128*M (1, 2, 4 or 8)
static inline int32_t pencil_pairs(int32_t max_lc) {
  return max_lc <= 128 ? 1 : max_lc <= 256 ? 2 : max_lc <= 512 ? 4 : 8;
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
// The same through an LDS base pointer plus a byte offset: a compile-time
// offset folds into the ds instruction's offset field (no VALU address add)
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ lds_u8 *to_lds(uint8_t *p) {
  return (lds_u8 *)(__attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ uint4 lds_read16_at(const lds_u8 *base, int off) {
  const u32x4_lds v = *(const __attribute__((address_space(3))) u32x4_lds *)(base + off);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lds_write16_at(lds_u8 *base, int off, uint4 v) {
  *(__attribute__((address_space(3))) u32x4_lds *)(base + off) = (u32x4_lds){v.x, v.y, v.z, v.w};
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

// The same cell in V-space (tests/test_cell_algebra.py replays it against the
// oracle): every value of cell (x,y,z) is stored shifted by lam*(x+y+z), a
// potential -- every path into a cell gains the same amount, so no max
// changes -- with lam = GE = -MISMATCH (the RTL's constants: 1). A transition
// that advances x+y+z by d then pays lam*d less, so (f16 form, the mismatch
// folded into the pair messages as above):
//  * the pair targets' extend penalty GE - MISMATCH - 2 lam vanishes:
//      Ixy' = max(G_z, best - (GO - GE)),  G_z = max(Ix, Iy, Ixy)  (G_x, G_y alike);
//  * a single target is the better of its own extension and the two pair
//    messages that share its gaps (the penalty table is a sum over the gapped
//    axes, src/PE_1cyc.v:172-194, so max(Ixy', Ixz') covers every other source):
//      Ix' = max(Ix - lam, max(Ixy', Ixz') - (GO + MISMATCH + lam));
//  * M adds no constant: 3 MISMATCH + 3 lam = 0 (the SOP form folds 3 lam into K).
// 24 instructions per pair (RTL) against cell_messages_f16's 33. Zero faces
// become lam*q at coordinate sum q: the kernel injects those (pencil_kernel.hip).
template <int M, bool SOP>
__device__ __forceinline__ void cell_messages_vs(
    const uint32_t (&a)[M], const uint32_t (&b)[M], const uint32_t (&c)[M],
    const uint32_t (&SBC)[M], const uint32_t (&K)[M], const uint32_t (&DMC)[M], const uint32_t (&DMB)[M],
    const PencilArgs &pa,
    const uint32_t (&inIx)[M], const uint32_t (&inIy)[M], const uint32_t (&inIz)[M],
    const uint32_t (&inIxy)[M], const uint32_t (&inIyz)[M], const uint32_t (&inIxz)[M],
    const uint32_t (&inM)[M], uint32_t (&nIx)[M], uint32_t (&oIy)[M], uint32_t (&oIz)[M],
    uint32_t (&oIxy)[M], uint32_t (&oIyz)[M], uint32_t (&oIxz)[M], uint32_t (&oBest)[M]) {
  const h2 LAM = H(pa.v_lam), CP = H(pa.v_cP), DO = H(pa.v_dO);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    // a & b is b's code on a match, 0 otherwise; DMB = dm / code(b) and (RTL) K
    // = (d0 + [b=c] d1) / code(b) per position and row: the products are exact
    const h2 eab = H(a[i] & b[i]), eac = H(a[i] & c[i]), DMCi = H(DMC[i]), DMBi = H(DMB[i]);
    const h2 sXY = hfma(eab, DMBi, H(inIxy[i]));  // src/PE_1cyc.v:159-161 (+mismatch folded)
    const h2 sXZ = hfma(eac, DMCi, H(inIxz[i]));
    const h2 sYZ = H(inIyz[i]) + H(SBC[i]);
    h2 sM;                                       // src/PE_1cyc.v:162
    if constexpr (SOP) sM = hfma(eab, DMBi, hfma(eac, DMCi, H(inM[i]))) + H(K[i]);
    else sM = hfma(eab, H(K[i]), H(inM[i]));     // ne + 3 lam = 0
    const h2 sX = H(inIx[i]), sY = H(inIy[i]), sZ = H(inIz[i]);
    const h2 Gx = vmax3(sY, sZ, sYZ), Gy = vmax3(sX, sZ, sXZ), Gz = vmax3(sX, sY, sXY);
    const h2 best = vmax3(Gx, Gy, hmax(sXY, sM));
    const h2 b1 = best - DO;
    const h2 pXY = hmax(Gz, b1), pYZ = hmax(Gx, b1), pXZ = hmax(Gy, b1);
    const h2 qXY = pXY - CP, qYZ = pYZ - CP, qXZ = pXZ - CP;
    oBest[i] = U(best);
    oIxy[i] = U(pXY);
    oIyz[i] = U(pYZ);
    oIxz[i] = U(pXZ);
    nIx[i] = U(vmax3(sX - LAM, qXY, qXZ));
    oIy[i] = U(vmax3(sY - LAM, qXY, qYZ));
    oIz[i] = U(vmax3(sZ - LAM, qYZ, qXZ));
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
// The same at a constant entry offset `off` from va, as an inbounds index of
// an LDS pointer, so the offset folds into the ds_read's offset field (a u32
// add could wrap, and the compiler then adds it in a VALU op)
template <int M>
__device__ __forceinline__ void load_a_off(uint32_t va, int off, uint32_t (&a)[M]) {
  const __attribute__((address_space(3))) uint32_t *p =
      (const __attribute__((address_space(3))) uint32_t *)(uintptr_t)va;
#pragma unroll
  for (int i = 0; i < M; ++i) a[i] = p[off + M - 1 - i];
}
// V-space, M = 2: entries OFF and OFF + 1 of va's table as one ds_read_b64
// (a[1] = entry OFF, a[0] = OFF + 1). The group's first entry va is odd, so
// the pair is 8-byte aligned in the table itself for odd OFF, and in the copy
// shifted by one entry (va_s: entry j holds the table's j + 1) for even OFF.
// Lanes 8 B apart then read 512 contiguous bytes, conflict-free in both
// 32-lane groups; ds_read2_b32 is serviced as two ds_read_b32 banked mod 32,
// which lanes two dwords apart make 2-way (MI355X_MICROARCH.md, LDS).
template <int OFF>
__device__ __forceinline__ void load_a_pair(uint32_t va, uint32_t va_s, uint32_t (&a)[2]) {
  const uint32_t addr = (OFF & 1) ? va + 4u * OFF : va_s + 4u * (OFF - 1);
  // one 64-bit integer load (a uint2 is split into two dword loads, which the
  // backend re-merges into ds_read2_b32 unless it can prove the alignment)
  const uint64_t v = *(const __attribute__((address_space(3))) uint64_t *)(uintptr_t)addr;
  a[1] = (uint32_t)v;
  a[0] = (uint32_t)(v >> 32);
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

// Host: packed constants of a parameter set (pencil_kernel.hip).
PencilArgs make_args(const KParams &kp, bool f16, bool vs);

// Instantiated helix shapes: M = 1, 2, 4, 8 pairs per lane (LC up to 128 M),
// 8 rows per workgroup; each in f16 / int16 arithmetic and RTL / SOP s3.
#define TSA_SHAPES(LAUNCH, M_, F16_, SOP_, ...)                                            \
  ((M_) == 1 ? TSA_ARITH(LAUNCH, 1, 8, F16_, SOP_, __VA_ARGS__)                            \
   : (M_) == 2 ? TSA_ARITH(LAUNCH, 2, 8, F16_, SOP_, __VA_ARGS__)                          \
   : (M_) == 4 ? TSA_ARITH(LAUNCH, 4, 8, F16_, SOP_, __VA_ARGS__)                          \
               : TSA_ARITH(LAUNCH, 8, 8, F16_, SOP_, __VA_ARGS__))
#define TSA_ARITH(LAUNCH, MM, NN, F16_, SOP_, ...)                                        \
  ((F16_) ? ((SOP_) ? LAUNCH<MM, NN, true, true>(__VA_ARGS__)                              \
                    : LAUNCH<MM, NN, true, false>(__VA_ARGS__))                            \
          : ((SOP_) ? LAUNCH<MM, NN, false, true>(__VA_ARGS__)                             \
                    : LAUNCH<MM, NN, false, false>(__VA_ARGS__)))

}  // namespace tsa
