// lap_kernel.hip -- TSA_KERNEL_PENCIL single-cube (lap) schedule.
//
// One cube (or a few) is cut into laps of RW = 2*NW rows (y) and z-tiles of
// ZT = 64*M positions; every (lap, tile) is its own workgroup and all of them
// run at once, chained through global memory -- the reference's slicing of
// the (y,z) plane into pencils with face SRAMs between them
// (src/TriAlign_1cyc.v:78-98,127-140, pic/Memory.png), with workgroups in place
// of the 8x8 PE array's passes and HBM rings in place of the face SRAMs.
//
// Inside a workgroup (tools/lap_emu.py replays this schedule on the CPU):
//  * NW compute waves; wave w holds TWO DP rows, y = L*RW + 2w + 1 in the low
//    16-bit half and y + 1 in the high half of every packed register;
//  * lane l, register i is tile position k = M*l + i (z = q*ZT + k + 1); half
//    h of wave w computes x = t - (2w + h) - k + 1 at local step t;
//  * the high half's row above is the wave's own low half one step earlier, the
//    low half's is wave w-1's high half of step t-1: one v_alignbit/v_perm per
//    record word (REC = {above.hi, own_prev.lo});
//  * z-1 neighbours shift one position per step (register rename, one DPP
//    wave_ror + one v_perm per message), the x = 1 position takes the x = 0
//    face (src/PE_1cyc.v:164-218 EN_i gating), as in the helix kernel.
// No workgroup barrier per step: the waves are a pipeline, each running its
// own loop and synchronised point to point through LDS (a systolic array of
// waves, as the RTL's PEs are one of registers):
//  * wave w writes its record of step t into an LDS ring of K slots and then
//    its progress word (t + 1); wave w+1 polls that word before reading, and
//    wave w polls wave w+1's before reusing a slot. A step costs one wave's
//    own instruction stream; the hand-off latency is paid once per wave, not
//    once per step (a barrier makes every step pay it);
//  * wave NW is the LOADER: it LDS-DMAs the records of the lap above (y) and of
//    the tile to the left (z) LPD steps ahead, checks their tags, re-fetches
//    stale ones and publishes its own progress word, which wave 0 polls -- the
//    global hand-off's latency and checks are off the compute waves' path.
// Between workgroups (MI355X_MICROARCH.md "handoff-1to1"):
//  * the last compute wave stores its per-step record (the high halves the
//    next lap's wave 0 needs) into a y ring of YR slots, and every wave's
//    lane 63 its last position ({Iz, Ixz, REC.z, REC.w}) into a z ring of ZR
//    slots for tile q+1;
//  * every 8-byte granule of a record carries a 32-bit tag of (launch epoch,
//    step), written by one sc1 store; the loader checks the tags (no flags on
//    the fast path); a stale tag re-fetches (bounded; on timeout the launch's
//    error word is set and the triple reports TSA_SCORE_INVALID);
//  * the rings are O(N^2) (O(N) per workgroup): a consumer publishes how far
//    its loader has checked, and a producer about to overwrite a slot the
//    consumer may still need waits for it (never on the fast path: the rings
//    hold 2-4x the natural lag);
//  * block b -> XCD b % 8 (observed dispatch, speed only): every lap of a z-tile
//    lands on one XCD, so the y chain's hand-offs stay in one L2's reach.
// A consumer only waits on laps of lower index (lap-major order), and a
// producer waits (back-pressure) only on a consumer of its own round -- across
// a round boundary its ring is full length. A grid beyond the resident slots is
// launched as one resident round (8 x SX workgroups) whose workgroups loop over
// their slots' later-round laps in lap order (up to LAP_MAX_WAVES rounds, any
// workgroups per CU), so no wait depends on the dispatcher's order; forward
// progress needs every launched workgroup co-resident (every wait is bounded
// and reports TSA_SCORE_INVALID).

#include <unistd.h>

#include <atomic>
#include <ctime>
#include <mutex>
#include <vector>

#include "pencil_common.h"
#include "lap_kernel.h"
#include "kernel_meta.h"

namespace tsa {

#ifndef TSA_LAP_PD1  // loader prefetch distance (steps) by M: build-time knobs. Short
#define TSA_LAP_PD1 2  // wins: a fetch issued before its producer stored is a tag miss
#endif                 // and a serial re-fetch (A/B on MI355X: 2 < 3 < 4 < 6)
#ifndef TSA_LAP_PD2
#define TSA_LAP_PD2 2
#endif
#ifndef TSA_LAP_PD4
#define TSA_LAP_PD4 3
#endif
__host__ __device__ constexpr int lap_pd(int M) {
  return M == 1 ? TSA_LAP_PD1 : M == 2 ? TSA_LAP_PD2 : TSA_LAP_PD4;
}
// LDS ring slots: wave -> wave (K) and loader -> wave 0 (K0); powers of 2
__host__ __device__ constexpr int lap_k(int M) { return M == 1 ? 4 : 2; }
__host__ __device__ constexpr int lap_k0(int M) { return M <= 2 ? 8 : 4; }
constexpr int LAP_ZL = 32;           // z records resident in LDS (power of 2)
constexpr int LAP_PUB = 4;           // the last wave publishes the consumer progress every LAP_PUB steps
constexpr int LAP_PROG_STRIDE = 32;  // progress words 128 B apart (one line each)
constexpr int LAP_ZREC_WAVE = 32;    // z record bytes per wave: 2 x {payload, tag, payload, tag}

static_assert(LAP_ZL >= 8 + 2 + TSA_LAP_PD1 + 2 && LAP_ZL >= 8 + 2 + TSA_LAP_PD2 + 2, "z slots");

// Tag of the record of step s in the launch with epoch e (32-bit): distinct
// steps of one launch never collide (odd multiplier).
__host__ __device__ __forceinline__ uint32_t lap_tag(uint32_t e, int32_t s) {
  return e ^ ((uint32_t)s * 0x9E3779B1u);
}

// A code pairs the table holds: the LIT loader reads a few entries further
// (its z = 0 faces run ZA steps ahead of the last compute step)
__host__ __device__ constexpr int32_t lap_na(int32_t la, int M, int NW, bool lit) {
  return la + 2 * 64 * M + 4 * NW + 8 + (lit ? 2 * NW + 8 : 0);
}
// final-cell words: best of the final step, or (LIT) its 7 input states + 8
__host__ __device__ constexpr int lap_fin_words(int M, bool lit) { return lit ? 7 * M * 64 + 8 : M * 64; }
static size_t lap_lds_bytes(int M, int NW, int32_t max_la, bool lit = false) {
  const int SLOT = M * 1024;
  return (size_t)(NW - 1) * lap_k(M) * SLOT + (size_t)lap_k0(M) * SLOT +
         (size_t)LAP_ZL * NW * LAP_ZREC_WAVE + (size_t)SLOT + (size_t)NW * LAP_ZREC_WAVE + 16 * 4 +
         (size_t)(NW + 1) * 256 + (size_t)lap_fin_words(M, lit) * 4 +
         4 * (((size_t)lap_na(max_la, M, NW, lit) + 3) & ~(size_t)3);
}

// Trace slots per block (TSA_LAP_TRACE): 8, plus with TSA_DIAG (the
// diagnostic build, scripts/build_variant.sh) 4 shader-clock accumulators per
// compute wave and the largest producer-consumer lag (steps) seen by the y and
// z stores -- the ring slots that workgroup needed.
#if defined(TSA_DIAG)
constexpr int LAP_TRACE_SLOTS = 8 + 4 * 8 + 2;
#else
constexpr int LAP_TRACE_SLOTS = 8;
#endif

// ---------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// The s_nop: a VMEM store of more than 8 bytes must not have its data VGPRs
// rewritten by the next VALU instruction (one wait state); the compiler's
// hazard recognizer does not look inside inline asm, so the asm carries it.
// SYS (a cube split over devices, lap_launch_split): system scope (sc0 sc1),
// so a record written into a peer device's fine-grained ring is visible there.
template <bool SYS = false>
__device__ __forceinline__ void store16_sc1(void *gptr, uint4 v) {
  const u32x4 d = {v.x, v.y, v.z, v.w};
  if constexpr (SYS)
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(gptr), "v"(d) : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(gptr), "v"(d) : "memory");
}
// the same store at sbase + voff + OFFB (SGPR base, 32-bit VGPR offset, immediate)
template <bool SYS, int OFFB>
__device__ __forceinline__ void store16_sc1_s(const uint8_t *sbase, uint32_t voff, uint4 v) {
  static_assert(OFFB >= 0 && OFFB < 4096, "13-bit signed global offset");
  const u32x4 d = {v.x, v.y, v.z, v.w};
  if constexpr (SYS)
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 sc0 sc1\n\ts_nop 1" ::"v"(voff), "v"(d), "s"(sbase),
                 "i"(OFFB)
                 : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 sc1\n\ts_nop 1" ::"v"(voff), "v"(d), "s"(sbase),
                 "i"(OFFB)
                 : "memory");
}
// the same store at gptr + OFFB (the instruction's immediate offset)
template <bool SYS, int OFFB>
__device__ __forceinline__ void store16_sc1_at(void *gptr, uint4 v) {
  static_assert(OFFB >= 0 && OFFB < 4096, "13-bit signed global offset");
  const u32x4 d = {v.x, v.y, v.z, v.w};
  if constexpr (SYS)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc0 sc1\n\ts_nop 1" ::"v"(gptr), "v"(d), "i"(OFFB)
                 : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc1\n\ts_nop 1" ::"v"(gptr), "v"(d), "i"(OFFB)
                 : "memory");
}
__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}
// {above.hi -> lo, own.lo -> hi}: the row above of both halves
__device__ __forceinline__ uint32_t rows2(uint32_t own, uint32_t above) {
  return __builtin_amdgcn_alignbit(own, above, 16);
}
// f16 bits of the integer lam * v in both halves (V-space face values; exact
// below 2048 in magnitude, which the host's range check guarantees)
__device__ __forceinline__ uint32_t lam_bits(int32_t lam, int32_t v) {
  const _Float16 h = (_Float16)(float)(lam * v);
  return (uint32_t)__builtin_bit_cast(uint16_t, h) * 0x00010001u;
}
// A wave-uniform 64-bit lane mask, forced into an SGPR pair (the compiler may
// compute a uniform shift in VALU and hand the VGPR pair to an "s" operand)
__device__ __forceinline__ uint64_t sgpr64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int32_t lds_word(const int32_t *p) {
  return __builtin_amdgcn_readfirstlane(
      *(volatile const __attribute__((address_space(3))) int32_t *)(
          const __attribute__((address_space(3))) void *)p);
}
// Progress word store: every lane writes its own copy (pw[wave][lane], one
// conflict-free ds_write_b32, no exec toggling); readers read lane 0's. LDS
// executes a wave's DS instructions in order, so a reader that sees the word
// also sees the record written before it; the empty asm keeps the compiler
// from moving LDS accesses across it.
__device__ __forceinline__ void lds_publish(int32_t *pw_wave, int32_t v, int lane) {
  asm volatile("" ::: "memory");
  *(volatile __attribute__((address_space(3))) int32_t *)(__attribute__((address_space(3))) void *)(
      pw_wave + lane) = v;
  asm volatile("" ::: "memory");
}
// Lane bit `k` of a 64-bit exec-style mask when 0 <= k < 64, else 0 -- in SALU
// (left to itself the compiler shifts a 64-bit 1 in VALU and reads it back).
__device__ __forceinline__ uint64_t lane_bit(int32_t k) {
  uint64_t r;
  asm("s_lshl_b64 %0, 1, %1\n\ts_cmp_lt_u32 %1, 64\n\ts_cselect_b64 %0, %0, 0"
      : "=&s"(r) : "s"(k) : "scc");
  return r;
}

// The lap kernel's cell, split at the row above (the message form of
// cell_messages_f16 / cell_messages, src/PE_1cyc.v:159-218): of a step's
// inputs only Iy comes from this step's record -- x-1, z-1, the diagonals and
// the scores are known when the step starts -- so every message is folded to
// max(Y - c, N) with the N's computed while the record is read. GO >= GE
// orders the penalties (E <= O, 2E <= O+E <= 2O, f16 form with the mismatch
// folded into E and O alike), so Y's dominated copies drop out:
//   best = max(Y, W),       W  = max(X, Z, XY, XZ, YZ, M)
//   Ix'  = max(Y - OE, N1), N1 = max(X - 2E, U1 - OE, W - 2O), U1 = max(X, Z, XY, XZ)
//   Iy'  = max(Y - 2E, N2), N2 = max(U2 - OE, W - 2O),         U2 = max(X, Z, XY, YZ)
//   Iz'  = max(Y - OE, N3), N3 = max(Z - 2E, U3 - OE, W - 2O), U3 = max(X, Z, XZ, YZ)
//   Ixy' = max(Y - E, N4),  N4 = max(max(X, XY) - E, W - O)
//   Iyz' = max(Y - E, N5),  N5 = max(max(YZ, Z) - E, W - O)
//   Ixz' = max(Y - O, N6),  N6 = max(max(X, Z, XZ) - E, W - O)
// (11 dependent instructions per pair after the record lands instead of ~30).
template <int M>
struct LapPre {
  uint32_t W[M], N1[M], N2[M], N3[M], N4[M], N5[M], N6[M];
};
template <int M, bool SOP>
__device__ __forceinline__ void lap_pre_f16(const uint32_t (&a)[M], const uint32_t (&b)[M],
                                            const uint32_t (&c)[M], const uint32_t (&SBC)[M],
                                            const uint32_t (&K)[M], const uint32_t (&DMC)[M],
                                            uint32_t Q, const PencilArgs &pa,
                                            const uint32_t (&inIx)[M], const uint32_t (&inIz)[M],
                                            const uint32_t (&inIxy)[M], const uint32_t (&inIyz)[M],
                                            const uint32_t (&inIxz)[M], const uint32_t (&inM)[M],
                                            LapPre<M> &p) {
  const h2 DM = H(pa.h_dm), E = H(pa.E), O = H(pa.O), E2 = H(pa.E2), OE = H(pa.OE), O2 = H(pa.O2);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const h2 eab = H(umin2(a[i] & b[i], Q)), eac = H(a[i] & c[i]), DMCi = H(DMC[i]);
    const h2 sXY = hfma(eab, DM, H(inIxy[i]));  // src/PE_1cyc.v:159-161 (+mismatch folded)
    const h2 sXZ = hfma(eac, DMCi, H(inIxz[i]));
    const h2 sYZ = H(inIyz[i]) + H(SBC[i]);
    h2 sM;                                       // src/PE_1cyc.v:162
    if constexpr (SOP) sM = hfma(eab, DM, hfma(eac, DMCi, H(inM[i]))) + H(K[i]);
    else sM = hfma(eab, H(K[i]), H(inM[i])) + H(pa.h_c3);
    const h2 X = H(inIx[i]), Z = H(inIz[i]);
    const h2 pXZ = hmax(X, Z);
    const h2 U1 = vmax3(pXZ, sXY, sXZ), U2 = vmax3(pXZ, sXY, sYZ), U3 = vmax3(pXZ, sYZ, sXZ);
    const h2 W = vmax3(U1, sYZ, sM);
    const h2 WO = W - O, WO2 = W - O2;
    p.W[i] = U(W);
    p.N1[i] = U(vmax3(X - E2, U1 - OE, WO2));
    p.N2[i] = U(hmax(U2 - OE, WO2));
    p.N3[i] = U(vmax3(Z - E2, U3 - OE, WO2));
    p.N4[i] = U(hmax(hmax(X, sXY) - E, WO));
    p.N5[i] = U(hmax(hmax(sYZ, Z) - E, WO));
    p.N6[i] = U(hmax(hmax(pXZ, sXZ) - E, WO));
  }
}
template <int M>
__device__ __forceinline__ void lap_post_f16(const PencilArgs &pa, const uint32_t (&Y)[M],
                                             const LapPre<M> &p, uint32_t (&nIx)[M],
                                             uint32_t (&oIy)[M], uint32_t (&oIz)[M],
                                             uint32_t (&oIxy)[M], uint32_t (&oIyz)[M],
                                             uint32_t (&oIxz)[M], uint32_t (&oBest)[M]) {
  const h2 E = H(pa.E), O = H(pa.O), E2 = H(pa.E2), OE = H(pa.OE);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const h2 y = H(Y[i]), yOE = y - OE, yE = y - E;
    oBest[i] = U(hmax(y, H(p.W[i])));
    nIx[i] = U(hmax(yOE, H(p.N1[i])));
    oIy[i] = U(hmax(y - E2, H(p.N2[i])));
    oIz[i] = U(hmax(yOE, H(p.N3[i])));
    oIxy[i] = U(hmax(yE, H(p.N4[i])));
    oIyz[i] = U(hmax(yE, H(p.N5[i])));
    oIxz[i] = U(hmax(y - O, H(p.N6[i])));
  }
}
// The V-space cell (cell_messages_vs: every value of cell (x,y,z) shifted by
// lam (x+y+z), lam = GE = -MISMATCH) split at the row above the same way.
// With Gx = max(Y, gx), Gz = max(Y, gz), best = max(Y, W) and DO = GO - GE
// >= 0, CP = GO + MISMATCH + lam >= lam (tests/test_cell_algebra.py):
//   W  = max(gx, Gy, XY', M'),  gx = max(Z, YZ'), gz = max(X, XY'), Gy = max(X, Z, XZ')
//   Ixy' = max(Y, NXY),      NXY = max(gz, W - DO)
//   Iyz' = max(Y, NYZ),      NYZ = max(gx, W - DO)
//   Ixz' = max(Y - DO, NXZ), NXZ = max(Gy, W - DO)
//   Ix'  = max(Y - CP, N1),  N1 = max(X - lam, NXY - CP, NXZ - CP)
//   Iy'  = max(Y - lam, N2), N2 = max(NXY - CP, NYZ - CP)
//   Iz'  = max(Y - CP, N3),  N3 = max(Z - lam, NYZ - CP, NXZ - CP)
// 23 instructions per pair before the record lands, 10 after (the message
// form: 32 + 11). LapPre slots: N4 = NXY, N5 = NYZ, N6 = NXZ.
template <int M, bool SOP>
__device__ __forceinline__ void lap_pre_vs(const uint32_t (&a)[M], const uint32_t (&b)[M],
                                           const uint32_t (&c)[M], const uint32_t (&SBC)[M],
                                           const uint32_t (&K)[M], const uint32_t (&DMC)[M],
                                           const uint32_t (&DMB)[M], const PencilArgs &pa,
                                           const uint32_t (&inIx)[M], const uint32_t (&inIz)[M],
                                           const uint32_t (&inIxy)[M], const uint32_t (&inIyz)[M],
                                           const uint32_t (&inIxz)[M], const uint32_t (&inM)[M],
                                           LapPre<M> &p) {
  const h2 LAM = H(pa.v_lam), CP = H(pa.v_cP), DO = H(pa.v_dO);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const h2 eab = H(a[i] & b[i]), eac = H(a[i] & c[i]), DMCi = H(DMC[i]), DMBi = H(DMB[i]);
    const h2 sXY = hfma(eab, DMBi, H(inIxy[i]));  // src/PE_1cyc.v:159-161 (+mismatch folded)
    const h2 sXZ = hfma(eac, DMCi, H(inIxz[i]));
    const h2 sYZ = H(inIyz[i]) + H(SBC[i]);
    h2 sM;                                        // src/PE_1cyc.v:162
    if constexpr (SOP) sM = hfma(eab, DMBi, hfma(eac, DMCi, H(inM[i]))) + H(K[i]);
    else sM = hfma(eab, H(K[i]), H(inM[i]));      // ne + 3 lam = 0
    const h2 X = H(inIx[i]), Z = H(inIz[i]);
    const h2 gx = hmax(Z, sYZ), gz = hmax(X, sXY), Gy = vmax3(X, Z, sXZ);
    const h2 W = vmax3(gx, Gy, hmax(sXY, sM));
    const h2 WD = W - DO;
    const h2 NXY = hmax(gz, WD), NYZ = hmax(gx, WD), NXZ = hmax(Gy, WD);
    const h2 qXY = NXY - CP, qYZ = NYZ - CP, qXZ = NXZ - CP;
    p.W[i] = U(W);
    p.N4[i] = U(NXY);
    p.N5[i] = U(NYZ);
    p.N6[i] = U(NXZ);
    p.N1[i] = U(vmax3(X - LAM, qXY, qXZ));
    p.N2[i] = U(hmax(qXY, qYZ));
    p.N3[i] = U(vmax3(Z - LAM, qYZ, qXZ));
  }
}
template <int M>
__device__ __forceinline__ void lap_post_vs(const PencilArgs &pa, const uint32_t (&Y)[M],
                                            const LapPre<M> &p, uint32_t (&nIx)[M],
                                            uint32_t (&oIy)[M], uint32_t (&oIz)[M],
                                            uint32_t (&oIxy)[M], uint32_t (&oIyz)[M],
                                            uint32_t (&oIxz)[M], uint32_t (&oBest)[M]) {
  const h2 LAM = H(pa.v_lam), CP = H(pa.v_cP), DO = H(pa.v_dO);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const h2 y = H(Y[i]), yCP = y - CP;
    oBest[i] = U(hmax(y, H(p.W[i])));
    oIxy[i] = U(hmax(y, H(p.N4[i])));
    oIyz[i] = U(hmax(y, H(p.N5[i])));
    oIxz[i] = U(hmax(y - DO, H(p.N6[i])));
    nIx[i] = U(hmax(yCP, H(p.N1[i])));
    oIy[i] = U(hmax(y - LAM, H(p.N2[i])));
    oIz[i] = U(hmax(yCP, H(p.N3[i])));
  }
}
// int16 form (two's complement halves): the same split of cell_messages
template <int M, bool SOP>
__device__ __forceinline__ void lap_pre_i16(const uint32_t (&a)[M], const uint32_t (&b)[M],
                                            const uint32_t (&c)[M], uint32_t ones,
                                            const PencilArgs &pa, const uint32_t (&inIx)[M],
                                            const uint32_t (&inIz)[M], const uint32_t (&inIxy)[M],
                                            const uint32_t (&inIyz)[M], const uint32_t (&inIxz)[M],
                                            const uint32_t (&inM)[M], LapPre<M> &p) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const uint32_t eab = pk_eq1(a[i], b[i], ones);
    const uint32_t eac = pk_eq1(a[i], c[i], ones);
    const uint32_t ebc = pk_eq1(b[i], c[i], ones);
    const uint32_t s2ab = pk_mad(eab, pa.dm, pa.mm);
    const uint32_t s2ac = pk_mad(eac, pa.dm, pa.mm);
    const uint32_t s2bc = pk_mad(ebc, pa.dm, pa.mm);
    uint32_t s3;
    if constexpr (SOP) s3 = pk_add(pk_add(s2ab, s2bc), s2ac);
    else s3 = pk_mad(eab, pk_mad(ebc, pa.s3_d1, pa.s3_d0), pa.s3_ne);
    const uint32_t sM = pk_add(inM[i], s3), X = inIx[i], Z = inIz[i];
    const uint32_t sXY = pk_add(inIxy[i], s2ab), sYZ = pk_add(inIyz[i], s2bc);
    const uint32_t sXZ = pk_add(inIxz[i], s2ac);
    const uint32_t pXZ = pk_max(X, Z);
    const uint32_t U1 = pk_max(pk_max(pXZ, sXY), sXZ), U2 = pk_max(pk_max(pXZ, sXY), sYZ);
    const uint32_t U3 = pk_max(pk_max(pXZ, sYZ), sXZ), W = pk_max(pk_max(U1, sYZ), sM);
    const uint32_t WO = pk_sub(W, pa.O), WO2 = pk_sub(W, pa.O2);
    p.W[i] = W;
    p.N1[i] = pk_max(pk_max(pk_sub(X, pa.E2), pk_sub(U1, pa.OE)), WO2);
    p.N2[i] = pk_max(pk_sub(U2, pa.OE), WO2);
    p.N3[i] = pk_max(pk_max(pk_sub(Z, pa.E2), pk_sub(U3, pa.OE)), WO2);
    p.N4[i] = pk_max(pk_sub(pk_max(X, sXY), pa.E), WO);
    p.N5[i] = pk_max(pk_sub(pk_max(sYZ, Z), pa.E), WO);
    p.N6[i] = pk_max(pk_sub(pk_max(pXZ, sXZ), pa.E), WO);
  }
}
template <int M>
__device__ __forceinline__ void lap_post_i16(const PencilArgs &pa, const uint32_t (&Y)[M],
                                             const LapPre<M> &p, uint32_t (&nIx)[M],
                                             uint32_t (&oIy)[M], uint32_t (&oIz)[M],
                                             uint32_t (&oIxy)[M], uint32_t (&oIyz)[M],
                                             uint32_t (&oIxz)[M], uint32_t (&oBest)[M]) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const uint32_t y = Y[i], yOE = pk_sub(y, pa.OE), yE = pk_sub(y, pa.E);
    oBest[i] = pk_max(y, p.W[i]);
    nIx[i] = pk_max(yOE, p.N1[i]);
    oIy[i] = pk_max(pk_sub(y, pa.E2), p.N2[i]);
    oIz[i] = pk_max(yOE, p.N3[i]);
    oIxy[i] = pk_max(yE, p.N4[i]);
    oIyz[i] = pk_max(yE, p.N5[i]);
    oIxz[i] = pk_max(pk_sub(y, pa.O), p.N6[i]);
  }
}

// LIT: the literal push-form cell (literal_kernel.hip:push_literal, the RTL's
// src/PE_1cyc.v:164-218 with every candidate wrapped at SCORE_BITS), split at
// the row above the same way: every candidate but Y's is maxed before the
// record lands, Y's seven after it (13 instructions per pair). an / bn / cn:
// the successors' symbol codes (a_{x'+1}, b_{y+1}, c_{z+1}); UYZ = s2(b_{y+1},
// c_{z+1}) - GE and K1 (the [b=c] part of s3) are per-position constants.
template <int M>
struct LitPre {
  uint32_t pIx[M], pIy[M], pIz[M], pIxy[M], pIyz[M], pIxz[M], pM[M], uxy[M], vxz[M], s3[M];
};
template <int M, bool SOP>
__device__ __forceinline__ void lit_pre(const LitArgs &c, const LitArgs &cv, uint32_t ones,
                                        const uint32_t (&an)[M], uint32_t bn, const uint32_t (&cn)[M],
                                        const uint32_t (&UYZ)[M], const uint32_t (&K1)[M],
                                        const uint32_t (&X)[M], const uint32_t (&Z)[M],
                                        const uint32_t (&XY)[M], const uint32_t (&YZ)[M],
                                        const uint32_t (&XZ)[M], const uint32_t (&MM)[M], LitPre<M> &p) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    // single targets, less Y's candidates (src/PE_1cyc.v:172-194)
    const uint32_t m2O = pk_add(MM[i], c.n2O);
    const uint32_t x2E = pk_add(X[i], c.n2E), xOE = pk_add(X[i], c.nOE);
    const uint32_t z2E = pk_add(Z[i], c.n2E), zOE = pk_add(Z[i], c.nOE);
    const uint32_t xyOE = pk_add(XY[i], c.nOE), xy2O = pk_add(XY[i], c.n2O);
    const uint32_t yzOE = pk_add(YZ[i], c.nOE), yz2O = pk_add(YZ[i], c.n2O);
    const uint32_t xzOE = pk_add(XZ[i], c.nOE), xz2O = pk_add(XZ[i], c.n2O);
    const uint32_t A = pk_max(pk_max(m2O, zOE), xyOE), Bv = pk_max(xOE, yzOE);
    p.pIx[i] = pk_max(pk_max(A, x2E), pk_max(yz2O, xzOE));
    p.pIy[i] = pk_max(pk_max(A, Bv), xz2O);
    p.pIz[i] = pk_max(pk_max(Bv, m2O), pk_max(z2E, pk_max(xy2O, xzOE)));
    // the successors' pair scores less GE (u) and less GO (v), src/PE_1cyc.v:159-161
    const uint32_t eab = pk_eq1(an[i], bn, ones), eac = pk_eq1(an[i], cn[i], ones);
    const uint32_t uxy = pk_mad(eab, cv.dmS, cv.mmE), vxy = pk_add(uxy, c.nDOE);
    const uint32_t uxz = pk_mad(eac, cv.dmS, cv.mmE), vxz = pk_add(uxz, c.nDOE);
    const uint32_t uyz = UYZ[i], vyz = pk_add(uyz, c.nDOE);
    p.pIxy[i] = pk_max(pk_max(pk_max(pk_add(X[i], uxy), pk_add(XY[i], uxy)), pk_max(pk_add(MM[i], vxy), pk_add(Z[i], vxy))),
                       pk_max(pk_add(YZ[i], vxy), pk_add(XZ[i], vxy)));
    p.pIyz[i] = pk_max(pk_max(pk_max(pk_add(Z[i], uyz), pk_add(YZ[i], uyz)), pk_max(pk_add(MM[i], vyz), pk_add(X[i], vyz))),
                       pk_max(pk_add(XY[i], vyz), pk_add(XZ[i], vyz)));
    p.pIxz[i] = pk_max(pk_max(pk_max(pk_add(X[i], uxz), pk_add(Z[i], uxz)), pk_max(pk_add(XZ[i], uxz), pk_add(MM[i], vxz))),
                       pk_max(pk_add(XY[i], vxz), pk_add(YZ[i], vxz)));
    // M: every state plus the successor's triple score (src/PE_1cyc.v:162-170)
    uint32_t s3;
    if constexpr (SOP) s3 = pk_mad(eab, cv.dmS, pk_mad(eac, cv.dmS, K1[i]));
    else s3 = pk_mad(eab, K1[i], cv.neS);
    p.pM[i] = pk_max(pk_max(pk_max(pk_add(MM[i], s3), pk_add(X[i], s3)), pk_max(pk_add(Z[i], s3), pk_add(XY[i], s3))),
                     pk_max(pk_add(YZ[i], s3), pk_add(XZ[i], s3)));
    p.uxy[i] = uxy;
    p.vxz[i] = vxz;
    p.s3[i] = s3;
  }
}
template <int M>
__device__ __forceinline__ void lit_post(const LitArgs &c, const uint32_t (&Y)[M], const uint32_t (&UYZ)[M],
                                         const LitPre<M> &p, uint32_t (&nIx)[M], uint32_t (&oIy)[M],
                                         uint32_t (&oIz)[M], uint32_t (&oIxy)[M], uint32_t (&oIyz)[M],
                                         uint32_t (&oIxz)[M], uint32_t (&oM)[M]) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const uint32_t y = Y[i], yOE = pk_add(y, c.nOE);
    nIx[i] = pk_max(p.pIx[i], yOE);
    oIy[i] = pk_max(p.pIy[i], pk_add(y, c.n2E));
    oIz[i] = pk_max(p.pIz[i], yOE);
    oIxy[i] = pk_max(p.pIxy[i], pk_add(y, p.uxy[i]));
    oIyz[i] = pk_max(p.pIyz[i], pk_add(y, UYZ[i]));
    oIxz[i] = pk_max(p.pIxz[i], pk_add(y, p.vxz[i]));
    oM[i] = pk_max(p.pM[i], pk_add(y, p.s3[i]));
  }
}
// A zero cell's pushes (the faces) into a pair target and into M, per half:
// s2 of the successor's pair as fP[0] / fP[1], and s3 wrapped (P[M][*] = 0)
__device__ __forceinline__ uint32_t lit_face_pair(const LitArgs &cv, uint32_t p, uint32_t q, uint32_t ones) {
  return pk_mad(pk_eq1(p, q, ones), pk_sub(cv.fP[1], cv.fP[0]), cv.fP[0]);
}
template <bool SOP>
__device__ __forceinline__ uint32_t lit_face_m(const LitArgs &cv, uint32_t an, uint32_t bn, uint32_t cn,
                                               uint32_t ones) {
  const uint32_t eab = pk_eq1(an, bn, ones), ebc = pk_eq1(bn, cn, ones), eac = pk_eq1(an, cn, ones);
  if constexpr (SOP) return pk_mad(eab, cv.dmS, pk_mad(ebc, cv.dmS, pk_mad(eac, cv.dmS, cv.mm3S)));
  else return pk_mad(eab, pk_mad(ebc, cv.d1S, cv.d0S), cv.neS);
}

// LDS (bytes):
//   xr    [NW-1][K][M][64][16]  wave w -> w+1 records {Iy, Ixy, Iyz, best}
//   xr0   [K0][M][64][16]       tagged y records of the lap above (loader, LDS-DMA)
//   zring [ZL][NW][32]          tagged z records of the tile to the left (loader)
//   yface [M][64][16]           y = 0 face in wave 0's record format (lap 0)
//   zface [NW][32]              z = 0 face in the z record format (tile 0)
//   wd    [16] i32              [9] back-pressure waits, [12] abort, [13..14] the
//                               consumers' progress (LDS-DMA'd), [15] loader stalls
//   pw    [NW+1][64] i32        progress words (steps done): compute wave w, loader NW
//   fin   [M][64] u32           best of the final step (LIT: [7][M][64] its input
//                               states, then the 7 unshifted values)
//   sA2   [..] u32              A code pairs: entry j = x j-OFF (lo), j-OFF-1 (hi)
// Minimum waves per SIMD the register allocation must allow. A workgroup's
// NW + 1 waves may sit ceil((NW + 1) / 4) to a SIMD (the dispatcher need not
// balance them), so two NW = 8 workgroups per CU need 6 waves per SIMD, i.e.
// <= 80 VGPRs: with 96 (5 waves) the CU admitted one, and the second half of
// a 1024^3 lap grid started only as the first half finished (ring-lag census,
// profiles/r3e_lap_lag.jsonl). M = 1 keeps 6 for the plain forms (the int16
// one needs the cap to stay two per CU, tests/test_kernel_meta.py) and asks
// for 4 for the checked and literal ones, which spill 8 bytes at 6; the f16
// single cubes stay <= 80 VGPRs either way and ran alike (same box: 64^3
// 0.0741 ms at 4 vs 0.0748 at 6, 256^3 0.351 vs 0.356; without the per-lap
// index launder (TSA_LAP_LAUNDER=0) 256^3 0.366, profiles/r4j_single_ab.jsonl).
// M >= 4 runs one per CU.
#ifndef TSA_LAP_WPE2
#define TSA_LAP_WPE2 4
#endif
#ifndef TSA_LAP_WPE2C  // the checked M = 2 form (5: 1024^3 3.38 vs 3.24 ms, profiles/r4q_checked_ab.jsonl)
#define TSA_LAP_WPE2C 4
#endif
#ifndef TSA_LAP_LAUNDER
#define TSA_LAP_LAUNDER 1
#endif
#ifndef TSA_LAP_WPE1
#define TSA_LAP_WPE1 6
#endif
// The checked kernel's monitor: per-wave slots written with plain stores and
// reduced per triple by lap_certify (1), or two same-address atomics per wave
// (0, rounds 1-4). Thousands of waves of one cube contend for the two words,
// and a looped workgroup waits for its atomics (vmcnt(0)) before its next lap.
#ifndef TSA_CHK_SLOTS
#define TSA_CHK_SLOTS 1
#endif
// Lean step: the producer's progress word read every step (no poll flag kept
// in a VGPR across the pre-cell, no conditional read), and the next A codes
// at a constant offset from a base set once per step pair
#ifndef TSA_LAP_LEAN
#define TSA_LAP_LEAN 1
#endif
// wave 0 reads only the payload words of its tagged y record (ds_read2_b32):
// a 16-byte read hands the compiler the two dead tag registers, which it
// reuses before the read has landed -- a write-after-write wait that puts
// the record read's latency in front of the pre-cell
#ifndef TSA_LAP_Y2  // (measured: 64^3 / 256^3 / 512^3 0.5-1 % faster, profiles/r5a_lap_y2_ab.jsonl)
#define TSA_LAP_Y2 1
#endif
// Four-step groups: a step's ring slots, z / y record addresses and next A
// codes sit at constant offsets (instruction immediates) from bases set once
// per group of four steps -- every ring length is a multiple of 4 and ZT of
// LAP_ZL -- instead of being computed every step. The message forms' constant
// y = 0 / z = 0 faces are prefilled into every slot of xr0 / zring (which the
// loader then leaves alone), so the offsets never depend on yin / zin.
#ifndef TSA_LAP_U4
#define TSA_LAP_U4 1
#endif
// In a four-step group, the back-pressure checks batched: the consumers' ring
// room once per group (for its last step; the rings hold >= 32 slots), the
// successor wave's slot every other step for K = 4 (covering the next step:
// it needs the successor past step t - 2 at the end of step t, which it
// normally is, one step behind)
#ifndef TSA_LAP_GCHK
#define TSA_LAP_GCHK 1
#endif
// In a four-step group, every LDS base a step reads or writes (the input and
// output record rings, the group's y / z ring slots, the two progress words)
// held in a VGPR laundered once per lap / group, so each access is one ds
// instruction with a constant offset; left alone the compiler keeps the
// uniform part in SGPRs -- one per ring slot, spilled to VGPR lanes -- and
// rebuilds every address with v_readlane / v_mov / v_add each step. The ring
// records go out through the SGPR-base form of global_store (no 64-bit VGPR
// address per store).
#ifndef TSA_LAP_VBASE
#define TSA_LAP_VBASE 1
#endif
// The loader fetches each ring record (two {payload, tag} granules) with one
// 16-byte load instead of two 8-byte ones: 2M + 2 load instructions per step
// become M + 1 (plus the progress words). 0: two 8-byte atomic loads; 1: a
// volatile 16-byte load (measured 1.8x slower: the memory legalizer follows
// each volatile load with vmcnt(0), serialising the fetch window,
// profiles/r5f_lap_loader_ab.jsonl); 2: a raw buffer load with sc1 (counted by
// the compiler like the atomics); -1 (default): 2 for the M = 1 forms, 0 for
// the rest (with the progress words every 4 steps: factored 64^3 / 256^3 /
// 512^3 5-6 % faster, profiles/r5i_lap_loader_ab.jsonl; literal 512^3 / 1024^3
// 5 / 4 % faster, r5j_lap_loader_lit_ab.jsonl; the M = 2 checked 1024^3
// neutral)
#ifndef TSA_LAP_L16
#define TSA_LAP_L16 -1
#endif
// The consumers' progress words (the producers' back-pressure input, relayed
// through LDS) fetched every TSA_LAP_PROGP steps instead of every step: fewer
// loads in the loader's window (the consumers publish every LAP_PUB = 4 steps
// anyway; a staler relay only waits more, never less). The loader loop then
// runs in periods of max(LPD, PROGP) steps with a static phase. -1 (default):
// 4 for the M = 1 forms, 2 for the rest (profiles/r5h_lap_prog_ab.jsonl,
// r5i_lap_loader_ab.jsonl, r5j_lap_loader_lit_ab.jsonl).
#ifndef TSA_LAP_PROGP
#define TSA_LAP_PROGP -1
#endif
// With the buffer loads (TSA_LAP_L16 = 2): the fetches a lap-0 / tile-0 loader
// does not need (its y / z inputs are faces) out of range, so no memory access
// (measured neutral: 64^3 - 512^3 within 0.5 %, profiles/r5j_lap_noface_ab.jsonl)
#ifndef TSA_LAP_NOFACE_FETCH
#define TSA_LAP_NOFACE_FETCH 1
#endif
__host__ __device__ constexpr int lap_waves_per_eu(int M, bool lit = false, bool chk = false) {
  return lit ? (M == 1 ? 4 : 3) : M == 1 ? (chk ? 4 : TSA_LAP_WPE1) : M == 2 ? (chk ? TSA_LAP_WPE2C : TSA_LAP_WPE2) : 2;
}
// f(integral_constant<J>) for J = B .. E-1, unrolled at compile time
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
// every step of the lap kernel inlined (outlined, the captures go to scratch)
#define LAP_INLINE(call) \
  do {                    \
    [[clang::always_inline]] call; \
  } while (0)

// CHK (int16 form only): the checked kernel -- every real cell's best is
// folded into a per-lane max / min; each wave's extremes go to its own monitor
// slots (TSA_CHK_SLOTS), and lap_certify() reduces a triple's and decides whether
// any candidate of the literal RTL recurrence could have wrapped.
// A launch runs laps [L0, L1) of the cube (a single launch: [0, G)). SYS: one
// part of a cube split over devices (lap_launch_split) -- every hand-off load
// and store at system scope, the y ring of lap L1-1 written into the next
// part's workspace (yf_out, its consumer's memory) and the progress words of
// lap L0 into the previous part's (prog_in, its producer's memory), so every
// poll reads local memory and only posted stores cross the link.
// LIT: the literal RTL arithmetic (tools/litlap_emu.py replays it): the push-
// form cell of the literal helix on this schedule -- a position computes
// x' = u (x' = 0 the x = 0 face: its 7 inputs forced to 0, one more step), it
// pushes with its successors' symbols, the loader writes the y = 0 / z = 0
// faces (zero cells pushing with the receivers' symbols, so they vary with the
// step) into the rings wave 0 and position 0 read, values are shifted left by
// 16 - SCORE_BITS so int16 adds wrap at the RTL word, and the final cell's 7
// input states go to mon (aux) as its final 7-tuple.
// The kernel's arguments, bundled on the host and passed as separate
// __restrict__ parameters (LAP_KARGS). Measured: one by-value struct read
// through the kernarg segment pointer ran single cubes 15 % slower (64^3 0.087
// vs 0.075 ms, 256^3 0.40 vs 0.355 ms, same box, profiles/r4i_single_ab.jsonl)
// -- likely the no-alias guarantee the parameters carry and the fields do not.
struct LapKArgs {
  const uint8_t *seqs;
  const int64_t *offs;
  int32_t G, GZ, NC, CH, YR, ZR;
  uint8_t *yf_base, *zf_base;
  LapRounds rd;
  int32_t *prog;
  uint32_t *err;
  int32_t *scores, *mon;
  PencilArgs pa;
  uint32_t epoch, spin_limit;
  int32_t L0, L1;
  uint8_t *yf_out;
  int32_t *prog_in;
  unsigned long long *trace;
  LitArgs lit;
};
#define LAP_KARGS(k)                                                                                   \
  k.seqs, k.offs, k.G, k.GZ, k.NC, k.CH, k.YR, k.ZR, k.yf_base, k.zf_base, k.rd, k.prog, k.err, k.scores, \
      k.mon, k.pa, k.epoch, k.spin_limit, k.L0, k.L1, k.yf_out, k.prog_in, k.trace, k.lit
// VS: the V-space f16 cell (lap_pre_vs), every value shifted by lam (x+y+z):
// the faces become lam q (the x = 0 face injected at x = 1, the y = 0 / z = 0
// faces written by the loader like the literal form's), the score shifted
// back at the end.
template <int M, int NW, bool F16, bool SOP, bool CHK, bool SYS = false, bool LIT = false, bool VS = false>
__global__ __launch_bounds__(64 * (NW + 1), lap_waves_per_eu(M, LIT, CHK)) void lap_kernel(
    const uint8_t *__restrict__ seqs_, const int64_t *__restrict__ offs_, int32_t G_, int32_t GZ_,
    int32_t NC_, int32_t CH_, int32_t YR_, int32_t ZR_, uint8_t *__restrict__ yf_base_,
    uint8_t *__restrict__ zf_base_, LapRounds rd_, int32_t *__restrict__ prog_, uint32_t *__restrict__ err_,
    int32_t *__restrict__ scores_, int32_t *__restrict__ mon_, PencilArgs pa_, uint32_t epoch_,
    uint32_t spin_limit_, int32_t L0_, int32_t L1_, uint8_t *__restrict__ yf_out_,
    int32_t *__restrict__ prog_in_, unsigned long long *__restrict__ trace_, LitArgs lit_) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  static_assert(!(CHK && F16), "the checked kernel runs the int16 form");
  static_assert(!(CHK && SYS), "a split cube runs the unchecked forms");
  static_assert(!(LIT && (F16 || CHK)), "the literal form: int16, unchecked");
  static_assert(!VS || (F16 && !CHK && !LIT && !SYS), "V-space: the f16 single-device form");
  // the loader writes the step-varying y = 0 / z = 0 faces (LIT, VS)
  constexpr bool FACES = LIT || VS;
  // four-step groups (TSA_LAP_U4) for M <= 2 (M = 4's checked form spills with
  // them), their VGPR bases (TSA_LAP_VBASE) but for the M = 1 factored int16
  // forms (at the 80-VGPR cap of two NW = 8 workgroups per CU they spill 8 bytes)
  constexpr bool U4K = TSA_LAP_U4 && M <= 2;
  constexpr bool VBK = TSA_LAP_VBASE && U4K && (F16 || LIT || M == 2);
  // the loader's record loads and progress-word period (TSA_LAP_L16 / _PROGP)
  constexpr bool FM1 = M == 1;
  constexpr int L16K = TSA_LAP_L16 >= 0 ? TSA_LAP_L16 : FM1 ? 2 : 0;
  constexpr int PROGPK = TSA_LAP_PROGP >= 0 ? TSA_LAP_PROGP : FM1 ? 4 : 2;
  constexpr int SCOPE = SYS ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT;
  constexpr int RW = 2 * NW, ZT = 64 * M, LPD = lap_pd(M), K = lap_k(M), K0 = lap_k0(M);
  constexpr int PAIR = 64 * REC_BYTES, SLOT = M * PAIR;
  // wave w's rows sit at step offsets 2w (low half) and 2w + 1 (high); lap L+1
  // reads lap L's record t + YOFF; loader step s checks y record s + YOFF and
  // z record s + ZT + ZA (ZA = NW: every wave's z reads stay covered)
  constexpr int YOFF = 2 * (NW - 1) + 1, ZA = NW;
  constexpr int ZREC = NW * LAP_ZREC_WAVE, OFF = ZT + 2 * NW;
  uint8_t *xr = smem;
  uint8_t *xr0 = xr + (NW - 1) * K * SLOT;
  uint8_t *zring = xr0 + K0 * SLOT;
  uint8_t *yface = zring + LAP_ZL * ZREC;
  uint8_t *zface = yface + SLOT;
  int32_t *wd = (int32_t *)(zface + ZREC);
  int32_t *pw = wd + 16;
  uint32_t *fin = (uint32_t *)(pw + 64 * (NW + 1));
  uint32_t *sA2 = fin + lap_fin_words(M, LIT);
  int32_t *const w_bp = wd + 9, *const w_abort = wd + 12, *const bpw = wd + 13, *const w_stall = wd + 15;

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // w == NW: the loader
  // block -> (lap, column): column c = tri*GZ + q (one z-tile of one triple), block
  // b = 8 * (L*CH + c/8) + c%8 -- a column's laps share b % 8 (one XCD), and
  // every producer ((L-1, c), (L, c-1)) has a lower block index than its consumer
  // Dispatch rounds are a loop, not a hope: the grid holds one round (every
  // workgroup resident), and physical block p runs the logical blocks of
  // slots p/8, p/8 + SX, p/8 + 2 SX, ... of its XCD one after another -- lap
  // order per physical workgroup whatever the dispatcher does, and a slot's
  // next lap starts the moment its previous one ends. One round: one pass.
  auto lap_body = [&](const int32_t slot) {
  const uint8_t *__restrict__ seqs = seqs_;
  const int64_t *__restrict__ offs = offs_;
  const int32_t G = G_, GZ = GZ_, NC = NC_, CH = CH_, YR = YR_, ZR = ZR_;
  uint8_t *__restrict__ yf_base = yf_base_, *__restrict__ zf_base = zf_base_;
  const LapRounds &rd = rd_;
  int32_t *__restrict__ prog = prog_;
  uint32_t *__restrict__ err = err_;
  int32_t *__restrict__ scores = scores_, *__restrict__ mon = mon_;
  const PencilArgs &pa = pa_;
  const uint32_t epoch = epoch_, spin_limit = spin_limit_;
  const int32_t L0 = L0_, L1 = L1_;
  uint8_t *__restrict__ yf_out = yf_out_;
  int32_t *__restrict__ prog_in = prog_in_;
  unsigned long long *__restrict__ trace = trace_;
  const LitArgs &lit = lit_;
  const int32_t b = 8 * slot + (int32_t)(blockIdx.x & 7);  // logical block
  // the lane / thread index laundered per lap: otherwise the compiler hoists
  // every per-lane address out of the round loop and keeps it live across
  // the whole body (+20 VGPRs, measured), where one pass rematerialises them
  int32_t tid = (int32_t)threadIdx.x;
#if TSA_LAP_LAUNDER
  asm volatile("" : "+v"(tid));
#endif
  const int lane = tid & 63;
  const int32_t L = L0 + slot / CH, col = (slot % CH) * 8 + (b & 7);
  if (col >= NC || L >= L1) return;  // padding block
  const int32_t tri = col / GZ, q = col % GZ;
  const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
  const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
  const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
  const int32_t nlap = (lb + RW - 1) / RW, ntile = (lc + ZT - 1) / ZT;
  if (L >= nlap || q >= ntile) return;  // beyond this triple's own laps / tiles
  auto stamp = [&](int s, unsigned long long v) {
    if (trace != nullptr && tid == 0) trace[(int64_t)b * LAP_TRACE_SLOTS + s] = v;
  };
  auto now = [&]() {
    unsigned long long v;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    return v;
  };
  if (trace != nullptr) {
    stamp(0, now());
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    stamp(3, x);
  }
  const int64_t lid = ((int64_t)tri * G + L) * GZ + q;  // logical workgroup id
  const bool yin = L > 0, zin = q > 0, yout = L + 1 < nlap, zout = q + 1 < ntile;
  const int32_t zt_q = min(ZT, lc - q * ZT), rows = min(RW, lb - L * RW);
  const bool final_wg = !yout && !zout;
  auto tau = [](int32_t r) { return 2 * (r >> 1) + (r & 1); };  // step offset of lap row r
  const int32_t r_f = lb - 1 - L * RW, k_f = lc - 1 - q * ZT;
  constexpr int32_t LX = LIT ? 1 : 0;  // LIT: x' = 0 .. la, one step more
  const int32_t T = final_wg ? (la - 1 + LX) + tau(r_f) + k_f + 1 : la + LX + tau(rows - 1) + zt_q - 1;
  const int32_t T_above = la + LX + tau(RW - 1) + zt_q - 1;  // records the lap above writes (same tile)
  const int32_t T_left = la + LX + tau(rows - 1) + ZT - 1;   // z records the tile to the left writes
  // Rings. A grid beyond the resident slots runs in rounds of rd.SX slots per
  // XCD, each resident workgroup looping over its slots in lap order (the
  // slot loop at the end of lap_kernel). A producer whose consumer is in a later
  // round gets a full-length ring from the boundary region (it never waits
  // for a consumer that may not have started); all others a slim ring of
  // YR / ZR slots, their consumers co-resident (lap_geom).
  const int32_t ch = slot % CH, xc = b & 7;
  auto round_of = [&](int32_t s) { return s / rd.SX; };
  auto y_bidx = [&](int32_t Lp, int32_t sp) {  // boundary index of producer (Lp, my column), or -1
    const int32_t sc = sp + CH;
    if (round_of(sc) == round_of(sp)) return -1;
    return (int32_t)(((int64_t)col * rd.KBY) + (CH >= rd.SX ? Lp - L0 : round_of(sp) - round_of(ch)));
  };
  auto z_bidx = [&](int32_t sp, int32_t xp) {  // boundary index of producer (slot sp, XCD xp), or -1
    return (xp == 7 && round_of(sp + 1) != round_of(sp)) ? round_of(sp) : -1;
  };
  const int32_t yb_me = yout ? y_bidx(L, slot) : -1, yb_pr = yin ? y_bidx(L - 1, slot - CH) : -1;
  const int32_t zb_me = zout ? z_bidx(slot, xc) : -1;
  const int32_t zb_pr = zin ? (xc == 0 ? z_bidx(slot - 1, 7) : -1) : -1;
  const int32_t YRm = yb_me >= 0 ? rd.YRB : YR, YRp = yb_pr >= 0 ? rd.YRB : YR;
  const int32_t ZRm = zb_me >= 0 ? rd.ZRB : ZR, ZRp = zb_pr >= 0 ? rd.ZRB : ZR;
  uint8_t *yf_mine = yb_me >= 0 ? rd.yb + (int64_t)yb_me * rd.YRB * SLOT
                                : (L == L1 - 1 ? yf_out : yf_base) + lid * YR * SLOT;  // in my consumer's memory
  // my progress word: read by the z producer (same part, local) and the y
  // producer -- at lap L0 of a split cube the previous part, so a copy goes there
  int32_t *const prog_x = (SYS && L == L0 && L0 > 0) ? prog_in + lid * LAP_PROG_STRIDE : nullptr;
  const uint8_t *yf_prev = !yin ? yf_mine
                           : yb_pr >= 0 ? rd.yb + (int64_t)yb_pr * rd.YRB * SLOT
                                        : yf_base + (lid - GZ) * YR * SLOT;
  uint8_t *zf_mine = zb_me >= 0 ? rd.zb + (int64_t)zb_me * rd.ZRB * ZREC : zf_base + lid * ZR * ZREC;
  const uint8_t *zf_prev = !zin ? zf_mine
                           : zb_pr >= 0 ? rd.zb + (int64_t)zb_pr * rd.ZRB * ZREC
                                        : zf_base + (lid - 1) * ZR * ZREC;
  const uint32_t ep19 = epoch & 0x7FFFFu;
  bool timed_out = false;
  auto fail = [&]() {  // every wait of this workgroup gives up from now on
    if (!timed_out && lane == 0) {
      __hip_atomic_store(err, epoch, __ATOMIC_RELEASE, SCOPE);
      *(volatile __attribute__((address_space(3))) int32_t *)(__attribute__((address_space(3))) void *)w_abort = 1;
    }
    timed_out = true;
  };
  // wait until an LDS progress word reaches `need` (bounded: a hand-off timeout
  // upstream aborts the workgroup, and no wait outlives ~4 x spin_limit polls)
  uint32_t n_wait = 0;
  auto wait_word = [&](const int32_t *word, int32_t &seen, int32_t need) {
    if (need <= seen) return;
    seen = lds_word(word);
    if (need <= seen) return;
    ++n_wait;
    for (uint32_t spin = 1;; ++spin) {
      seen = lds_word(word);
      if (need <= seen) return;
      if ((spin & 255) == 0 && (timed_out || lds_word(w_abort) != 0 || spin >= 4 * spin_limit)) {
        fail();
        seen = 1 << 24;
        return;
      }
      if (spin > 64) __builtin_amdgcn_s_sleep(1);
    }
  };

  // ---- A code pairs, zeroed words
  const int32_t na = lap_na(la, M, NW, LIT);
  for (int j = tid; j < na; j += 64 * (NW + 1)) {
    const int x0 = j - OFF, x1 = j - OFF - 1;
    const uint32_t c0 = (x0 >= 0 && x0 < la) ? SYM0 << tsa_sym(seqs, o0 + x0, pa.packed) : 0u;
    const uint32_t c1 = (x1 >= 0 && x1 < la) ? SYM0 << tsa_sym(seqs, o0 + x1, pa.packed) : 0u;
    sA2[j] = c0 | (c1 << 16);
  }
  if (tid < 16) wd[tid] = 0;
  // face records, so a lap-0 wave 0 / tile-0 wave reads its y / z inputs the
  // same way as any other (no branch in the step): y {Iy, Ixy | Iyz, best} low
  // halves (wave 0's perm format), z {Iz, -, Ixz, - | Iyz, -, M, -}
  for (int j = tid; j < M * 64; j += 64 * (NW + 1))
    ((uint4 *)yface)[j] = make_uint4((pa.f_single & 0xFFFFu) | (pa.f_pair & 0xFFFF0000u), 0u,
                                     pa.f_pair & 0xFFFFu, 0u);
  if (tid < 2 * NW)
    ((uint4 *)zface)[tid] = (tid & 1) ? make_uint4(pa.f_pair, 0u, 0u, 0u)
                                                      : make_uint4(pa.f_single, 0u, pa.f_pair, 0u);
  if constexpr (U4K && !FACES) {  // the same records in every ring slot (no loader writes)
    if (!yin)
      for (int j = tid; j < K0 * M * 64; j += 64 * (NW + 1))
        ((uint4 *)xr0)[j] = make_uint4((pa.f_single & 0xFFFFu) | (pa.f_pair & 0xFFFF0000u), 0u,
                                       pa.f_pair & 0xFFFFu, 0u);
    if (!zin)
      for (int j = tid; j < LAP_ZL * 2 * NW; j += 64 * (NW + 1))
        ((uint4 *)zring)[j] = (j & 1) ? make_uint4(pa.f_pair, 0u, 0u, 0u)
                                      : make_uint4(pa.f_single, 0u, pa.f_pair, 0u);
  }
  pw[tid] = 0;  // blockDim = 64 (NW + 1): one word per thread
  // the wave-to-wave rings: step 0 reads slot K-1 before any write (its cells
  // are not real, but the checked kernel's monitor must not see stale LDS)
  for (int j = tid; j < (NW - 1) * K * SLOT / 16; j += 64 * (NW + 1))
    ((uint4 *)xr)[j] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();

  if (w == NW) {
    // =================== loader wave ===================
    // Records are fetched LPD steps ahead into registers with 8-byte sc1 loads
    // (one {payload, tag} granule each: relaxed agent-scope atomics, so the
    // compiler counts vmcnt itself), their tags checked in registers, then
    // written to LDS (xr0 / zring) and published.
    uint32_t stalls = 0;
    typedef unsigned long long u64;
    // TSA_LAP_L16: a record's two granules by one 16-byte load (volatile:
    // sc0 sc1, L1 bypassed, L2-served; each naturally aligned 8-byte {payload,
    // tag} granule of it is untorn, so the per-granule tag check stands)
    typedef u64 u64x2 __attribute__((ext_vector_type(2)));
    auto gl16 = [&](const uint8_t *p) -> u64x2 {
      return *(volatile const __attribute__((address_space(1))) u64x2 *)(
          const __attribute__((address_space(1))) void *)p;
    };
    // TSA_LAP_L16 = 2: the same 16 bytes by a raw buffer load with sc1 (a
    // compiler-counted load, no vmcnt(0) behind it), off a per-lap resource
    // of the ring's base
    // (TSA_LAP_NOFACE_FETCH: a lap-0 / tile-0 loader, whose y / z fetches feed
    // nothing, gets a zero-length resource -- its loads stay in the window, so
    // the compiler's vmcnt counting stays static, but return 0 without a
    // memory access)
    const int32_t ny = (TSA_LAP_NOFACE_FETCH && !yin) ? 0 : 0x7FFFFFFF;
    const int32_t nz = (TSA_LAP_NOFACE_FETCH && !zin) ? 0 : 0x7FFFFFFF;
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)yf_prev, (short)0, ny, 0x00020000);
    const __amdgpu_buffer_rsrc_t rzr = __builtin_amdgcn_make_buffer_rsrc((void *)zf_prev, (short)0, nz, 0x00020000);
    auto bl16 = [&](__amdgpu_buffer_rsrc_t r, uint32_t off) -> u64x2 {
      if constexpr (SYS)  // 17: sc0 sc1 (system scope, as the 8-byte loads of the split)
        return __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17));
      else  // 16: sc1
        return __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
    };
    auto gl8 = [&](const uint8_t *p) -> u64 {
      return __hip_atomic_load((const u64 *)p, __ATOMIC_RELAXED, SCOPE);
    };
    const int64_t cons_y = yout ? lid + GZ : lid, cons_z = zout ? lid + 1 : lid;
    struct Fetch {
      u64 y[2 * M], z[2];
      int32_t py, pz;  // my consumers' progress words (lane 0)
    };
    auto fetch_y = [&](int32_t s, Fetch &f) {  // y record s + YOFF
      const int32_t r = s + YOFF;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const uint8_t *g = yf_prev + ((int64_t)(r & (YRp - 1)) * M + i) * PAIR + lane * REC_BYTES;
        if constexpr (L16K == 2) {
          const u64x2 v = bl16(ry, (uint32_t)(((int64_t)(r & (YRp - 1)) * M + i) * PAIR + lane * REC_BYTES));
          f.y[2 * i] = v[0];
          f.y[2 * i + 1] = v[1];
        } else if constexpr (L16K == 1) {
          const u64x2 v = gl16(g);
          f.y[2 * i] = v[0];
          f.y[2 * i + 1] = v[1];
        } else {
          f.y[2 * i] = gl8(g);
          f.y[2 * i + 1] = gl8(g + 8);
        }
      }
    };
    auto fetch_z = [&](int32_t rz, Fetch &f) {  // z record rz (lanes 0 .. 2NW-1)
      const uint8_t *g = zf_prev + (int64_t)(rz & (ZRp - 1)) * ZREC + (lane & (2 * NW - 1)) * 16;
      if constexpr (L16K == 2) {
        const u64x2 v = bl16(rzr, (uint32_t)((int64_t)(rz & (ZRp - 1)) * ZREC + (lane & (2 * NW - 1)) * 16));
        f.z[0] = v[0];
        f.z[1] = v[1];
      } else if constexpr (L16K == 1) {
        const u64x2 v = gl16(g);
        f.z[0] = v[0];
        f.z[1] = v[1];
      } else {
        f.z[0] = gl8(g);
        f.z[1] = gl8(g + 8);
      }
    };
    auto fetch = [&](int32_t s, Fetch &f, bool progw = true) {
      fetch_y(s, f);
      fetch_z(s + ZT + ZA, f);
      if (progw) {
        f.py = __hip_atomic_load(prog + cons_y * LAP_PROG_STRIDE, __ATOMIC_RELAXED, SCOPE);
        f.pz = __hip_atomic_load(prog + cons_z * LAP_PROG_STRIDE, __ATOMIC_RELAXED, SCOPE);
      }
    };
    // LIT: the y = 0 (lap 0) and z = 0 (tile 0) faces, written into the rings
    // wave 0 and position 0 read: zero cells pushing with the receivers'
    // symbols (tools/litlap_emu.py zero_push), so they vary with the step
    uint32_t lones = 0x00010001u, lb1 = 0, lc1 = 0, lby2 = 0, lcn[M], lfyz[M];
    LitArgs cv = lit;
    if constexpr (LIT) {
      asm volatile("" : "+v"(lones), "+v"(cv.dmS), "+v"(cv.d1S), "+v"(cv.d0S), "+v"(cv.neS), "+v"(cv.mm3S),
                   "+v"(cv.fP[0]), "+v"(cv.fP[1]));
      auto code = [&](int64_t base, int32_t i, int32_t len) -> uint32_t {
        return (i >= 0 && i < len) ? SYM0 << tsa_sym(seqs, base + i, pa.packed) : 0u;
      };
      lb1 = code(o1, 0, lb) * 0x00010001u;  // b_1 (the y = 0 face is lap 0's)
      lc1 = code(o2, 0, lc) * 0x00010001u;  // c_1
      const int32_t yz = L * RW + 2 * ((lane & (2 * NW - 1)) >> 1);
      lby2 = code(o1, yz, lb) | (code(o1, yz + 1, lb) << 16);  // b_y of the two rows of wave lane / 2
#pragma unroll
      for (int i = 0; i < M; ++i) {
        lcn[i] = code(o2, q * ZT + M * lane + i + 1, lc) * 0x00010001u;  // c_{z+1}
        lfyz[i] = lit_face_pair(cv, lb1, lcn[i], lones);
      }
    }
    // wave 0's record of step s: row 0's pushes into row 1 at x' = s - k, in
    // the tagged record format (low halves: Iy | Ixy << 16, Iyz | M << 16)
    auto yface_lit = [&](int32_t s, int i) -> uint4 {
      const uint32_t an = sA2[s - (M * lane + i) + OFF] & 0xFFFFu;  // a_{x'+1}
      const uint32_t fxy = lit_face_pair(cv, an, lb1, lones), fm = lit_face_m<SOP>(cv, an, lb1, lcn[i], lones);
      return make_uint4((cv.fS[1] & 0xFFFFu) | (fxy << 16), 0u, (lfyz[i] & 0xFFFFu) | (fm << 16), 0u);
    };
    // z record rz (lanes 0 .. 2NW-1: wave lane / 2, word pair lane & 1): the
    // z = 0 cells of that wave's two rows at x' = rz - ZT + 1 - 2w - h
    auto zface_lit = [&](int32_t rz) -> uint4 {
      const int32_t wz = (lane & (2 * NW - 1)) >> 1;
      const uint32_t a2 = sA2[rz - ZT + 1 - 2 * wz + OFF];  // a_{x'+1}: row 2wz (lo), 2wz + 1 (hi)
      if (lane & 1)
        return make_uint4(lit_face_pair(cv, lby2, lc1, lones), 0u, lit_face_m<SOP>(cv, a2, lby2, lc1, lones), 0u);
      return make_uint4(cv.fS[2], 0u, lit_face_pair(cv, a2, lc1, lones), 0u);
    };
    // VS: the same faces as V-space values -- a face cell at coordinate sum
    // q_f sends lam q_f to a pair target and to M, lam q_f - lam to a single
    // target. Lap 0's record of step s (wave 0's low halves, rows 0 -> 1):
    // Iy = lam (s + zoff + 1), Ixy = Iyz = best = lam (s + zoff + 2), the same
    // on every lane (x + z is the step); tile 0's z record for step t = rz - ZT
    // (position 0 of every wave): Iz = Iyz = M = lam (t + L RW + 2), Ixz one lam more
    const int32_t zoff = q * ZT;
    auto yface_vs = [&](int32_t s) -> uint4 {
      const uint32_t f1 = lam_bits(pa.lam, s + zoff + 1) & 0xFFFFu, f2 = lam_bits(pa.lam, s + zoff + 2) & 0xFFFFu;
      return make_uint4(f1 | (f2 << 16), 0u, f2 | (f2 << 16), 0u);
    };
    auto zface_vs = [&](int32_t rz) -> uint4 {
      const int32_t t = rz - ZT;
      const uint32_t g1 = lam_bits(pa.lam, t + L * RW + 2);
      if (lane & 1) return make_uint4(g1, 0u, g1, 0u);                  // {Iyz, -, M, -}
      return make_uint4(g1, 0u, lam_bits(pa.lam, t + L * RW + 3), 0u);  // {Iz, -, Ixz, -}
    };
    auto tag_ok = [](u64 g, uint32_t tg) { return (uint32_t)(g >> 32) == tg; };
    auto y_ok = [&](int32_t s, const Fetch &f) {
      const uint32_t tg = lap_tag(epoch, s + YOFF);
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 2 * M; ++i) ok = ok && tag_ok(f.y[i], tg);
      return __all(ok) != 0;
    };
    auto z_ok = [&](int32_t rz, const Fetch &f) {
      const uint32_t tg = lap_tag(epoch, rz);
      return __all(lane >= 2 * NW || (tag_ok(f.z[0], tg) && tag_ok(f.z[1], tg))) != 0;
    };
    // slow path: fetch again until the tags match (the producer has not stored yet)
    auto settle_y = [&](int32_t s, Fetch &f) {
      ++stalls;
      for (uint32_t spin = 0;; ++spin) {
        if (spin >= spin_limit || timed_out || ((spin & 63) == 63 && lds_word(w_abort) != 0)) {
          fail();
          return;
        }
        fetch_y(s, f);
        if (y_ok(s, f)) return;
        __builtin_amdgcn_s_sleep(1);
      }
    };
    auto settle_z = [&](int32_t rz, Fetch &f) {
      ++stalls;
      for (uint32_t spin = 0;; ++spin) {
        if (spin >= spin_limit || timed_out || ((spin & 63) == 63 && lds_word(w_abort) != 0)) {
          fail();
          return;
        }
        fetch_z(rz, f);
        if (z_ok(rz, f)) return;
        __builtin_amdgcn_s_sleep(1);
      }
    };
    // records beyond the producer's last step are never checked; they only
    // feed cells past the cube, stored as zeros (the checked kernel's monitor
    // sees those cells too, and must not see stale ring contents)
    auto put_z = [&](int32_t rz, const Fetch &f) {
      const bool real = rz < T_left;
      if (U4K && !FACES && !zin) return;  // zring holds the prefilled z = 0 face
      if (lane < 2 * NW) {
        uint4 v = real ? make_uint4((uint32_t)f.z[0], (uint32_t)(f.z[0] >> 32), (uint32_t)f.z[1],
                                    (uint32_t)(f.z[1] >> 32))
                       : make_uint4(0u, 0u, 0u, 0u);
        if constexpr (LIT) {
          if (!zin) v = zface_lit(rz);
        }
        if constexpr (VS) {
          if (!zin) v = zface_vs(rz);
        }
        lds_write16(zring + (rz & (LAP_ZL - 1)) * ZREC + lane * 16, v);
      }
    };
    int32_t seen_w0 = 0, seen_wl = 0;
    // prologue: z records ZT-2 .. ZT+ZA-1 (position 0's step-0 inputs and the
    // z reads of steps the loader's progress does not cover), checked now
    if (zin || FACES) {  // (LIT / VS tile 0: the z = 0 faces of those records)
      for (int rz = ZT - 2; rz < ZT + ZA; ++rz) {
        Fetch f;
        f.z[0] = f.z[1] = 0;
        if (zin) {
          fetch_z(rz, f);
          if (rz < T_left && !z_ok(rz, f)) settle_z(rz, f);
        }
        put_z(rz, f);
      }
    }
    __syncthreads();  // (matches the compute waves' prologue barrier)
    Fetch fq[LPD];
    // the loop period LU (a multiple of LPD): the progress words ride with the
    // fetch processed at phase 0 of a period, issued LPD steps earlier
    constexpr bool PTHIN = PROGPK > 1;
    constexpr int LU = (PROGPK > LPD && PROGPK % LPD == 0) ? PROGPK : LPD;
#pragma unroll
    for (int j = 0; j < LPD; ++j) fetch(j, fq[j], !PTHIN || j == 0);
    // one step: check the fetch of step s (registers fq[j]), store it to LDS,
    // publish, refill fq[j] with step s + LPD
    auto lstep = [&](auto ph, int32_t s) {
      constexpr int PHL = decltype(ph)::value;  // phase in the loop period
      constexpr int j = PHL % LPD;
      Fetch &f = fq[j];
      if (yin && s + YOFF < T_above && !y_ok(s, f)) settle_y(s, f);
      const int32_t rz = s + ZT + ZA;
      if (zin && rz < T_left && !z_ok(rz, f)) settle_z(rz, f);
      constexpr bool PROGW = !PTHIN || PHL == 0;  // this fetch carries the progress words
      if (PROGW && lane == 0) {  // my consumers' progress, for the producing waves' back-pressure
        bpw[0] = f.py;
        bpw[1] = f.pz;
      }
      wait_word(pw, seen_w0, s - K0 + 1);                           // wave 0 is done with xr0 slot s % K0
      wait_word(pw + 64 * (NW - 1), seen_wl, s + ZA - LAP_ZL + 1);  // the last wave with zring's old record
      uint8_t *dst = xr0 + (s & (K0 - 1)) * SLOT + lane * REC_BYTES;
      const bool yreal = s + YOFF < T_above;
      const bool ywrite = !(U4K && !FACES) || yin;  // else xr0 holds the prefilled y = 0 face
      if (ywrite) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          uint4 v = yreal ? make_uint4((uint32_t)f.y[2 * i], (uint32_t)(f.y[2 * i] >> 32),
                                       (uint32_t)f.y[2 * i + 1], (uint32_t)(f.y[2 * i + 1] >> 32))
                          : make_uint4(0u, 0u, 0u, 0u);
          if constexpr (LIT) {
            if (!yin) v = yface_lit(s, i);
          }
          if constexpr (VS) {
            if (!yin) v = yface_vs(s);
          }
          lds_write16(dst + i * PAIR, v);
        }
      }
      put_z(rz, f);
      lds_publish(pw + 64 * NW, s + 1, lane);  // wave 0 may run step s
      fetch(s + LPD, f, !PTHIN || (PHL + LPD) % LU == 0);
    };
    int32_t s = 0;
#pragma unroll 1
    for (; s + LU <= T; s += LU)
      static_for<0, LU>([&](auto ph) { LAP_INLINE(lstep(ph, s + decltype(ph)::value)); });
    static_for<0, LU>([&](auto ph) {
      if (s + decltype(ph)::value < T) LAP_INLINE(lstep(ph, s + decltype(ph)::value));
    });
    if (lane == 0) w_stall[0] = (int32_t)stalls;
  } else {
    // =================== compute waves ===================
    // a[i] of this lane at step t = sA2[t - 2w - (M lane + i) + OFF]
    const uint32_t a_lane = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)sA2 +
                            4u * (uint32_t)(OFF - 2 * w - M * lane - (M - 1));
    const int32_t y0 = L * RW + 2 * w;  // rows y0 (lo) and y0 + 1 (hi), 0-based
    const uint32_t bw = (y0 < lb ? SYM0 << tsa_sym(seqs, o1 + y0, pa.packed) : 0u) |
                        ((y0 + 1 < lb ? SYM0 << tsa_sym(seqs, o1 + y0 + 1, pa.packed) : 0u) << 16);
    uint32_t bv[M], c[M], SBC[M], K_[M], DMC[M], DMB[M];
    uint32_t oIx[M], shIz[M], svIxy[M], svIyz[M], shIxz[2][M], svM[2][M];
    uint32_t pIy[M], pIxy[M], pIyz[M], pBest[M];  // this wave's record of the previous step
    {
      uint32_t one1 = 0x00010001u, sbcv = pa.h_sbc, kdv = pa.h_kd, k0v = pa.h_k0;
      uint32_t dmb = 0u;
      if constexpr (VS) {
        // the [a=b] terms multiply b's one-hot code itself (a & b, no min):
        // DMB = dm / code(b) and, RTL s3, K = (d0 + [b=c] d1) / code(b)
        // (cell_messages_vs); both rows of the wave, one per half
        dmb = dm_over_code(pa.dmf, bw);
        if constexpr (!SOP) {
          k0v = dm_over_code(pa.d0f, bw);
          const uint32_t kb1 = dm_over_code(pa.d0f + pa.d1f, bw);
          kdv = (((kb1 & 0xFFFFu) - (k0v & 0xFFFFu)) & 0xFFFFu) | ((((kb1 >> 16) - (k0v >> 16)) & 0xFFFFu) << 16);
        }
      }
      asm volatile("" : "+v"(one1), "+v"(sbcv), "+v"(kdv), "+v"(k0v));
      const int64_t oc = o2 + (int64_t)q * ZT;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int k = M * lane + i;
        c[i] = (k < zt_q ? SYM0 << tsa_sym(seqs, oc + k, pa.packed) : 0u) * 0x00010001u;
        DMC[i] = dm_over_code(pa.dmf, c[i]);
        bv[i] = bw;
        const uint32_t e01 = pk_eq1(bw, c[i], one1);
        SBC[i] = pk_mad(e01, sbcv, 0u);
        K_[i] = pk_mad(e01, kdv, k0v);
        DMB[i] = dmb;
        oIx[i] = shIz[i] = pa.f_single;
        shIxz[0][i] = shIxz[1][i] = svIxy[i] = svIyz[i] = pa.f_pair;
        svM[0][i] = svM[1][i] = 0;
        pIy[i] = pIxy[i] = pIyz[i] = pBest[i] = 0;
      }
    }
    // LIT: the successors' symbols b_{y+1} (per half) and c_{z+1} (per position),
    // the per-position pair score of (y+1, z+1) less GE and the [b=c] part of
    // s3; the launch passes f_single = f_pair = 0, so the x' = 0 face column's
    // forced inputs and the initial states are zeros
    uint32_t bn = 0, cnl[M], UYZ[M], K1[M], lones = 0x00010001u;
    LitArgs cv = lit;
    if constexpr (LIT) {
      asm volatile("" : "+v"(lones), "+v"(cv.dmS), "+v"(cv.mmE), "+v"(cv.neS));
      bn = (y0 + 1 < lb ? SYM0 << tsa_sym(seqs, o1 + y0 + 1, pa.packed) : 0u) |
           ((y0 + 2 < lb ? SYM0 << tsa_sym(seqs, o1 + y0 + 2, pa.packed) : 0u) << 16);
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int32_t z1 = q * ZT + M * lane + i + 1;
        cnl[i] = (z1 < lc ? SYM0 << tsa_sym(seqs, o2 + z1, pa.packed) : 0u) * 0x00010001u;
        const uint32_t ebc = pk_eq1(bn, cnl[i], lones);
        UYZ[i] = pk_mad(ebc, cv.dmS, cv.mmE);
        K1[i] = SOP ? pk_mad(ebc, cv.dmS, lit.mm3S) : pk_mad(ebc, lit.d1S, lit.d0S);
      }
    }
    // CHK: halves of real cells (row y < lb, position z < LC of the tile); the
    // rest is masked to 0, a value the monitor's range contains anyway (faces)
    uint32_t vmask[M], vmax[M], vmin[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const uint32_t rowm = (y0 < lb ? 0x0000FFFFu : 0u) | (y0 + 1 < lb ? 0xFFFF0000u : 0u);
      vmask[i] = M * lane + i < zt_q ? rowm : 0u;
      vmax[i] = vmin[i] = 0u;
    }
    uint32_t Q = F16 ? 0x08000800u : 0x00010001u, fsv = pa.f_single, fpv = pa.f_pair;
    uint32_t mlo = 0x0000FFFFu, mhi = 0xFFFF0000u;
    asm volatile("" : "+v"(Q), "+v"(fsv), "+v"(fpv), "+v"(mlo), "+v"(mhi));
    const PencilArgs pv = F16 ? pa : pin_score_consts(pa);
    const uint32_t sel0 = lane == 0 ? 0x03020100u : 0x07060504u;  // lane 0: whole word from the face
    // VS: the x = 0 face at the x = 1 cells of step t -- the low half's
    // position t - 2w and the high half's one behind share x + y + z =
    // t + L RW + zoff + 3, so one value for both: lam (t + L RW + zoff + 1)
    // for Ix, Ixy, Ixz (one lam less for M: the previous step's)
    uint32_t hx_cur = 0u, hx_prev = 0u;
    if constexpr (VS) {
      hx_cur = lam_bits(pa.lam, L * RW + q * ZT + 1);
      hx_prev = lam_bits(pa.lam, L * RW + q * ZT);
    }
    __syncthreads();  // the loader's prologue z records are in LDS
    if (zin || FACES) {  // position 0 before step 0 (tools/lap_emu.py: the same initial shifts)
      const uint8_t *r1 = zring + ((ZT - 1) & (LAP_ZL - 1)) * ZREC + w * LAP_ZREC_WAVE;
      const uint8_t *r2 = zring + ((ZT - 2) & (LAP_ZL - 1)) * ZREC + w * LAP_ZREC_WAVE;
      const uint4 a0 = lds_read16(r1), a1 = lds_read16(r1 + 16);
      const uint4 b0 = lds_read16(r2), b1 = lds_read16(r2 + 16);
      if (lane == 0) {
        shIz[0] = a0.x;
        svIyz[0] = a1.x;
        shIxz[1][0] = a0.z;
        svM[1][0] = a1.z;
        shIxz[0][0] = b0.z;
        svM[0][0] = b1.z;
      }
    }
    unsigned long long clk0 = 0;
    if (trace != nullptr) {
      stamp(1, now());
      clk0 = __builtin_amdgcn_s_memtime();  // shader clock: the loop's cycles (slot 6)
    }
    // wave 0's y input: xr0 slot t % K0, or the face record (stride 0)
    // (LIT / VS: always the loader's, which writes the step-varying faces)
    // (U4K: always xr0, which then holds the prefilled face)
    const bool yring = U4K || yin || FACES, zring_in = U4K || zin || FACES;
    const uint8_t *const ysrc = (yring ? xr0 : yface) + lane * REC_BYTES;
    const int32_t ystride = yring ? SLOT : 0;
    // position 0's z input: zring slot (t + ZT) % ZL = t % ZL, or the face record
    static_assert(ZT % LAP_ZL == 0, "z slot of step t: t % LAP_ZL");
    const uint8_t *const zsrc = (zring_in ? zring : zface) + w * LAP_ZREC_WAVE;
    const int32_t zstride = zring_in ? ZREC : 0;
    uint32_t a_nx[M];
    load_a<M>(a_lane, a_nx);
    uint32_t a_pair = a_lane;  // TSA_LAP_LEAN: a_lane's entry of the step pair's first step
    // U4K: the bases of the current group of four steps (t0 = t & ~3)
    uint32_t a_grp = a_lane;
    const uint8_t *y_grp = ysrc, *z_grp = zsrc;
    uint8_t *zst_grp = nullptr, *yst_grp = nullptr;
    // VBK: three VGPR bases (see the knob) -- v_rw: this lane's
    // record in the ring read (slot 0; wave 0: the ring it writes), the ring
    // written K slots above it; v_pwb: this lane's copy of the progress word
    // of wave w - 1 (wave 0: its own), the others at constant offsets above
    // it (every lane holds a copy, so a per-lane address reads the same
    // value); vlane: the SGPR-base stores' offset (the z record, stored by lane
    // 63, from a base 63 records lower)
    lds_u8 *v_rw = to_lds(xr + (w > 0 ? (w - 1) * K * SLOT : 0) + lane * REC_BYTES);
    lds_u8 *v_pwb = to_lds((uint8_t *)(pw + 64 * (w > 0 ? w - 1 : 0) + lane));
    // byte offsets from v_pwb: the input word (wave 0: the loader's), the own, the successor's
    auto pw_in = [](auto role) { return decltype(role)::value == 0 ? 4 * 64 * NW : 0; };
    auto pw_own = [](auto role) { return decltype(role)::value == 0 ? 0 : 4 * 64; };
    constexpr int WR_OFF = K * SLOT;  // v_rw + WR_OFF: the ring written (waves 1 ..)
    const lds_u8 *vy_grp = to_lds((uint8_t *)ysrc), *vz_grp = to_lds((uint8_t *)zsrc);
    const uint8_t *zst_s = zf_mine, *yst_s = yf_mine;  // SGPR bases of the group's ring records
    uint32_t vlane = (uint32_t)lane * REC_BYTES;
    if constexpr (VBK) asm volatile("" : "+v"(v_rw), "+v"(v_pwb), "+v"(vlane));
    auto set_group = [&](int32_t t0) {
      a_grp = a_lane + 4u * (uint32_t)t0;
      y_grp = ysrc + (t0 & (K0 - 1)) * SLOT;
      z_grp = zsrc + (t0 & (LAP_ZL - 1)) * ZREC;
      zst_grp = zf_mine + (int64_t)(t0 & (ZRm - 1)) * ZREC + w * LAP_ZREC_WAVE;
      yst_grp = yf_mine + (int64_t)(t0 & (YRm - 1)) * SLOT + lane * REC_BYTES;
      if constexpr (VBK) {
        vy_grp = to_lds((uint8_t *)y_grp);
        vz_grp = to_lds((uint8_t *)z_grp);
        asm volatile("" : "+v"(vy_grp), "+v"(vz_grp));
        zst_s = (const uint8_t *)sgpr64((uint64_t)(uintptr_t)(zf_mine + (int64_t)(t0 & (ZRm - 1)) * ZREC +
                                                              w * LAP_ZREC_WAVE - 63 * REC_BYTES));
        yst_s = (const uint8_t *)sgpr64((uint64_t)(uintptr_t)(yf_mine + (int64_t)(t0 & (YRm - 1)) * SLOT));
      }
    };
    // producer side: my consumers' progress (y: the lap below, via the last
    // wave; z: the tile to the right, every wave), LDS-DMA'd by the loader
    int32_t seen_in = 0, seen_out = 0, seen_y = 0, seen_z = 0;
    uint32_t n_bp = 0;
#if defined(TSA_DIAG)  // shader cycles: reads + pre-cell, check, post + stores, step gap
    uint64_t prof[4] = {0, 0, 0, 0}, prof_last = 0;
    int32_t lag_y = 0, lag_z = 0;  // t - the consumer's progress, at the ring stores
#endif
    constexpr int LM = M == 1 ? 0 : M == 2 ? 1 : M == 4 ? 2 : 3;  // log2 M
    int32_t klo = -2 * w, ihi = 0;  // x = 1 position of the low half at the current step
    uint64_t lm_hi = 0;             // the high half's lane mask (previous step's low)
    auto prog_decode = [&](int32_t v) -> int32_t {
      return ((uint32_t)v >> 13) == ep19 ? (int32_t)(v & 0x1FFF) : 0;
    };
    auto wait_consumer = [&](int64_t cons, int32_t &seen, int32_t *word, int32_t need) {
      if (need <= seen) return;
      seen = max(seen, prog_decode(lds_word(word)));
      if (need <= seen) return;
      ++n_bp;
      for (uint32_t spin = 0;; ++spin) {
        const int32_t v = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(prog + cons * LAP_PROG_STRIDE, __ATOMIC_RELAXED, SCOPE));
        seen = max(seen, prog_decode(v));
        if (need <= seen) return;
        if (spin >= spin_limit || timed_out || ((spin & 63) == 63 && lds_word(w_abort) != 0)) {
          fail();
          seen = 1 << 24;
          return;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    };
    const int64_t cons_y = yout ? lid + GZ : -1, cons_z = zout ? lid + 1 : -1;
    // Room in my z ring for record tt: the consumer's loader checks record
    // s + ZT + ZA at its step s, so a published progress p covers records up
    // to p - 1 + ZT + ZA -- and its prologue reads ZT - 2 .. ZT + ZA - 1
    // before it publishes anything, so overwriting one of those (or later)
    // needs p >= 1 even where that formula gives <= 0: a consumer that starts
    // late (its physical workgroup still on a lap of the previous round) would
    // otherwise find its prologue records overwritten and wait forever
    auto z_need = [&](int32_t tt) -> int32_t {
      const int32_t r = tt - ZRm;  // the record slot tt & (ZRm - 1) holds before
      return r >= ZT - 2 ? max(1, r - ZT - ZA + 1) : 0;
    };

    // ROLE: 0 = wave 0, 1 = middle waves, 2 = the last wave (NW >= 2)
    // QS: t & 3 in a four-step group (addresses at constant offsets from the
    // group's bases), -1: addresses from t
    auto step = [&](auto ph, auto role, int32_t t, auto fin_step, auto qs) {
      constexpr int PH = decltype(ph)::value;
      constexpr int ROLE = decltype(role)::value;
      constexpr bool FIN = decltype(fin_step)::value;
      constexpr int QS = decltype(qs)::value;
      uint32_t a[M];
#pragma unroll
      for (int i = 0; i < M; ++i) a[i] = a_nx[i];
      if constexpr (QS >= 0) load_a_off<M>(a_grp, QS + 1, a_nx);
      else if constexpr (TSA_LAP_LEAN) load_a_off<M>(a_pair, PH + 1, a_nx);  // entry t + 1 of a_lane's table
      else load_a<M>(a_lane + 4u * (uint32_t)(t + 1), a_nx);
      // ---- input reads, issued first: the producer's progress word (unless the
      // cached value covers step t), then its record. LDS executes a wave's DS
      // instructions in order, so a word read that covers t proves the record
      // read behind it current; the check waits until the pre-cell is done.
#if defined(TSA_DIAG)
      const uint64_t pt0 = __builtin_amdgcn_s_memtime();
#endif
      const int32_t need = ROLE == 0 ? t + 1 : t;
      const int32_t *const pword = ROLE == 0 ? pw + 64 * NW : pw + 64 * (w - 1);
      const bool waits = ROLE != 0 || yin || zin || FACES;
      const bool poll = TSA_LAP_LEAN ? waits : (waits && seen_in < need);
      int32_t fl_v = 0;
      constexpr bool VB = QS >= 0 && VBK;  // this step's accesses off the VGPR bases
      if (poll) {
        if constexpr (VB)
          fl_v = *(volatile const __attribute__((address_space(3))) int32_t *)(v_pwb + pw_in(role));
        else
          fl_v = *(volatile const __attribute__((address_space(3))) int32_t *)(
              const __attribute__((address_space(3))) void *)pword;
      }
      asm volatile("" ::: "memory");
      const uint8_t *src = QS >= 0 ? (ROLE == 0 ? y_grp + QS * SLOT
                                                : xr + ((w - 1) * K + ((QS + K - 1) & (K - 1))) * SLOT + lane * REC_BYTES)
                         : ROLE == 0 ? ysrc + (t & (K0 - 1)) * ystride
                                     : xr + ((w - 1) * K + ((t - 1) & (K - 1))) * SLOT + lane * REC_BYTES;
      const lds_u8 *srcl = VB ? (ROLE == 0 ? vy_grp + (VB ? QS : 0) * SLOT
                                           : v_rw + (((VB ? QS : 0) + K - 1) & (K - 1)) * SLOT)
                              : to_lds((uint8_t *)src);
      uint4 rv[M];
      auto read_rec = [&]() {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          if constexpr (ROLE == 0 && TSA_LAP_Y2) {  // {payload, tag, payload, tag}: the payloads only
            const __attribute__((address_space(3))) uint32_t *p =
                (const __attribute__((address_space(3))) uint32_t *)(srcl + i * PAIR);
            rv[i] = make_uint4(p[0], 0u, p[2], 0u);
          } else {
            rv[i] = lds_read16_at(srcl, i * PAIR);
          }
        }
      };
      read_rec();
      // the successor's progress, read now and consulted before the record store
      // (TSA_LAP_GCHK groups, K = 4: on even steps only, covering the next step too)
      constexpr bool SUCC_HERE = !(QS >= 0 && TSA_LAP_GCHK && K == 4) || (QS & 1) == 0;
      int32_t succ_v = 0;
      if constexpr (ROLE != 2 && SUCC_HERE && VB)
        succ_v = *(volatile const __attribute__((address_space(3))) int32_t *)(v_pwb + pw_own(role) + 4 * 64);
      else if constexpr (ROLE != 2 && SUCC_HERE)
        succ_v = *(volatile const __attribute__((address_space(3))) int32_t *)(
            const __attribute__((address_space(3))) void *)(pw + 64 * (w + 1));
      // position 0's z-1 neighbour for the next step: the z = 0 face, or the
      // left tile's record t + ZT (checked by the loader: see ZA)
      // (four 4-byte reads, merged into two ds_read2_b32: reading the tags too
      // hands the compiler dead registers it reuses, forcing lgkmcnt(0) waits)
      const uint8_t *zr = QS >= 0 ? z_grp + QS * ZREC : zsrc + ((t + ZT) & (LAP_ZL - 1)) * zstride;
      const lds_u8 *zrl = VB ? vz_grp + (VB ? QS : 0) * ZREC : to_lds((uint8_t *)zr);
      auto lds32 = [](const lds_u8 *p) { return *(const __attribute__((address_space(3))) uint32_t *)p; };
      const uint32_t fIz = lds32(zrl), fIxz = lds32(zrl + 8), fIyz = lds32(zrl + 16), fM = lds32(zrl + 24);
      uint32_t inIx[M], inIz[M], inIxy[M], inIyz[M], inIxz[M], inM[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        inIx[i] = oIx[i];
        inIz[i] = shIz[i];
        inIxy[i] = svIxy[i];
        inIyz[i] = svIyz[i];
        inIxz[i] = shIxz[PH][i];
        inM[i] = svM[PH][i];
      }
      // ---- x = 1: low half at position klo = t - 2w, high half one position
      // behind (= the low half's position of the previous step); their x - 1
      // inputs are the x = 0 face (src/PE_1cyc.v:164-178,196-218). Branch-free:
      // SALU lane masks (zero outside the tile) and one bfi mask per register.
      const uint64_t lm_lo = lane_bit(klo >> LM);
      const int32_t ilo = klo & (M - 1);
      uint32_t mx[M];  // LIT: the x' = 0 halves, whose Y is forced to 0 as it lands
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const uint64_t ml = (M == 1 || ilo == i) ? lm_lo : 0ull;
        const uint64_t mh = (M == 1 || ihi == i) ? lm_hi : 0ull;
        uint32_t m0, m1;
        asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m0) : "v"(mhi), "s"(mh));
        asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(m1) : "v"(m0), "v"(mlo), "s"(ml));
        inIx[i] = vbfi(m1, VS ? hx_cur : fsv, inIx[i]);
        inIxy[i] = vbfi(m1, VS ? hx_cur : fpv, inIxy[i]);
        inIxz[i] = vbfi(m1, VS ? hx_cur : fpv, inIxz[i]);
        inM[i] = vbfi(m1, VS ? hx_prev : 0u, inM[i]);
        if constexpr (LIT) {
          inIz[i] = vbfi(m1, 0u, inIz[i]);
          inIyz[i] = vbfi(m1, 0u, inIyz[i]);
          mx[i] = m1;
        }
      }
      if constexpr (VS) {
        hx_prev = hx_cur;
        hx_cur = U(H(hx_cur) + H(pa.v_lam));
      }
      lm_hi = lm_lo;
      ihi = ilo;
      ++klo;
      // ---- the cell, up to the row above
      LapPre<M> pre;
      LitPre<M> lpre;
      if constexpr (LIT)
        lit_pre<M, SOP>(lit, cv, lones, a, bn, cnl, UYZ, K1, inIx, inIz, inIxy, inIyz, inIxz, inM, lpre);
      else if constexpr (VS)
        lap_pre_vs<M, SOP>(a, bv, c, SBC, K_, DMC, DMB, pa, inIx, inIz, inIxy, inIyz, inIxz, inM, pre);
      else if constexpr (F16)
        lap_pre_f16<M, SOP>(a, bv, c, SBC, K_, DMC, Q, pa, inIx, inIz, inIxy, inIyz, inIxz, inM, pre);
      else
        lap_pre_i16<M, SOP>(a, bv, c, Q, pv, inIx, inIz, inIxy, inIyz, inIxz, inM, pre);
      // pin the pre-cell here: left alone the compiler sinks it below the
      // progress check, so the record read's latency would not be covered
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if constexpr (LIT) {
          asm volatile("" : "+v"(lpre.pIx[i]), "+v"(lpre.pIy[i]), "+v"(lpre.pIz[i]), "+v"(lpre.pIxy[i]),
                       "+v"(lpre.pIyz[i]), "+v"(lpre.pIxz[i]), "+v"(lpre.pM[i]));
          asm volatile("" : "+v"(lpre.uxy[i]), "+v"(lpre.vxz[i]), "+v"(lpre.s3[i]));
        } else {
          asm volatile("" : "+v"(pre.W[i]), "+v"(pre.N1[i]), "+v"(pre.N2[i]), "+v"(pre.N3[i]),
                       "+v"(pre.N4[i]), "+v"(pre.N5[i]), "+v"(pre.N6[i]));
        }
      }
#if defined(TSA_DIAG)
      const uint64_t pt1 = __builtin_amdgcn_s_memtime();
#endif
      // ---- the input record is current? (slow path: poll, then read it again)
      if (poll) {
        seen_in = max(seen_in, (int32_t)__builtin_amdgcn_readfirstlane(fl_v));
        if (seen_in < need) {
          wait_word(pword, seen_in, need);
          asm volatile("" ::: "memory");
          read_rec();
        }
      }
      // ---- the row above of both halves
      uint32_t Ry[M], Rxy[M], Ryz[M], Rb[M];
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if constexpr (ROLE != 0) {  // wave w-1's high halves
          Ry[i] = rows2(pIy[i], rv[i].x);
          Rxy[i] = rows2(pIxy[i], rv[i].y);
          Ryz[i] = rows2(pIyz[i], rv[i].z);
          Rb[i] = rows2(pBest[i], rv[i].w);
        } else {  // tagged record {Iy.hi | Ixy.hi << 16, tag, Iyz.hi | best.hi << 16, tag}
          Ry[i] = perm(pIy[i], rv[i].x, 0x05040100u);
          Rxy[i] = perm(pIxy[i], rv[i].x, 0x05040302u);
          Ryz[i] = perm(pIyz[i], rv[i].z, 0x05040100u);
          Rb[i] = perm(pBest[i], rv[i].z, 0x05040302u);
        }
      }
#if defined(TSA_DIAG)
      asm volatile("" :: "v"(Ry[0]));
      const uint64_t pt2 = __builtin_amdgcn_s_memtime();
#endif
      uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
      if constexpr (LIT) {  // (oBest: the push into M, the record's fourth word)
#pragma unroll
        for (int i = 0; i < M; ++i) Ry[i] = vbfi(mx[i], 0u, Ry[i]);
        lit_post<M>(lit, Ry, UYZ, lpre, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
      } else if constexpr (VS) {
        lap_post_vs<M>(pa, Ry, pre, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
      } else if constexpr (F16) {
        lap_post_f16<M>(pa, Ry, pre, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
      } else {
        lap_post_i16<M>(pv, Ry, pre, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
      }
      if constexpr (CHK) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const uint32_t v = oBest[i] & vmask[i];
          vmax[i] = pk_max(vmax[i], v);
          vmin[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
                                                     __builtin_bit_cast(s16x2, vmin[i]),
                                                     __builtin_bit_cast(s16x2, v)));
        }
      }
      if constexpr (FIN) {  // the final cell (src/TriAlign_1cyc.v:141-142,342-345)
        if (final_wg && w == (r_f >> 1)) {  // row r_f: half r_f & 1 of wave r_f / 2
#pragma unroll
          for (int i = 0; i < M; ++i) {
            if constexpr (LIT) {  // the cell's 7 inputs {M, Ix, Iy, Iz, Ixy, Iyz, Ixz}
              fin[(0 * M + i) * 64 + lane] = inM[i];
              fin[(1 * M + i) * 64 + lane] = inIx[i];
              fin[(2 * M + i) * 64 + lane] = Ry[i];
              fin[(3 * M + i) * 64 + lane] = inIz[i];
              fin[(4 * M + i) * 64 + lane] = inIxy[i];
              fin[(5 * M + i) * 64 + lane] = inIyz[i];
              fin[(6 * M + i) * 64 + lane] = inIxz[i];
            } else {
              fin[i * 64 + lane] = oBest[i];
            }
          }
        }
      }
      // ---- records: to the wave below (LDS), or (last wave) the y ring
      if constexpr (ROLE != 2) {
        if constexpr (SUCC_HERE) {
          constexpr int AHEAD = (QS >= 0 && TSA_LAP_GCHK && K == 4) ? 1 : 0;
          seen_out = max(seen_out, (int32_t)__builtin_amdgcn_readfirstlane(succ_v));
          wait_word(pw + 64 * (w + 1), seen_out, t + AHEAD - K + 2);  // wave w+1 read slot t % K's old record
        }
        uint8_t *dst = xr + (w * K + ((QS >= 0 ? QS : t) & (K - 1))) * SLOT + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const uint4 v = make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]);
          if constexpr (VB) lds_write16_at(v_rw, (ROLE == 0 ? 0 : WR_OFF) + ((VB ? QS : 0) & (K - 1)) * SLOT + i * PAIR, v);
          else lds_write16(dst + i * PAIR, v);
        }
      } else {
        if (yout) {
#if defined(TSA_DIAG)
          lag_y = max(lag_y, t - prog_decode(lds_word(bpw)));
#endif
          // (TSA_LAP_GCHK groups: once per group, for its last step)
          if (!(QS >= 0 && TSA_LAP_GCHK)) wait_consumer(cons_y, seen_y, bpw, t - YRm - YOFF + 1);
          else if (QS == 0) wait_consumer(cons_y, seen_y, bpw, t + 3 - YRm - YOFF + 1);
          const uint32_t tg = lap_tag(epoch, t);
          static_for<0, M>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            const uint4 v = make_uint4(perm(oIxy[i], oIy[i], 0x07060302u), tg,
                                       perm(oBest[i], oIyz[i], 0x07060302u), tg);
            constexpr int OFFB = (QS * M + i) * PAIR;
            if constexpr (VB && OFFB < 4096) store16_sc1_s<SYS, (VB ? OFFB : 0)>(yst_s, vlane, v);
            else if constexpr (QS >= 0 && OFFB < 4096) store16_sc1_at<SYS, OFFB>(yst_grp, v);
            else if constexpr (QS >= 0) store16_sc1<SYS>(yst_grp + OFFB, v);
            else store16_sc1<SYS>(yf_mine + ((int64_t)(t & (YRm - 1)) * M + i) * PAIR + lane * REC_BYTES, v);
          });
        }
        // my producers' back-pressure: the loader has checked at least
        // t - NW + 2 steps (wave 0 ran t - NW + 1 before this wave's step t)
        const bool pub_step = (QS >= 0 && LAP_PUB == 4) ? QS == 0 : (t & (LAP_PUB - 1)) == 0;
        if ((yin || zin) && pub_step && lane == 0)
        {
          const int32_t pv_ = (int32_t)((ep19 << 13) | (uint32_t)max(t - NW + 2, 0));
          __hip_atomic_store(prog + lid * LAP_PROG_STRIDE, pv_, __ATOMIC_RELAXED, SCOPE);
          if constexpr (SYS) {
            if (prog_x != nullptr) __hip_atomic_store(prog_x, pv_, __ATOMIC_RELAXED, SCOPE);
          }
        }
      }
      // ---- z record of this wave's last position (lane 63, register M-1)
      if (zout) {
#if defined(TSA_DIAG)
        lag_z = max(lag_z, t - prog_decode(lds_word(bpw + 1)));
#endif
        if (!(QS >= 0 && TSA_LAP_GCHK)) wait_consumer(cons_z, seen_z, bpw + 1, z_need(t));
        else if (QS == 0) wait_consumer(cons_z, seen_z, bpw + 1, z_need(t + 3));
        if (lane == 63) {
          const uint32_t tg = lap_tag(epoch, t);
          if constexpr (VB) {
            store16_sc1_s<SYS, (VB ? QS : 0) * ZREC>(zst_s, vlane, make_uint4(oIz[M - 1], tg, oIxz[M - 1], tg));
            store16_sc1_s<SYS, (VB ? QS : 0) * ZREC + 16>(zst_s, vlane, make_uint4(Ryz[M - 1], tg, Rb[M - 1], tg));
          } else if constexpr (QS >= 0) {
            store16_sc1_at<SYS, (QS >= 0 ? QS : 0) * ZREC>(zst_grp, make_uint4(oIz[M - 1], tg, oIxz[M - 1], tg));
            store16_sc1_at<SYS, (QS >= 0 ? QS : 0) * ZREC + 16>(zst_grp, make_uint4(Ryz[M - 1], tg, Rb[M - 1], tg));
          } else {
            uint8_t *zdst = zf_mine + (int64_t)(t & (ZRm - 1)) * ZREC + w * LAP_ZREC_WAVE;
            store16_sc1<SYS>(zdst, make_uint4(oIz[M - 1], tg, oIxz[M - 1], tg));
            store16_sc1<SYS>(zdst + 16, make_uint4(Ryz[M - 1], tg, Rb[M - 1], tg));
          }
        }
      }
      if constexpr (VB) {  // lds_publish through the base
        asm volatile("" ::: "memory");
        *(volatile __attribute__((address_space(3))) int32_t *)(v_pwb + pw_own(role)) = t + 1;
        asm volatile("" ::: "memory");
      } else {
        lds_publish(pw + 64 * w, t + 1, lane);
      }
#if defined(TSA_DIAG)
      const uint64_t pt3 = __builtin_amdgcn_s_memtime();
      prof[0] += pt1 - pt0;
      prof[1] += pt2 - pt1;
      prof[2] += pt3 - pt2;
      prof[3] += prof_last ? pt0 - prof_last : 0;
      prof_last = pt3;
#endif
      // ---- advance the systolic registers
#pragma unroll
      for (int i = 0; i < M; ++i) {
        oIx[i] = nIx[i];
        svIxy[i] = Rxy[i];
        pIy[i] = oIy[i];
        pIxy[i] = oIxy[i];
        pIyz[i] = oIyz[i];
        pBest[i] = oBest[i];
      }
      zshift<M>(shIxz[PH], oIxz, sel0, fIxz);
      zshift<M>(shIz, oIz, sel0, fIz);
      zshift<M>(svIyz, Ryz, sel0, fIyz);
      zshift<M>(svM[PH], Rb, sel0, fM);
    };
    auto run = [&](auto role) {  // the last step peeled off (it records the final cell)
      int32_t t = 0;
      const int32_t T1 = T - 1;
      constexpr std::integral_constant<int, 0> P0{};
      constexpr std::integral_constant<int, 1> P1{};
      constexpr std::false_type mid{};
      constexpr std::true_type last{};
      constexpr std::integral_constant<int, -1> QD{};
      if constexpr (U4K) {
        constexpr std::integral_constant<int, 0> Q0{};
        constexpr std::integral_constant<int, 1> Q1{};
        constexpr std::integral_constant<int, 2> Q2{};
        constexpr std::integral_constant<int, 3> Q3{};
#pragma unroll 1
        for (; t + 3 < T1; t += 4) {
          set_group(t);
          LAP_INLINE(step(P0, role, t, mid, Q0));
          LAP_INLINE(step(P1, role, t + 1, mid, Q1));
          LAP_INLINE(step(P0, role, t + 2, mid, Q2));
          LAP_INLINE(step(P1, role, t + 3, mid, Q3));
        }
      }
#pragma unroll 1
      for (; t + 1 < T1; t += 2) {
        a_pair = a_lane + 4u * (uint32_t)t;
        LAP_INLINE(step(P0, role, t, mid, QD));
        LAP_INLINE(step(P1, role, t + 1, mid, QD));
      }
      a_pair = a_lane + 4u * (uint32_t)t;
      if (t < T1) {
        LAP_INLINE(step(P0, role, t, mid, QD));
        LAP_INLINE(step(P1, role, t + 1, last, QD));
      } else {
        LAP_INLINE(step(P0, role, t, last, QD));
      }
    };
    static_assert(NW >= 2, "wave 0 and the last wave are distinct roles");
    if (w == 0) LAP_INLINE(run(std::integral_constant<int, 0>{}));
    else if (w == NW - 1) LAP_INLINE(run(std::integral_constant<int, 2>{}));
    else LAP_INLINE(run(std::integral_constant<int, 1>{}));
    if (trace != nullptr) {
      const unsigned long long clk1 = __builtin_amdgcn_s_memtime();
      stamp(2, now());
      if (tid == 0) {
        trace[(int64_t)b * LAP_TRACE_SLOTS + 5] = n_wait;
        trace[(int64_t)b * LAP_TRACE_SLOTS + 6] = clk1 - clk0;
      }
    }
    if (w == NW - 1 && lane == 0) w_bp[0] = (int32_t)n_bp;
    if constexpr (CHK) {  // the wave's extremes -> the triple's monitor words
      int32_t mx = 0, mn = 0;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int32_t lo0 = (int16_t)(vmax[i] & 0xFFFF), hi0 = (int16_t)(vmax[i] >> 16);
        const int32_t lo1 = (int16_t)(vmin[i] & 0xFFFF), hi1 = (int16_t)(vmin[i] >> 16);
        mx = max(mx, max(lo0, hi0));
        mn = min(mn, min(lo1, hi1));
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        mx = max(mx, __shfl_xor(mx, d));
        mn = min(mn, __shfl_xor(mn, d));
      }
      if (lane == 0) {
        if constexpr (TSA_CHK_SLOTS) {  // this wave's slot of [max] NC G NW, [min] NC G NW
          const int64_t nslot = (int64_t)NC * G * NW;
          mon[lid * NW + w] = mx;
          mon[nslot + lid * NW + w] = mn;
        } else {
          const int32_t ntri = NC / GZ;
          atomicMax(mon + tri, mx);
          atomicMin(mon + ntri + tri, mn);
        }
      }
    }
#if defined(TSA_DIAG)
    if (trace != nullptr && lane == 0 && w < 8)
      for (int k = 0; k < 4; ++k) trace[(int64_t)b * LAP_TRACE_SLOTS + 8 + 4 * w + k] = prof[k];
    if (trace != nullptr && lane == 0) {
      atomicMax(trace + (int64_t)b * LAP_TRACE_SLOTS + 40, (unsigned long long)max(lag_y, 0));
      atomicMax(trace + (int64_t)b * LAP_TRACE_SLOTS + 41, (unsigned long long)max(lag_z, 0));
    }
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the final cell and the loader's counters are in LDS
  if (trace != nullptr && tid == 0) {
    trace[(int64_t)b * LAP_TRACE_SLOTS + 4] = (unsigned long long)w_stall[0];
    trace[(int64_t)b * LAP_TRACE_SLOTS + 7] = (unsigned long long)w_bp[0];
  }
  if constexpr (LIT) {
    if (final_wg) {  // block-uniform: the final cell's 7-tuple, unshifted, and its MAX7
      const int32_t kf = k_f, hf = r_f & 1;
      if (tid < 7) {
        const uint32_t v = fin[(tid * M + kf % M) * 64 + kf / M];
        fin[7 * M * 64 + tid] = (uint32_t)((int32_t)(int16_t)(uint16_t)(hf ? (v >> 16) : (v & 0xFFFF)) >> lit.sh);
      }
      __syncthreads();
      if (tid == 0) {
        const bool bad = __hip_atomic_load(err, __ATOMIC_RELAXED, SCOPE) == epoch;
        int32_t best = (int32_t)fin[7 * M * 64];
        for (int k = 1; k < 7; ++k) best = max(best, (int32_t)fin[7 * M * 64 + k]);
        scores[tri] = bad ? TSA_SCORE_INVALID : best;  // FINAL MAX7, src/TriAlign_1cyc.v:141-142
        if (mon != nullptr)
          for (int k = 0; k < 7; ++k) mon[7 * (int64_t)tri + k] = (int32_t)fin[7 * M * 64 + k];
      }
    }
  } else if (final_wg && tid == 0) {
    const int32_t kf = k_f, hf = r_f & 1;
    const uint32_t v = fin[(kf % M) * 64 + kf / M];
    const uint16_t hb = (uint16_t)(hf ? (v >> 16) : (v & 0xFFFF));
    // a timed-out hand-off anywhere upstream invalidates the score (every
    // workgroup of the triple precedes this one): report it in-band
    const bool bad = __hip_atomic_load(err, __ATOMIC_RELAXED, SCOPE) == epoch;
    // VS: the final cell's value sits lam (la + lb + lc) above its score
    const int32_t vsh = VS ? pa.lam * (la + lb + lc) : 0;
    scores[tri] = bad ? TSA_SCORE_INVALID
                      : F16 ? (int32_t)(float)__builtin_bit_cast(_Float16, hb) - vsh : (int32_t)(int16_t)hb;
  }
  };
  const int32_t slots = (L1_ - L0_) * CH_, sx = rd_.SX;  // logical slots per XCD
  for (int32_t slot = (int32_t)(blockIdx.x >> 3); slot < slots; slot += sx) {
    lap_body(slot);
    __syncthreads();  // the next lap re-initialises this workgroup's LDS
  }
}

// Certification of the checked kernel's triples: a score stands when every
// best it saw lies in [best_min, best_max]. TSA_CHK_SLOTS: one workgroup per
// triple reduces its per_tri wave slots ([max] at mon, [min] at mon + nslot;
// slots of waves that did not run keep the launch's neutral fill); otherwise
// one thread per triple reads its two atomic words.
__global__ __launch_bounds__(256) void lap_certify(const int32_t *__restrict__ mon, int32_t n, int64_t nslot,
                                                   int32_t per_tri, CheckLimits lim, int32_t *__restrict__ scores) {
  if constexpr (TSA_CHK_SLOTS) {
    __shared__ int32_t red[2][4];
    const int32_t i = blockIdx.x;
    const int64_t base = (int64_t)i * per_tri;
    int32_t mx = INT32_MIN, mn = INT32_MAX;
    for (int32_t j = threadIdx.x; j < per_tri; j += 256) {
      mx = max(mx, mon[base + j]);
      mn = min(mn, mon[nslot + base + j]);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      mx = max(mx, __shfl_xor(mx, d));
      mn = min(mn, __shfl_xor(mn, d));
    }
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = mx;
      red[1][threadIdx.x >> 6] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      mx = max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3]));
      mn = min(min(red[1][0], red[1][1]), min(red[1][2], red[1][3]));
      if ((mx > lim.best_max || mn < lim.best_min) && scores[i] != TSA_SCORE_INVALID)
        scores[i] = TSA_SCORE_UNCERTIFIED;
    }
  } else {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (mon[i] > lim.best_max || mon[n + i] < lim.best_min) {
      if (scores[i] != TSA_SCORE_INVALID) scores[i] = TSA_SCORE_UNCERTIFIED;
    }
  }
}

// ---------------------------------------------------------------------------
// Host planning.

// Per-device facts the residency check needs, read once per device.
struct DevInfo {
  int cus = 256;
  bool known = false;
};
static DevInfo dev_info() {
  static DevInfo cache[64];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return DevInfo{};
  if (!cache[d].known) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && cus > 0)
      cache[d].cus = cus;
    cache[d].known = true;
  }
  return cache[d];
}

// The register bound on lap workgroups per CU: waves per SIMD the SGPR and
// VGPR files admit (build-time kernel table, kernel_meta.h), a workgroup of
// NW + 1 waves taking up to ceil((NW + 1) / 4) of them on one SIMD. The
// occupancy API counts waves per CU instead and reads one workgroup high at
// the SGPR edge (MI355X_MICROARCH.md:463) and, measured, at 96 VGPRs with
// 9-wave workgroups (it said 2, the CU ran 1).
// The bound is taken over every instantiation of the shape and form -- the
// checked (CHK) and split (SYS) ones too, whose register counts can differ
// from the plain kernel's -- so the grid plan holds whichever of them runs.
int lap_simd_blocks_per_cu(int M, int NW, bool f16, bool sop, bool lit) {
  // memo (value + 1; 0 = not yet computed): the table scans run per plan
  static std::atomic<int> memo[4][2][2][2][2];
  const int mi = M == 1 ? 0 : M == 2 ? 1 : M == 4 ? 2 : 3;
  std::atomic<int> &slot = memo[mi][NW == 8][f16][sop][lit];
  if (const int v = slot.load(std::memory_order_relaxed)) return v - 1;
  int sgpr = -1, vgpr = -1;
  for (int chk = 0; chk < 2; ++chk)
    for (int sys = 0; sys < 2; ++sys) {
      char prefix[80];  // lap_kernel<M, NW, F16, SOP, CHK, SYS, LIT>
      snprintf(prefix, sizeof prefix, "_ZN3tsa10lap_kernelILi%dELi%dELb%dELb%dELb%dELb%dELb%dE", M, NW,
               f16 ? 1 : 0, sop ? 1 : 0, chk, sys, lit ? 1 : 0);
      sgpr = std::max(sgpr, kernel_sgpr_max(prefix));
      vgpr = std::max(vgpr, kernel_vgpr_max(prefix));
    }
  const int waves = std::min(sgpr_waves_per_simd(sgpr < 0 ? 112 : sgpr), vgpr_waves_per_simd(vgpr < 0 ? 256 : vgpr));
  const int r = waves / ((NW + 1 + 3) / 4);
  slot.store(r + 1, std::memory_order_relaxed);
  return r;
}
// Workgroups of one shape a CU holds, from the HIP occupancy API on the real
// kernels (VGPRs, LDS) capped by the SGPR bound (the API reads one block high
// at 81-112 SGPRs); without a device, the LDS / wave-slot model. The API is
// asked about every instantiation the plan can launch -- the plain kernel, the
// checked (CHK) one of the int16 form and the V-space (VS) one of the f16
// form -- and the least count stands, so the looped grid's residency holds
// whichever of them runs. Memoized per (device, LDS bytes): a single-cube call
// plans a dozen geometries, and each occupancy query is host latency on that
// call.
template <int M, int NW, bool F16, bool SOP, bool LIT = false>
static int lap_blocks_per_cu_t(size_t lds) {
  struct Entry {
    int dev;
    size_t lds;
    int nb;
  };
  static std::mutex mu;
  static std::vector<Entry> memo;
  int nb = 0;
  int dev = -1;
  const int sg = lap_simd_blocks_per_cu(M, NW, F16, SOP, LIT);
  if (hipGetDevice(&dev) == hipSuccess) {
    {
      std::lock_guard<std::mutex> g(mu);
      for (const Entry &e : memo)
        if (e.dev == dev && e.lds == lds) return e.nb;
    }
    auto query = [&](auto kfn) -> int {
      int k = 0;
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(&k, kfn, 64 * (NW + 1), lds) == hipSuccess ? k : -1;
    };
    nb = query(lap_kernel<M, NW, F16, SOP, false, false, LIT>);
    if (nb >= 0) {
      if constexpr (!F16 && !LIT) nb = std::min(nb, std::max(0, query(lap_kernel<M, NW, false, SOP, true>)));
      if constexpr (F16 && !LIT)
        nb = std::min(nb, std::max(0, query(lap_kernel<M, NW, true, SOP, false, false, false, true>)));
      nb = std::min(nb, sg);
      std::lock_guard<std::mutex> g(mu);
      if (memo.size() < 4096) memo.push_back(Entry{dev, lds, nb});
      return nb;
    }
  }
  return (int)std::min<size_t>(std::min<size_t>(LDS_MAX / std::max<size_t>(lds, 1), 32 / (NW + 1)), sg);
}
template <int M, int NW, bool SOP>
static int lap_blocks_per_cu_lit(size_t lds) {
  return lap_blocks_per_cu_t<M, NW, false, SOP, true>(lds);
}
#define TSA_LAP_SHAPES(FN, M_, NW_, F16_, SOP_, ...)                                          \
  ((M_) == 1 ? ((NW_) == 4 ? TSA_ARITH(FN, 1, 4, F16_, SOP_, __VA_ARGS__)                      \
                           : TSA_ARITH(FN, 1, 8, F16_, SOP_, __VA_ARGS__))                     \
   : (M_) == 2 ? ((NW_) == 4 ? TSA_ARITH(FN, 2, 4, F16_, SOP_, __VA_ARGS__)                    \
                             : TSA_ARITH(FN, 2, 8, F16_, SOP_, __VA_ARGS__))                   \
               : ((NW_) == 4 ? TSA_ARITH(FN, 4, 4, F16_, SOP_, __VA_ARGS__)                    \
                             : TSA_ARITH(FN, 4, 8, F16_, SOP_, __VA_ARGS__)))
// The literal form's shapes: M = 1, 2 and NW = 4, 8, by s3 mode
#define TSA_LIT_SOP(FN, MM, NN, SOP_, ...) ((SOP_) ? FN<MM, NN, true>(__VA_ARGS__) : FN<MM, NN, false>(__VA_ARGS__))
#define TSA_LIT_SHAPES(FN, M_, NW_, SOP_, ...)                                                         \
  ((M_) == 1 ? ((NW_) == 4 ? TSA_LIT_SOP(FN, 1, 4, SOP_, __VA_ARGS__) : TSA_LIT_SOP(FN, 1, 8, SOP_, __VA_ARGS__)) \
             : ((NW_) == 4 ? TSA_LIT_SOP(FN, 2, 4, SOP_, __VA_ARGS__) : TSA_LIT_SOP(FN, 2, 8, SOP_, __VA_ARGS__)))

// Step time (us) along the chain, fitted on MI355X to single cubes
// (geometry sweeps profiles/r4m_lapgeo.jsonl, r4u_lap_nw.jsonl via
// scripts/gpu_lapgeo.sh; tools/lap_trace.py; DESIGN.md 4.4: 64^3..1024^3
// within ~10 %) and to batches of 4..128 cubes (profiles/r3o_chunk.jsonl:
// M = 4, 16 x 256^3 .. 4 x 1024^3), growing with the workgroups per CU -- the
// chain steps include the hand-off stalls.
// LIT: the literal cell's step, ~1.6x the message form's (single cubes and
// batches, profiles/r3l_literal_lap_vs_plane.jsonl, r3o_chunk.jsonl).
// M = 1 with two workgroups per CU (the latency-bound waves share SIMDs):
// ~0.97 us per chained step (16 x 256^3 and 1024^3 in rounds,
// profiles/r4c_lapab.jsonl), twice the one-per-CU step.
static double lap_step_us(int M, int NW, int64_t wg_per_cu, bool lit = false, bool one_round = false) {
  const double base = M == 1 ? (NW == 4 ? 0.40 : 0.49) : M == 2 ? 0.62 : 1.45;
  // per extra workgroup on the CU: two 9-wave M = 1 workgroups (4.5 waves per
  // SIMD) ~double the step; two 5-wave ones in one resident round barely slow
  // it (profiles/r4u_lap_nw.jsonl: 512^3 NW = 4 0.815 ms vs NW = 8 0.816,
  // 384^3 0.568 vs 0.599, literal 512^3 1.046 vs 1.132)
  const double share = M == 1 ? (NW == 4 && one_round ? 0.1 : 1.0) : 0.22;
  return (lit ? 1.6 : 1.0) * base * (1.0 + share * (double)(std::max<int64_t>(wg_per_cu, 1) - 1));
}

LapGeom lap_geom(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, int M, int NW,
                 bool full_rings, bool f16, bool sop, bool lit) {
#if defined(TSA_DIAG)  // A/B knob: full-length rings (no back-pressure) on every lap launch
  if (const char *e = getenv("TSA_LAP_FULL_RINGS")) full_rings = full_rings || atoi(e) != 0;
#endif
  LapGeom g{};
  g.M = M;
  g.NW = NW;
  g.chunk = 0;
  g.max_la = max_la;
  g.max_lb = max_lb;
  g.max_lc = max_lc;
  const int RW = 2 * NW, ZT = 64 * M, LPD = lap_pd(M);
  g.G = (max_lb + RW - 1) / RW;
  g.GZ = (max_lc + ZT - 1) / ZT;
  g.NC = n * g.GZ;             // columns: (triple, z-tile)
  g.CH = (g.NC + 7) / 8;       // columns per XCD
  const int YOFF = 2 * (NW - 1) + 1;  // lap lag of a record (kernel: YOFF)
  const int32_t T = max_la + YOFF + ZT;  // >= every workgroup's step count
  auto pow2 = [](int64_t v) { int64_t p = 1; while (p < v) p <<= 1; return (int32_t)p; };
  g.lds = lap_lds_bytes(M, NW, max_la, lit);
  const int64_t wgs = (int64_t)n * g.G * g.GZ;
  if (lit && (f16 || M > 2)) return g;  // the literal form's instantiations (.ok = false)
  const int per_cu = (g.lds > LDS_MAX) ? 0
                     : lit             ? TSA_LIT_SHAPES(lap_blocks_per_cu_lit, M, NW, sop, g.lds)
                                       : TSA_LAP_SHAPES(lap_blocks_per_cu_t, M, NW, f16, sop, g.lds);
  const int cus = dev_info().cus;
  // Slim rings: the lag between co-resident neighbours stays small (ring-lag
  // census, TSA_DIAG, profiles/r3e_lap_lag.jsonl): y <= 55 steps, z <= 207
  // beyond the natural ZT + ZA with one workgroup per CU; ~100 / ~200 with two
  // sharing a CU. So 32 (one per CU) or 96 slots beyond the natural lag,
  // rounded up to a power of 2. The big lags of round 2 (its workgroups start
  // as round-1 ones finish: 671 steps at 1024^3) go to the boundary rings.
  // A/B knob TSA_LAP_RING_SLACK (TSA_DIAG builds).
  int slack = (per_cu >= 2 && wgs > cus) ? 96 : 32;
#if defined(TSA_DIAG)
  if (const char *e = getenv("TSA_LAP_RING_SLACK")) slack = std::max(16, atoi(e));
#endif
  g.YR = full_rings ? pow2(T) : pow2(YOFF + LPD + slack);
  g.ZR = full_rings ? pow2(T) : pow2(ZT + LPD + slack);
  g.YRB = g.ZRB = pow2(T);
  g.blocks = (int64_t)g.G * g.CH * 8;
  // progress words, the error word (+63 spare), the checked kernel's monitor (2 n)
  // progress words, the error word (+63 spare), the checked kernel's monitor
  // (TSA_CHK_SLOTS: two words per compute wave; else two per triple)
  const size_t mon_words = TSA_CHK_SLOTS ? 2 * (size_t)wgs * NW : 2 * (size_t)n;
  g.prog_bytes = (((size_t)wgs * LAP_PROG_STRIDE + 64 + mon_words) * sizeof(int32_t) + 255) &
                 ~(size_t)255;
  g.yf_bytes = (size_t)wgs * g.YR * M * 1024;
  g.zf_bytes = (size_t)wgs * g.ZR * NW * LAP_ZREC_WAVE;
  if (g.lds > LDS_MAX || g.blocks > 0x7FFFFFFF) return g;
  // residency per XCD: block b runs on XCD b % 8 (column c's laps on XCD
  // c % 8), in block order, SX at a time (measured: tools/lap_trace.py xcc and
  // start stamps)
  const int64_t wg_per_xcd = (int64_t)g.G * g.CH;
  const int64_t slots_xcd = (int64_t)std::max(1, cus / 8) * per_cu;
  g.per_cu = per_cu;
  g.waves = per_cu > 0 ? (wg_per_xcd + slots_xcd - 1) / slots_xcd : 0;
  // dispatch rounds: boundary rings for producers whose consumer is in a later
  // round (kernel: y_bidx / z_bidx); one round, or full rings: none
  g.SX = (full_rings || g.waves <= 1 || per_cu <= 0) ? (1 << 30) : (int32_t)slots_xcd;
  g.grid = g.SX < (1 << 30) ? 8 * (int64_t)g.SX : g.blocks;  // one resident round, looped
  g.KBY = g.KBZ = 0;
  if (g.SX < (1 << 30)) {
    if (g.CH >= g.SX) {
      g.KBY = g.G;
    } else {
      for (int32_t c = 0; c < g.CH; ++c)
        g.KBY = std::max(g.KBY, ((g.G - 1) * g.CH + c) / g.SX - c / g.SX);
    }
    g.KBZ = (int32_t)g.waves;  // index: the producer's round (< rounds)
  }
  g.yb_bytes = (size_t)g.NC * g.KBY * g.YRB * M * 1024;
  g.zb_bytes = (size_t)g.KBZ * g.ZRB * NW * LAP_ZREC_WAVE;
  // one workgroup is the helix's job; a TSA_DIAG build allows it with
  // TSA_LAP_SINGLE=1 (the step time with no hand-off)
#if defined(TSA_DIAG)
  const bool single = getenv("TSA_LAP_SINGLE") && atoi(getenv("TSA_LAP_SINGLE")) != 0;
#else
  const bool single = false;
#endif
  g.ok = per_cu > 0 && (g.G >= 2 || g.GZ >= 2 || single);
  // estimated latency (us): the chain to the final workgroup -- each lap adds
  // YOFF + LPD + ~3 steps, each tile ZT + LPD + ~2 -- plus its own steps;
  // several workgroups on one CU share its SIMDs.
  const int64_t xcd_cus = std::max(1, cus / 8);
  const int64_t wg_cu = std::max<int64_t>(1, std::min<int64_t>(per_cu, (wg_per_xcd + xcd_cus - 1) / xcd_cus));
  const double steps = (double)(g.G - 1) * (YOFF + LPD + 3) + (double)(g.GZ - 1) * (ZT + LPD + 2) +
                       (double)(max_la + YOFF + ZT);
  const double step = lap_step_us(M, NW, wg_cu, lit, g.waves <= 1);
  const double chain = steps * step;
  // a slot's lap of round r + 1 starts when its lap of round r ends: one lap's
  // steps after its start, against (laps per round - 1) hand-offs of the chain
  // -- a round boundary delays the chain by the difference (round 2 of 1024^3,
  // M = 2, one workgroup per CU: 3.04 ms measured against a 2.25 ms chain)
  double delay = 0.0;
  if (g.waves > 1) {
    const double lpr = std::max(1.0, (double)g.SX / (double)g.CH);  // laps of a column per round
    const double lap_steps = (double)(max_la + YOFF + ZT) + (double)(g.GZ - 1) * (ZT + LPD + 2) / lpr;
    delay = std::max(0.0, lap_steps - (lpr - 1.0) * (YOFF + LPD + 3)) * step * 1.5;
  }
  g.est_us = chain + (double)(std::max<int64_t>(g.waves, 1) - 1) * delay;
  // refit on the round-4 runs (profiles/r4m_lapgeo.jsonl, r4j_lapab.jsonl,
  // r4t_literal_geo.jsonl): measured / estimated over several rounds is
  // 0.69-0.90 for M = 1 (1024^3 0.86, 768^3 0.90, 8 x 512^3 0.69, 16 x 256^3
  // 0.74) and 0.72-0.76 for the literal M = 1 (1024^3, 768^3), against
  // 0.84-1.15 for M = 2; the factors put 768^3 (1.90 vs 2.12 ms) and literal
  // 1024^3 (4.10 vs 4.37) on M = 1 and leave 1024^3 (2.98 vs 3.08), 8 x 512^3
  // and 16 x 256^3 on M = 2
  if (M == 1 && g.waves > 1) g.est_us *= lit ? 0.7 : 0.8;
  return g;
}

LapGeom lap_geom_chunked(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, int M, int NW, bool f16,
                         bool sop, bool lit) {
  LapGeom best{};
  best.ok = false;
  int32_t forced = 0;
  if (const char *e = getenv("TSA_LAP_CHUNK")) forced = std::max(0, atoi(e));  // knob (tests)
  // chunk sizes n, ceil(n/2), ceil(n/4), .. 1: a later launch starts once
  // the earlier one drains (~5 us between launches on one stream)
  for (int32_t k = n;; k = (k + 1) / 2) {
    const int32_t kk = forced > 0 ? std::min(forced, n) : k;
    LapGeom g = lap_geom(kk, max_la, max_lb, max_lc, M, NW, false, f16, sop, lit);
    // rounds run as each workgroup's loop over its slots (lap_kernel), in lap
    // order whatever the workgroups per CU
    if (g.ok && g.waves <= LAP_MAX_WAVES) {
      const int64_t launches = (n + kk - 1) / kk;
      g.chunk = kk < n ? kk : 0;
      g.est_us = g.est_us * (double)launches + 5.0 * (double)(launches - 1);
      if (!best.ok || g.est_us < best.est_us) best = g;
    }
    if (forced > 0 || k == 1) break;
  }
  return best;
}

size_t lap_workspace_bytes(const LapGeom &g) {
  return g.prog_bytes + g.yf_bytes + g.zf_bytes + g.yb_bytes + g.zb_bytes;
}
static LapRounds lap_rounds(const LapGeom &g, void *d_ws) {
  uint8_t *yb = (uint8_t *)d_ws + g.prog_bytes + g.yf_bytes + g.zf_bytes;
  return LapRounds{g.SX, g.KBY, g.YRB, g.ZRB, yb, yb + g.yb_bytes};
}
// The error word sits after the progress words of the workgroups the
// geometry was built for (NC * G; one chunk's, whatever the batch size), the
// checked kernel's monitor words 64 words further.
uint32_t *lap_err_word(const LapGeom &g, int32_t n, void *d_ws) {
  (void)n;
  return (uint32_t *)((int32_t *)d_ws + (int64_t)g.NC * g.G * LAP_PROG_STRIDE);
}

static uint32_t lap_spin_limit() {
  if (const char *e = getenv("TSA_LAP_SPIN_LIMIT")) return (uint32_t)strtoul(e, nullptr, 0);
  return 1u << 22;
}
static uint32_t lap_next_epoch() {
  static std::atomic<uint32_t> ctr{(uint32_t)time(nullptr) * 2654435761u ^ (uint32_t)getpid() * 40503u};
  uint32_t e;
  do { e = ctr.fetch_add(1) + 1; } while (e == 0);
  return e;
}

typedef decltype(&lap_kernel<1, 4, true, false, false>) LapKernelFn;  // every instantiation's type
// aux: the checked kernel's monitor words (chk), or the LIT kernel's final
// 7-tuples (may be null)
// One launch of n triples on geometry g (built for n) inside the workspace
// of the allocation geometry ga (the batch's chunk geometry; g itself for a
// single launch): every region at ga's offset -- progress words, y / z rings,
// boundary rings -- and the error word / the checked kernel's monitor words at
// ga's place (lap_err_word), the same for every chunk of a batch.
static int launch_lap_fn(LapKernelFn kfn, int NW, const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                         const LapGeom &g, const LapGeom &ga, int32_t *d_scores, void *d_ws,
                         const PencilArgs &pa, const LitArgs &lit, int32_t *aux, hipStream_t stream,
                         const CheckLimits *chk) {
  if (g.lds > LDS_MAX) return TSA_EINVAL;
  if (g.prog_bytes > ga.prog_bytes || g.yf_bytes > ga.yf_bytes || g.zf_bytes > ga.zf_bytes ||
      g.yb_bytes > ga.yb_bytes || g.zb_bytes > ga.zb_bytes)
    return TSA_EINTERNAL;  // a chunk's regions must fit the batch's
  int32_t *prog = (int32_t *)d_ws;
  uint32_t *err = lap_err_word(ga, n, d_ws);
  // [max(best)] nslot, [min(best)] nslot: one slot per compute wave of this
  // launch (TSA_CHK_SLOTS), else per triple; neutral fill for waves that do not run
  int32_t *mon = chk ? (int32_t *)err + 64 : aux;
  const int64_t nslot = TSA_CHK_SLOTS ? (int64_t)g.NC * g.G * NW : (int64_t)n;
  if (chk && (hipMemsetAsync(mon, 0x80, (size_t)nslot * 4, stream) != hipSuccess ||
              hipMemsetAsync(mon + nslot, 0x7F, (size_t)nslot * 4, stream) != hipSuccess))
    return TSA_EDEVICE;
  uint8_t *yf = (uint8_t *)d_ws + ga.prog_bytes;
  uint8_t *zf = yf + ga.yf_bytes;
  uint8_t *yb = zf + ga.zf_bytes;
  const LapRounds rd{g.SX, g.KBY, g.YRB, g.ZRB, yb, yb + ga.yb_bytes};
  unsigned long long *trace = nullptr;
  const char *tpath = getenv("TSA_LAP_TRACE");  // diagnostic: per-WG timestamps to a CSV file
  const size_t tbytes = (size_t)g.blocks * LAP_TRACE_SLOTS * 8;
  if (tpath && hipMalloc(&trace, tbytes) != hipSuccess) return TSA_ENOMEM;
  if (trace && hipMemsetAsync(trace, 0, tbytes, stream) != hipSuccess)
    return TSA_EDEVICE;
  const uint32_t epoch = lap_next_epoch();
  const LapKArgs ka{d_seqs, d_offsets, g.G, g.GZ, g.NC, g.CH, g.YR, g.ZR, yf, zf, rd, prog, err,
                    d_scores, mon, pa, epoch, lap_spin_limit(), 0, g.G, yf, prog, trace, lit};
  if (launch_with_lds((const void *)kfn, g.lds, [&] {
        hipLaunchKernelGGL(kfn, dim3((uint32_t)g.grid), dim3(64 * (NW + 1)), g.lds, stream, LAP_KARGS(ka));
      }) != hipSuccess)
    return TSA_EDEVICE;
  if (chk) {
    hipLaunchKernelGGL(lap_certify, dim3((uint32_t)(TSA_CHK_SLOTS ? n : (n + 255) / 256)), dim3(256), 0, stream,
                       mon, n, nslot, (int32_t)(g.G * g.GZ * NW), *chk, d_scores);
  }
  if (hipGetLastError() != hipSuccess) return TSA_EDEVICE;
  if (trace) {
    std::vector<unsigned long long> h((size_t)g.blocks * LAP_TRACE_SLOTS);
    if (hipMemcpyAsync(h.data(), trace, h.size() * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return TSA_EDEVICE;
    (void)hipFree(trace);
    if (FILE *fp = fopen(tpath, "w")) {
      fprintf(fp, "block,tri,lap,tile,start,loop_begin,loop_end,xcc,stalls,w0_waits,loop_clk,bp_waits");
      for (int k = 8; k < 40 && k < LAP_TRACE_SLOTS; ++k)  // TSA_DIAG: wave (k-8)/4, phase (k-8)%4
        fprintf(fp, ",prof%d_%d", (k - 8) / 4, (k - 8) % 4);
      if (LAP_TRACE_SLOTS > 40) fprintf(fp, ",lag_y,lag_z");
      fprintf(fp, "\n");
      for (int64_t b = 0; b < g.blocks; ++b) {
        const unsigned long long *hb = h.data() + b * LAP_TRACE_SLOTS;
        if (hb[0] == 0) continue;  // padding block
        const int64_t slot = b >> 3, col = (slot % g.CH) * 8 + (b & 7);
        fprintf(fp, "%lld,%lld,%lld,%lld,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu", (long long)b,
                (long long)(col / g.GZ), (long long)(slot / g.CH), (long long)(col % g.GZ), hb[0],
                hb[1], hb[2], hb[3], hb[4], hb[5], hb[6], hb[7]);
        for (int k = 8; k < LAP_TRACE_SLOTS; ++k) fprintf(fp, ",%llu", hb[k]);
        fprintf(fp, "\n");
      }
      fclose(fp);
    }
  }
  return TSA_OK;
}
// A batch on geometry g: one launch, or (g.chunk) launches of g.chunk
// triples one after another on the stream, each with its own epoch; the last
// chunk's geometry is built for its own size, inside g's workspace.
template <class F>
static int for_each_chunk(const LapGeom &g, int32_t n, bool f16, bool sop, bool lit, F &&launch) {
  const int32_t k = (g.chunk > 0 && g.chunk < n) ? g.chunk : n;
  for (int32_t c0 = 0; c0 < n; c0 += k) {
    const int32_t cn = std::min(k, n - c0);
    const LapGeom gc = cn == k ? g : lap_geom(cn, g.max_la, g.max_lb, g.max_lc, g.M, g.NW, false, f16, sop, lit);
    if (!gc.ok && cn != k) return TSA_EINTERNAL;
    const int rc = launch(gc, c0, cn);
    if (rc) return rc;
  }
  return TSA_OK;
}
template <int M, int NW, bool F16, bool SOP>
static int launch_lap(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                      const LapGeom &g, int32_t *d_scores, void *d_ws, const PencilArgs &pa,
                      hipStream_t stream, const CheckLimits *chk) {
  if (chk && F16) return TSA_EINVAL;
  // pa.lam != 0: the V-space cell (make_args(..., vs = true); f16 only)
  LapKernelFn kfn = chk ? lap_kernel<M, NW, F16, SOP, !F16> : lap_kernel<M, NW, F16, SOP, false>;
  if constexpr (F16) {
    if (pa.lam != 0) kfn = lap_kernel<M, NW, true, SOP, false, false, false, true>;
  }
  return for_each_chunk(g, n, F16, SOP, false, [&](const LapGeom &gc, int32_t c0, int32_t cn) {
    return launch_lap_fn(kfn, NW, d_seqs, d_offsets + 3 * (int64_t)c0, cn, gc, g, d_scores + c0, d_ws, pa,
                         LitArgs{}, nullptr, stream, chk);
  });
}
template <int M, int NW, bool SOP>
static int launch_lap_lit(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, const LapGeom &g,
                          int32_t *d_scores, int32_t *d_final7, void *d_ws, const PencilArgs &pa,
                          const LitArgs &lit, hipStream_t stream) {
  return for_each_chunk(g, n, false, SOP, true, [&](const LapGeom &gc, int32_t c0, int32_t cn) {
    return launch_lap_fn(lap_kernel<M, NW, false, SOP, false, false, true>, NW, d_seqs, d_offsets + 3 * (int64_t)c0,
                         cn, gc, g, d_scores + c0, d_ws, pa, lit, d_final7 ? d_final7 + 7 * (int64_t)c0 : nullptr,
                         stream, nullptr);
  });
}

int lap_launch_lit(const LapGeom &g, bool sop, const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                   int32_t *d_scores, int32_t *d_final7, void *d_ws, const KParams &kp, hipStream_t stream,
                   int32_t **d_err) {
  if (g.M > 2 || (g.NW != 4 && g.NW != 8)) return TSA_EINVAL;
  if (d_err) {  // synchronous caller: clear the error word, it reads it back
    *d_err = (int32_t *)lap_err_word(g, n, d_ws);
    if (hipMemsetAsync(*d_err, 0, sizeof(int32_t), stream) != hipSuccess) return TSA_EDEVICE;
  }
  PencilArgs pa{};  // the literal form reads only the packed flag; zero faces
  pa.packed = kp.packed;
  const LitArgs lit = lit_args(kp);
  return TSA_LIT_SHAPES(launch_lap_lit, g.M, g.NW, sop, d_seqs, d_offsets, n, g, d_scores, d_final7, d_ws, pa,
                        lit, stream);
}

int lap_launch(const LapGeom &g, bool f16, bool sop, const uint8_t *d_seqs,
               const int64_t *d_offsets, int32_t n, int32_t *d_scores, void *d_ws,
               const PencilArgs &pa, hipStream_t stream, int32_t **d_err,
               const CheckLimits *chk) {
  if (d_err) {  // synchronous caller: clear the error word, it reads it back
    *d_err = (int32_t *)lap_err_word(g, n, d_ws);
    if (hipMemsetAsync(*d_err, 0, sizeof(int32_t), stream) != hipSuccess) return TSA_EDEVICE;
  }
  return TSA_LAP_SHAPES(launch_lap, g.M, g.NW, f16, sop, d_seqs, d_offsets, n, g, d_scores, d_ws,
                        pa, stream, chk);
}

// ---------------------------------------------------------------------------
// One cube split over devices by laps (tsa_score_gpu_multi): part p runs laps
// [L0_p, L1_p) on its own device; part p's last lap writes its y records into
// part p+1's workspace and part p+1's first lap copies its progress words into
// part p's, so each hand-off crossing the link is a posted store and every
// poll stays local. The error word and the score live with the last part.
static int launch_split_fn(LapKernelFn kfn, int NW, const LapGeom &g, const PencilArgs &pa, const LitArgs &lit,
                           const LapPart *parts, int np, int32_t *d_score, uint32_t *d_err) {
  const uint32_t epoch = lap_next_epoch();
  const uint32_t spin = lap_spin_limit();
  for (int p = 0; p < np; ++p) {
    const LapPart &q = parts[p];
    if (hipSetDevice(q.device) != hipSuccess) return TSA_EDEVICE;
    int32_t *prog = (int32_t *)q.d_ws;
    uint8_t *yf = (uint8_t *)q.d_ws + g.prog_bytes;
    uint8_t *zf = yf + g.yf_bytes;
    uint8_t *yf_out = p + 1 < np ? (uint8_t *)parts[p + 1].d_ws + g.prog_bytes : yf;
    int32_t *prog_in = p > 0 ? (int32_t *)parts[p - 1].d_ws : prog;
    const int64_t blocks = (int64_t)(q.L1 - q.L0) * g.CH * 8;
    const LapKArgs ka{q.d_seqs, q.d_offsets, g.G, g.GZ, g.NC, g.CH, g.YR, g.ZR, yf, zf, lap_rounds(g, q.d_ws),
                      prog, d_err, d_score, (int32_t *)nullptr, pa, epoch, spin, q.L0, q.L1, yf_out, prog_in,
                      (unsigned long long *)nullptr, lit};
    if (launch_with_lds((const void *)kfn, g.lds, [&] {
          hipLaunchKernelGGL(kfn, dim3((uint32_t)blocks), dim3(64 * (NW + 1)), g.lds, q.stream, LAP_KARGS(ka));
        }) != hipSuccess)
      return TSA_EDEVICE;
  }
  return TSA_OK;
}
template <int M, int NW, bool F16, bool SOP>
static int launch_lap_split(const LapGeom &g, const PencilArgs &pa, const LapPart *parts, int np,
                            int32_t *d_score, uint32_t *d_err) {
  return launch_split_fn(lap_kernel<M, NW, F16, SOP, false, true>, NW, g, pa, LitArgs{}, parts, np, d_score, d_err);
}
template <int M, int NW, bool SOP>
static int launch_lap_split_lit(const LapGeom &g, const PencilArgs &pa, const LitArgs &lit, const LapPart *parts,
                                int np, int32_t *d_score, uint32_t *d_err) {
  return launch_split_fn(lap_kernel<M, NW, false, SOP, false, true, true>, NW, g, pa, lit, parts, np, d_score,
                         d_err);
}
static int split_parts_ok(const LapGeom &g, const LapPart *parts, int np) {
  if (np < 1 || g.lds > LDS_MAX) return 0;
  for (int p = 0; p < np; ++p)
    if (parts[p].L0 >= parts[p].L1 || parts[p].L0 != (p ? parts[p - 1].L1 : 0)) return 0;
  return parts[np - 1].L1 == g.G;
}

int lap_launch_split(const LapGeom &g, bool f16, bool sop, const PencilArgs &pa, const LapPart *parts,
                     int np, int32_t *d_score, uint32_t *d_err) {
  if (!split_parts_ok(g, parts, np)) return TSA_EINVAL;
  return TSA_LAP_SHAPES(launch_lap_split, g.M, g.NW, f16, sop, g, pa, parts, np, d_score, d_err);
}

int lap_launch_split_lit(const LapGeom &g, bool sop, const KParams &kp, const LapPart *parts, int np,
                         int32_t *d_score, uint32_t *d_err) {
  if (!split_parts_ok(g, parts, np) || g.M > 2 || (g.NW != 4 && g.NW != 8)) return TSA_EINVAL;
  PencilArgs pa{};  // as lap_launch_lit: the packed flag only, zero faces
  pa.packed = kp.packed;
  const LitArgs lit = lit_args(kp);
  return TSA_LIT_SHAPES(launch_lap_split_lit, g.M, g.NW, sop, g, pa, lit, parts, np, d_score, d_err);
}

}  // namespace tsa
