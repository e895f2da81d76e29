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
//  * wave w holds TWO DP rows, y = L*RW + 2w + 1 in the low 16-bit half and
//    y + 1 in the high half of every packed register -- a lap of RW rows needs
//    only NW waves, one per SIMD for NW = 4, which is what a latency-bound
//    chain wants (a step is one wave's dependent instruction stream, not four
//    waves sharing a SIMD);
//  * lane l, register i is tile position k = M*l + i (z = q*ZT + k + 1); half
//    h of wave w computes x = t - (2w + h) - k + 1 at local step t;
//  * the high half's row above is the wave's own low half one step earlier, the
//    low half's is wave w-1's high half (LDS record, one barrier per step):
//    one v_alignbit/v_perm per record word (REC = {above.hi, own_prev.lo});
//  * z-1 neighbours shift one position per step (register rename, one DPP
//    wave_ror + one v_perm per message), the x = 1 position takes the x = 0
//    face (src/PE_1cyc.v:164-218 EN_i gating), as in the helix kernel.
// Between workgroups (MI355X_MICROARCH.md "handoff-1to1"):
//  * the last wave stores its per-step record (the high halves the next lap's
//    wave 0 needs) into a y ring of YR slots, and every wave's last position
//    ({Iz, Ixz, REC.z, REC.w}) goes into a z ring of ZR slots for tile q+1;
//  * every 8-byte granule of a record carries a 32-bit tag of (launch epoch,
//    step), written by one sc1 store: the consumer LDS-DMAs records LPD steps
//    ahead and checks the tags where it uses them -- no flags, no polls on the
//    fast path; a stale tag re-fetches (bounded; on timeout the launch's error
//    word is set and the triple reports TSA_SCORE_INVALID);
//  * the rings are O(N^2) (O(N) per workgroup): a consumer publishes its
//    progress every 4 steps and a producer about to overwrite a slot the
//    consumer may still need waits for it (never on the fast path: the rings
//    hold 2-4x the natural lag);
//  * block b -> XCD b % 8 (observed dispatch, speed only): every lap of a z-tile
//    lands on one XCD, so the y chain's hand-offs stay in one L2's reach.
// A workgroup only waits on workgroups of lower block index (lap-major order),
// so a grid beyond the resident slots is safe with in-order dispatch when the
// rings are full length (no back-pressure): LAP_STREAM uses that.

#include <unistd.h>

#include <atomic>
#include <ctime>
#include <vector>

#include "pencil_common.h"
#include "lap_kernel.h"

namespace tsa {

#ifndef TSA_LAP_PD1  // LDS-DMA prefetch distance (steps) by M: build-time knobs
#define TSA_LAP_PD1 3
#endif
#ifndef TSA_LAP_PD2
#define TSA_LAP_PD2 6
#endif
#ifndef TSA_LAP_PD4
#define TSA_LAP_PD4 4
#endif
__host__ __device__ constexpr int lap_pd(int M) {
  return M == 1 ? TSA_LAP_PD1 : M == 2 ? TSA_LAP_PD2 : TSA_LAP_PD4;
}
constexpr int LAP_ZL = 16;         // z records resident in LDS (power of 2, > lap_pd + 2)
constexpr int LAP_PUB = 4;         // consumers publish their progress every LAP_PUB steps
constexpr int LAP_PROG_STRIDE = 32;  // progress words 128 B apart (one line each)
constexpr int LAP_ZREC_WAVE = 32;  // z record bytes per wave: 4 x {payload, tag}

#ifndef TSA_LAP_SKEW  // steps between a wave's high row and the next wave's low row
#define TSA_LAP_SKEW 1
#endif
// SK = 1: one barrier per step, the wave below reads this step's record next
// step; SK = 2: a wave reads the record of two steps ago, one barrier per two
// steps (tools/lap_emu.py replays both)
constexpr int LAP_SK = TSA_LAP_SKEW;
static_assert(LAP_SK == 1 || LAP_SK == 2, "lap skew");
static_assert(LAP_ZL > TSA_LAP_PD1 + 2 + LAP_SK && LAP_ZL > TSA_LAP_PD2 + 2 + LAP_SK, "z slots");

// Tag of the record of step s in the launch with epoch e (32-bit): distinct
// steps of one launch never collide (odd multiplier).
__host__ __device__ __forceinline__ uint32_t lap_tag(uint32_t e, int32_t s) {
  return e ^ ((uint32_t)s * 0x9E3779B1u);
}

static size_t lap_lds_bytes(int M, int NW, int32_t max_la) {
  const int ZT = 64 * M, SLOT = M * 1024;
  return (size_t)(NW - 1) * 2 * LAP_SK * SLOT + (size_t)lap_pd(M) * SLOT + 4 * (size_t)NW * 16 +
         (size_t)LAP_ZL * NW * LAP_ZREC_WAVE + 16 + (size_t)M * 256 +
         4 * (((size_t)max_la + 2 * ZT + 2 * (LAP_SK + 1) * NW + 8 + 3) & ~(size_t)3);
}

// ---------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// The s_nop: a VMEM store of more than 8 bytes must not have its data VGPRs
// rewritten by the next VALU instruction (one wait state); the compiler's
// hazard recognizer does not look inside inline asm, so the asm carries it.
__device__ __forceinline__ void store16_sc1(void *gptr, uint4 v) {
  const u32x4 d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(gptr), "v"(d) : "memory");
}
__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}
// {above.hi -> lo, own.lo -> hi}: the row above of both halves
__device__ __forceinline__ uint32_t rows2(uint32_t own, uint32_t above) {
  return __builtin_amdgcn_alignbit(own, above, 16);
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

// LDS (bytes):
//   xr    [NW-1][2SK][M][64][16] wave w -> w+1 records {Iy, Ixy, Iyz, best}
//   xr0   [LPD][M][64][16]      tagged y records of the lap above (LDS-DMA)
//   zst   [4][NW][16]           z staging {Iz, Ixz, REC.z, REC.w} of lane 63
//   zring [ZL][NW][32]          tagged z records of the tile to the left
//   bpw   [4] i32               consumers' progress words (LDS-DMA'd)
//   fin   [M][64] u32           best of the final step
//   sA2   [..] u32              A code pairs: entry j = x j-OFF (lo), j-OFF-1 (hi)
// Minimum waves per SIMD the register allocation must allow: pins occupancy
// (and keeps SGPRs <= ~80, which the CU's admission of 256-thread blocks also
// depends on, MI355X_MICROARCH.md "Residency"), so the occupancy API's answer
// is what the hardware admits and a resident grid stays resident.
__host__ __device__ constexpr int lap_waves_per_eu(int M) { return M == 1 ? 8 : M == 2 ? 4 : 2; }
// every step of the lap kernel inlined (outlined, the captures go to scratch)
#define LAP_INLINE(call) \
  do {                    \
    [[clang::always_inline]] call; \
  } while (0)

template <int M, int NW, bool F16, bool SOP>
__global__ __launch_bounds__(64 * NW, lap_waves_per_eu(M)) void lap_kernel(
    const uint8_t *__restrict__ seqs, const int64_t *__restrict__ offs, int32_t G, int32_t GZ,
    int32_t NC, int32_t CH, int32_t YR, int32_t ZR, uint8_t *__restrict__ yf_base,
    uint8_t *__restrict__ zf_base, int32_t *__restrict__ prog, uint32_t *__restrict__ err,
    int32_t *__restrict__ scores, PencilArgs pa, uint32_t epoch, uint32_t spin_limit,
    unsigned long long *__restrict__ trace) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int RW = 2 * NW, ZT = 64 * M, LPD = lap_pd(M);
  constexpr int PAIR = 64 * REC_BYTES, SLOT = M * PAIR;
  // wave w's rows sit at step offsets WO*w (low half) and WO*w + 1 (high);
  // lap L+1 reads lap L's record t + YOFF; z records are checked ZV steps ahead
  constexpr int SK = LAP_SK, WO = SK + 1, NSL = 2 * SK, YOFF = WO * (NW - 1) + 1, ZV = SK;
  constexpr int ZREC = NW * LAP_ZREC_WAVE, OFF = ZT + WO * NW;
  uint8_t *xr = smem;
  uint8_t *xr0 = xr + (NW - 1) * NSL * SLOT;
  uint8_t *zst = xr0 + LPD * SLOT;
  uint8_t *zring = zst + 4 * NW * 16;
  int32_t *bpw = (int32_t *)(zring + LAP_ZL * ZREC);
  uint32_t *fin = (uint32_t *)(bpw + 4);
  uint32_t *sA2 = fin + M * 64;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block -> (lap, column): column c = tri*GZ + q (one z-tile of one triple), block
  // b = 8 * (L*CH + c/8) + c%8 -- a column's laps share b % 8 (one XCD), and
  // every producer ((L-1, c), (L, c-1)) has a lower block index than its consumer
  const int32_t b = blockIdx.x, slot = b >> 3;
  const int32_t L = slot / CH, col = (slot % CH) * 8 + (b & 7);
  if (col >= NC) return;  // padding block
  const int32_t tri = col / GZ, q = col % GZ;
  const int64_t o0 = offs[3 * (int64_t)tri], o1 = offs[3 * (int64_t)tri + 1];
  const int64_t o2 = offs[3 * (int64_t)tri + 2], o3 = offs[3 * (int64_t)tri + 3];
  const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
  const int32_t nlap = (lb + RW - 1) / RW, ntile = (lc + ZT - 1) / ZT;
  if (L >= nlap || q >= ntile) return;  // beyond this triple's own laps / tiles
  auto stamp = [&](int s, unsigned long long v) {
    if (trace != nullptr && threadIdx.x == 0) trace[(int64_t)b * 8 + s] = v;
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
  auto tau = [](int32_t r) { return WO * (r >> 1) + (r & 1); };  // step offset of lap row r
  const int32_t r_f = lb - 1 - L * RW, k_f = lc - 1 - q * ZT;
  const int32_t T = final_wg ? (la - 1) + tau(r_f) + k_f + 1 : la + tau(rows - 1) + zt_q - 1;
  const int32_t T_above = la + tau(RW - 1) + zt_q - 1;  // records the lap above writes (same tile)
  const int32_t T_left = la + tau(rows - 1) + ZT - 1;   // z records the tile to the left writes
  uint8_t *yf_mine = yf_base + lid * YR * SLOT;
  const uint8_t *yf_prev = yin ? yf_base + (lid - GZ) * YR * SLOT : yf_mine;
  uint8_t *zf_mine = zf_base + lid * ZR * ZREC;
  const uint8_t *zf_prev = zin ? zf_base + (lid - 1) * ZR * ZREC : zf_mine;
  const uint32_t ep19 = epoch & 0x7FFFFu;
  bool timed_out = false;
  auto fail = [&]() {  // release: visible before any record this workgroup stores later
    if (!timed_out && lane == 0)
      __hip_atomic_store(err, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    timed_out = true;
  };

  // ---- A code pairs, per-row and per-position registers
  const int32_t na = la + 2 * ZT + 2 * WO * NW + 8;
  for (int j = threadIdx.x; j < na; j += 64 * NW) {
    const int x0 = j - OFF, x1 = j - OFF - 1;
    const uint32_t c0 = (x0 >= 0 && x0 < la) ? SYM0 << (seqs[o0 + x0] & 3) : 0u;
    const uint32_t c1 = (x1 >= 0 && x1 < la) ? SYM0 << (seqs[o0 + x1] & 3) : 0u;
    sA2[j] = c0 | (c1 << 16);
  }
  // a[i] of this lane at step t = sA2[t - WO w - (M lane + i) + OFF]
  const uint32_t a_lane = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)sA2 +
                          4u * (uint32_t)(OFF - WO * w - M * lane - (M - 1));
  const int32_t y0 = L * RW + 2 * w;  // rows y0 (lo) and y0 + 1 (hi), 0-based
  const uint32_t bw = (y0 < lb ? SYM0 << (seqs[o1 + y0] & 3) : 0u) |
                      ((y0 + 1 < lb ? SYM0 << (seqs[o1 + y0 + 1] & 3) : 0u) << 16);
  uint32_t bv[M], c[M], SBC[M], K[M], DMC[M];
  uint32_t oIx[M], shIz[M], svIxy[M], svIyz[M], shIxz[2][M], svM[2][M];
  uint32_t pIy[M], pIxy[M], pIyz[M], pBest[M];  // this wave's record of the previous step
  {
    uint32_t one1 = 0x00010001u, sbcv = pa.h_sbc, kdv = pa.h_kd, k0v = pa.h_k0;
    asm volatile("" : "+v"(one1), "+v"(sbcv), "+v"(kdv), "+v"(k0v));
    const int64_t oc = o2 + (int64_t)q * ZT;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int k = M * lane + i;
      c[i] = (k < zt_q ? SYM0 << (seqs[oc + k] & 3) : 0u) * 0x00010001u;
      DMC[i] = dm_over_code(pa.dmf, c[i]);
      bv[i] = bw;
      const uint32_t e01 = pk_eq1(bw, c[i], one1);
      SBC[i] = pk_mad(e01, sbcv, 0u);
      K[i] = pk_mad(e01, kdv, k0v);
      oIx[i] = shIz[i] = pa.f_single;
      shIxz[0][i] = shIxz[1][i] = svIxy[i] = svIyz[i] = pa.f_pair;
      svM[0][i] = svM[1][i] = 0;
      pIy[i] = pIxy[i] = pIyz[i] = pBest[i] = 0;
    }
  }
  uint32_t Q = F16 ? 0x08000800u : 0x00010001u, fsv = pa.f_single, fpv = pa.f_pair;
  uint32_t mlo = 0x0000FFFFu, mhi = 0xFFFF0000u;
  asm volatile("" : "+v"(Q), "+v"(fsv), "+v"(fpv), "+v"(mlo), "+v"(mhi));
  const PencilArgs pv = F16 ? pa : pin_score_consts(pa);
  const uint32_t sel0 = lane == 0 ? 0x03020100u : 0x07060504u;  // lane 0: whole word from the face

  // ---- producer side (last wave): the consumers' progress (y: lap below, z: tile right)
  const int64_t cons_y = yout ? lid + GZ : -1, cons_z = zout ? lid + 1 : -1;
  int32_t seen_y = -1, seen_z = -1;  // consumer steps known to be complete
  auto prog_decode = [&](int32_t v) -> int32_t {
    return ((uint32_t)v >> 13) == ep19 ? (int32_t)(v & 0x1FFF) - 1 : -1;
  };
  uint32_t n_stall = 0, n_bp = 0;  // diagnostics (trace)
  // wait until the consumer's progress covers `need`; the LDS word is a lower
  // bound refreshed by LDS-DMA every 8 steps, the blocking poll the slow path
  auto wait_consumer = [&](int64_t cons, int32_t &seen, int32_t *word, int32_t need) {
    if (need <= seen) return;
    seen = max(seen, prog_decode(lds_word(word)));
    if (need <= seen) return;
    ++n_bp;
    for (uint32_t spin = 0;; ++spin) {
      const int32_t v = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(prog + cons * LAP_PROG_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      seen = max(seen, prog_decode(v));
      if (need <= seen) return;
      if (spin >= spin_limit) { fail(); seen = 1 << 20; return; }
      __builtin_amdgcn_s_sleep(2);
    }
  };

  // ---- consumer side (wave 0): fetches, tag checks
  auto fetch_y = [&](int32_t s) {  // records of step s (row s + YOFF above) -> xr0 slot s % LPD
    const int32_t r = s + YOFF;
#pragma unroll
    for (int i = 0; i < M; ++i)
      dma16(yf_prev + ((int64_t)(r & (YR - 1)) * M + i) * PAIR + lane * REC_BYTES,
            xr0 + (s % LPD) * SLOT + i * PAIR);
  };
  auto fetch_z = [&](int32_t rz) {  // z record rz -> zring slot rz % ZL (lanes 0 .. 2NW-1)
    if (lane < 2 * NW)
      dma16(zf_prev + (int64_t)(rz & (ZR - 1)) * ZREC + lane * 16,
            zring + (rz & (LAP_ZL - 1)) * ZREC);
  };
  auto y_ok = [&](const uint4 (&rv)[M], int32_t r) {
    const uint32_t tg = lap_tag(epoch, r);
    bool ok = true;
#pragma unroll
    for (int i = 0; i < M; ++i) ok = ok && rv[i].y == tg && rv[i].w == tg;
    return __all(ok) != 0;
  };
  auto z_ok = [&](int32_t rz) {
    const uint32_t tg = lap_tag(epoch, rz);
    bool ok = true;
    if (lane < 2 * NW) {
      const uint4 v = lds_read16(zring + (rz & (LAP_ZL - 1)) * ZREC + lane * 16);
      ok = v.y == tg && v.w == tg;
    }
    return __all(ok) != 0;
  };
  // slow path: re-fetch until the tags match (the producer has not stored yet)
  auto settle_z = [&](int32_t rz) {
    if (!zin || rz >= T_left) return;
    if (z_ok(rz)) return;
    ++n_stall;
    for (uint32_t spin = 0;; ++spin) {
      if (spin >= spin_limit) { fail(); return; }
      __builtin_amdgcn_s_sleep(1);
      fetch_z(rz);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (z_ok(rz)) return;
    }
  };

  // prologue (wave 0): z records ZT-2 and ZT-1 (what the shifts of steps -2 and
  // -1 would have brought into position 0: its Iz/Iyz inputs of step 0 and its
  // Ixz/M inputs of steps 0 and 1) and ZT .. ZT+ZV-1 (the shifts before the
  // first check); then LPD steps of y and z fetches -- M + 1 DMAs per step,
  // always (dummy ones where there is no producer), so the per-step vmcnt count
  // is a constant
  if (w == 0) {
    if (lane < 4) bpw[lane] = 0;
    if (zin) {
      for (int rz = ZT - 2; rz < ZT + ZV; ++rz) fetch_z(rz);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int rz = ZT - 2; rz < ZT + ZV; ++rz) settle_z(rz);
    }
    for (int s = 0; s < LPD; ++s) {
      fetch_y(s);
      fetch_z(s + ZT + ZV);
    }
  }
  __syncthreads();
  if (zin) {  // position 0 before step 0 (tools/lap_emu.py: the same initial shifts)
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
  if (trace != nullptr) stamp(1, now());
  const uint4 face = make_uint4(pa.f_single, pa.f_pair, pa.f_pair, 0u);
  uint32_t a_nx[M];
  load_a<M>(a_lane, a_nx);

  // ROLE: 0 = wave 0, 1 = middle waves, 2 = the last wave (NW >= 2)
  auto step = [&](auto ph, auto role, int32_t t, auto fin_step) {
    constexpr int PH = decltype(ph)::value;
    constexpr int ROLE = decltype(role)::value;
    constexpr bool FIN = decltype(fin_step)::value;
    uint32_t a[M];
#pragma unroll
    for (int i = 0; i < M; ++i) a[i] = a_nx[i];
    load_a<M>(a_lane + 4u * (uint32_t)(t + 1), a_nx);  // lands by the step barrier
    // ---- the row above of both halves
    uint32_t Ry[M], Rxy[M], Ryz[M], Rb[M];
    if constexpr (ROLE == 0) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((M + 1) * (LPD - 1)) : "memory");
      if (yin) {
        const int32_t r = t + YOFF;
        uint4 rv[M];
        const uint8_t *src = xr0 + (t % LPD) * SLOT + lane * REC_BYTES;
#pragma unroll
        for (int i = 0; i < M; ++i) rv[i] = lds_read16(src + i * PAIR);
        if (r < T_above && !y_ok(rv, r)) {
          ++n_stall;
          for (uint32_t spin = 0;; ++spin) {
            if (spin >= spin_limit) { fail(); break; }
            __builtin_amdgcn_s_sleep(1);
            fetch_y(t);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < M; ++i) rv[i] = lds_read16(src + i * PAIR);
            if (y_ok(rv, r)) break;
          }
        }
        // tagged record {Iy.hi | Ixy.hi << 16, tag, Iyz.hi | best.hi << 16, tag}
#pragma unroll
        for (int i = 0; i < M; ++i) {
          Ry[i] = perm(pIy[i], rv[i].x, 0x05040100u);
          Rxy[i] = perm(pIxy[i], rv[i].x, 0x05040302u);
          Ryz[i] = perm(pIyz[i], rv[i].z, 0x05040100u);
          Rb[i] = perm(pBest[i], rv[i].z, 0x05040302u);
        }
      } else {  // y = 0 face above row 1
#pragma unroll
        for (int i = 0; i < M; ++i) {
          Ry[i] = rows2(pIy[i], face.x);
          Rxy[i] = rows2(pIxy[i], face.y);
          Ryz[i] = rows2(pIyz[i], face.z);
          Rb[i] = rows2(pBest[i], face.w);
        }
      }
      settle_z(t + ZT + ZV);  // the z record all waves shift in ZV steps from now
    } else {  // the record wave w-1 wrote SK steps ago
      const uint8_t *src = xr + ((w - 1) * NSL + ((t + NSL - SK) & (NSL - 1))) * SLOT + lane * REC_BYTES;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const uint4 rv = lds_read16(src + i * PAIR);
        Ry[i] = rows2(pIy[i], rv.x);
        Rxy[i] = rows2(pIxy[i], rv.y);
        Ryz[i] = rows2(pIyz[i], rv.z);
        Rb[i] = rows2(pBest[i], rv.w);
      }
    }
    uint32_t inIx[M], inIy[M], inIz[M], inIxy[M], inIyz[M], inIxz[M], inM[M];
#pragma unroll
    for (int i = 0; i < M; ++i) {
      inIx[i] = oIx[i];
      inIy[i] = Ry[i];
      inIz[i] = shIz[i];
      inIxy[i] = svIxy[i];
      inIyz[i] = svIyz[i];
      inIxz[i] = shIxz[PH][i];
      inM[i] = svM[PH][i];
    }
    // ---- x = 1: low half at position t - 2w, high half one position behind;
    // their x - 1 inputs are the x = 0 face (src/PE_1cyc.v:164-178,196-218)
    const int32_t klo = __builtin_amdgcn_readfirstlane(t - WO * w);  // uniform: SGPR lane masks
    if (klo >= 0 && klo <= ZT) {
      const int32_t khi = klo - 1;
      const uint64_t lm_lo = sgpr64(klo < ZT ? 1ull << (klo / M) : 0ull);
      const uint64_t lm_hi = sgpr64(khi >= 0 ? 1ull << (khi / M) : 0ull);
      const int32_t ilo = klo % M, ihi = (khi + M) % M;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (M == 1 || i == ilo || i == ihi) {
          uint32_t m1;
          if constexpr (M == 1) {  // lanes klo and klo - 1 are different lanes
            uint32_t mh;
            asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(mh) : "v"(mhi), "s"(lm_hi));
            asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(m1) : "v"(mh), "v"(mlo), "s"(lm_lo));
          } else {  // M >= 2: one register gets at most one of the two halves
            const uint64_t lm = i == ilo ? lm_lo : lm_hi;
            const uint32_t hm = i == ilo ? mlo : mhi;
            asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(m1) : "v"(hm), "s"(lm));
          }
          inIx[i] = vbfi(m1, fsv, inIx[i]);
          inIxy[i] = vbfi(m1, fpv, inIxy[i]);
          inIxz[i] = vbfi(m1, fpv, inIxz[i]);
          inM[i] = vbfi(m1, 0u, inM[i]);
        }
      }
    }
    uint32_t oIy[M], oIxy[M], oIyz[M], oBest[M], oIz[M], oIxz[M], nIx[M];
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (F16)
      cell_messages_f16<M, SOP>(a, bv, c, SBC, K, DMC, Q, pa, inIx, inIy, inIz, inIxy, inIyz, inIxz,
                                inM, nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
    else
      cell_messages<M, SOP ? 1 : 0>(a, bv, c, Q, pv, inIx, inIy, inIz, inIxy, inIyz, inIxz, inM,
                                    nIx, oIy, oIz, oIxy, oIyz, oIxz, oBest);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (FIN) {  // the final cell (src/TriAlign_1cyc.v:141-142,342-345)
      if (final_wg && w == (r_f >> 1)) {  // row r_f: half r_f & 1 of wave r_f / 2
#pragma unroll
        for (int i = 0; i < M; ++i) fin[i * 64 + lane] = oBest[i];
      }
    }
    // ---- z staging: this wave's last position (lane 63, register M-1)
    if (zout && lane == 63)
      lds_write16(zst + ((t & 3) * NW + w) * 16,
                  make_uint4(oIz[M - 1], oIxz[M - 1], Ryz[M - 1], Rb[M - 1]));
    // ---- records: to the wave below, or (last wave) the y ring and z ring
    if constexpr (ROLE != 2) {
      uint8_t *dst = xr + (w * NSL + (t & (NSL - 1))) * SLOT + lane * REC_BYTES;
#pragma unroll
      for (int i = 0; i < M; ++i)
        lds_write16(dst + i * PAIR, make_uint4(oIy[i], oIxy[i], oIyz[i], oBest[i]));
    } else {
      if (yout) {
        wait_consumer(cons_y, seen_y, bpw, t - YR - YOFF);
        const uint32_t tg = lap_tag(epoch, t);
#pragma unroll
        for (int i = 0; i < M; ++i)
          store16_sc1(yf_mine + ((int64_t)(t & (YR - 1)) * M + i) * PAIR + lane * REC_BYTES,
                      make_uint4(perm(oIxy[i], oIy[i], 0x07060302u), tg,
                                 perm(oBest[i], oIyz[i], 0x07060302u), tg));
      }
      if (zout && t >= SK) {  // z record of step t-SK: complete in LDS since the last barrier
        const int32_t s = t - SK;
        wait_consumer(cons_z, seen_z, bpw + 1, s - ZR - ZT - ZV);
        if (lane < 2 * NW) {
          const uint32_t tg = lap_tag(epoch, s);
          const uint4 v = lds_read16(zst + ((s & 3) * NW + (lane >> 1)) * 16);
          const uint4 o = (lane & 1) ? make_uint4(v.z, tg, v.w, tg) : make_uint4(v.x, tg, v.y, tg);
          store16_sc1(zf_mine + (int64_t)(s & (ZR - 1)) * ZREC + lane * 16, o);
        }
      }
      if ((t & 7) == 0 && lane == 0) {  // refresh the consumers' progress words
        if (yout) dma4(prog + cons_y * LAP_PROG_STRIDE, bpw);
        if (zout) dma4(prog + cons_z * LAP_PROG_STRIDE, bpw + 1);
      }
    }
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
    // position 0's z-1 neighbour: the z = 0 face, or the left tile's record t + ZT
    uint32_t fIz = pa.f_single, fIxz = pa.f_pair, fIyz = pa.f_pair, fM = 0u;
    if (zin) {
      const uint8_t *zr = zring + ((t + ZT) & (LAP_ZL - 1)) * ZREC + w * LAP_ZREC_WAVE;
      const uint4 z0 = lds_read16(zr), z1 = lds_read16(zr + 16);
      fIz = z0.x;
      fIxz = z0.z;
      fIyz = z1.x;
      fM = z1.z;
    }
    zshift<M>(shIxz[PH], oIxz, sel0, fIxz);
    zshift<M>(shIz, oIz, sel0, fIz);
    zshift<M>(svIyz, Ryz, sel0, fIyz);
    zshift<M>(svM[PH], Rb, sel0, fM);
    if constexpr (ROLE == 0) {
      fetch_y(t + LPD);
      fetch_z(t + LPD + ZT + ZV);
    }
    // progress of this workgroup as a consumer: by the last barrier (t-1 is
    // odd) wave 0 had landed and checked the y records <= (t-1) + YOFF and the z
    // records <= (t-1) + ZT + ZV; published as t (decoded: step t-1 complete)
    if constexpr (ROLE == 1) {
      if (w == 1 && (t & (LAP_PUB - 1)) == 0 && lane == 0 && (yin || zin))
        __hip_atomic_store(prog + lid * LAP_PROG_STRIDE, (int32_t)((ep19 << 13) | (uint32_t)t),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (SK == 1 || PH == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto run = [&](auto role) {  // the last step peeled off (it records the final cell)
    int32_t t = 0;
    const int32_t T1 = T - 1;
    constexpr std::integral_constant<int, 0> P0{};
    constexpr std::integral_constant<int, 1> P1{};
    constexpr std::false_type mid{};
    constexpr std::true_type last{};
#pragma unroll 1
    for (; t + 1 < T1; t += 2) {
      LAP_INLINE(step(P0, role, t, mid));
      LAP_INLINE(step(P1, role, t + 1, mid));
    }
    if (t < T1) {
      LAP_INLINE(step(P0, role, t, mid));
      LAP_INLINE(step(P1, role, t + 1, last));
    } else {
      LAP_INLINE(step(P0, role, t, last));
    }
  };
  static_assert(NW >= 2, "wave 1 publishes the progress");
  if (w == 0) LAP_INLINE(run(std::integral_constant<int, 0>{}));
  else if (w == NW - 1) LAP_INLINE(run(std::integral_constant<int, 2>{}));
  else LAP_INLINE(run(std::integral_constant<int, 1>{}));
  if (trace != nullptr) {
    stamp(2, now());
    if (threadIdx.x == 0) {
      trace[(int64_t)b * 8 + 4] = n_stall;
      trace[(int64_t)b * 8 + 5] = n_bp;
    }
  }
  // the z records of the last SK steps and the final cell: staged before this barrier
  __syncthreads();
  if (w == NW - 1 && zout && lane < 2 * NW) {
    for (int32_t s = max(T - SK, 0); s < T; ++s) {
      wait_consumer(cons_z, seen_z, bpw + 1, s - ZR - ZT - ZV);
      const uint32_t tg = lap_tag(epoch, s);
      const uint4 v = lds_read16(zst + ((s & 3) * NW + (lane >> 1)) * 16);
      const uint4 o = (lane & 1) ? make_uint4(v.z, tg, v.w, tg) : make_uint4(v.x, tg, v.y, tg);
      store16_sc1(zf_mine + (int64_t)(s & (ZR - 1)) * ZREC + lane * 16, o);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (final_wg && threadIdx.x == 0) {
    const int32_t kf = k_f, hf = r_f & 1;
    const uint32_t v = fin[(kf % M) * 64 + kf / M];
    const uint16_t hb = (uint16_t)(hf ? (v >> 16) : (v & 0xFFFF));
    // a timed-out hand-off anywhere upstream invalidates the score (every
    // workgroup of the triple precedes this one): report it in-band
    const bool bad = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
    scores[tri] = bad ? TSA_SCORE_INVALID
                      : F16 ? (int32_t)(float)__builtin_bit_cast(_Float16, hb) : (int32_t)(int16_t)hb;
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

// Workgroups of one instantiation a CU holds, from the HIP occupancy API on the
// real kernel (VGPRs, LDS); without a device, the LDS / wave-slot model.
template <int M, int NW, bool F16, bool SOP>
static int lap_blocks_per_cu_t(size_t lds) {
  int nb = 0;
  int dev = -1;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lap_kernel<M, NW, F16, SOP>, 64 * NW,
                                                   lds) == hipSuccess)
    return nb;
  return (int)std::min<size_t>(LDS_MAX / std::max<size_t>(lds, 1), 32 / NW);
}
#define TSA_LAP_SHAPES(FN, M_, NW_, F16_, SOP_, ...)                                          \
  ((M_) == 1 ? ((NW_) == 4 ? TSA_ARITH(FN, 1, 4, F16_, SOP_, __VA_ARGS__)                      \
                           : TSA_ARITH(FN, 1, 8, F16_, SOP_, __VA_ARGS__))                     \
   : (M_) == 2 ? ((NW_) == 4 ? TSA_ARITH(FN, 2, 4, F16_, SOP_, __VA_ARGS__)                    \
                             : TSA_ARITH(FN, 2, 8, F16_, SOP_, __VA_ARGS__))                   \
               : ((NW_) == 4 ? TSA_ARITH(FN, 4, 4, F16_, SOP_, __VA_ARGS__)                    \
                             : TSA_ARITH(FN, 4, 8, F16_, SOP_, __VA_ARGS__)))

// Step time (us) along the chain, fitted to single-cube runs on MI355X
// (scripts/gpu_lap.sh): 64^3..512^3 with one workgroup per CU
// give 0.48-0.56 (M = 1), 0.62-0.67 (M = 2), 0.81 (M = 4); 1024^3 with 2-4
// workgroups per CU 0.84-0.87 -- the chain steps include the hand-off stalls.
static double lap_step_us(int M, int NW, int64_t wg_per_cu) {
  const double base = M == 1 ? (NW == 4 ? 0.50 : 0.52) : M == 2 ? 0.65 : 0.82;
  return base * (1.0 + 0.22 * (double)(std::max<int64_t>(wg_per_cu, 1) - 1));
}

LapGeom lap_geom(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, int M, int NW,
                 bool full_rings, bool f16, bool sop) {
  LapGeom g{};
  g.M = M;
  g.NW = NW;
  const int RW = 2 * NW, ZT = 64 * M, LPD = lap_pd(M);
  g.G = (max_lb + RW - 1) / RW;
  g.GZ = (max_lc + ZT - 1) / ZT;
  g.NC = n * g.GZ;             // columns: (triple, z-tile)
  g.CH = (g.NC + 7) / 8;       // columns per XCD
  const int YOFF = (LAP_SK + 1) * (NW - 1) + 1;  // lap lag of a record (kernel: YOFF)
  const int32_t T = max_la + YOFF + ZT;  // >= every workgroup's step count
  auto pow2 = [](int64_t v) { int64_t p = 1; while (p < v) p <<= 1; return (int32_t)p; };
  g.YR = full_rings ? pow2(T) : pow2(YOFF + LPD + 48);
  g.ZR = full_rings ? pow2(T) : pow2(ZT + LPD + 48);
  g.lds = lap_lds_bytes(M, NW, max_la);
  if (const char *e = getenv("TSA_LAP_LDS_EXTRA")) g.lds += (size_t)atoi(e);  // diagnostic knob
  const int64_t wgs = (int64_t)n * g.G * g.GZ;
  g.blocks = (int64_t)g.G * g.CH * 8;
  g.prog_bytes = (((size_t)wgs * LAP_PROG_STRIDE + 64) * sizeof(int32_t) + 255) & ~(size_t)255;
  g.yf_bytes = (size_t)wgs * g.YR * M * 1024;
  g.zf_bytes = (size_t)wgs * g.ZR * NW * LAP_ZREC_WAVE;
  if (g.lds > LDS_MAX || g.blocks > 0x7FFFFFFF) return g;
  const int per_cu = TSA_LAP_SHAPES(lap_blocks_per_cu_t, M, NW, f16, sop, g.lds);
  const int cus = dev_info().cus;
  // residency per XCD: column c (all its laps) lands on XCD c % 8
  const int64_t wg_per_xcd = (int64_t)g.G * g.CH;
  const int64_t slots_xcd = (int64_t)std::max(1, cus / 8) * per_cu;
  g.per_cu = per_cu;
  g.waves = per_cu > 0 ? std::max<int64_t>((wg_per_xcd + slots_xcd - 1) / slots_xcd,
                                           (wgs + (int64_t)cus * per_cu - 1) / ((int64_t)cus * per_cu))
                       : 0;
  g.ok = per_cu > 0 && (g.G >= 2 || g.GZ >= 2);
  // estimated latency (us): the chain to the final workgroup -- each lap adds
  // YOFF + LPD + ~3 steps, each tile ZT + LPD + ~2 -- plus its own steps;
  // several workgroups on one CU share its SIMDs. A grid beyond the resident
  // slots runs in dispatch waves that barely overlap (~2.8x per wave).
  const int64_t xcd_cus = std::max(1, cus / 8);
  const int64_t wg_cu = std::max<int64_t>(1, std::min<int64_t>(per_cu, (wg_per_xcd + xcd_cus - 1) / xcd_cus));
  const double steps = (double)(g.G - 1) * (YOFF + LPD + 3) + (double)(g.GZ - 1) * (ZT + LPD + 2) +
                       (double)(max_la + YOFF + ZT);
  const double chain = steps * lap_step_us(M, NW, wg_cu);
  g.est_us = g.waves <= 1 ? chain : 2.8 * (double)g.waves * chain;
  return g;
}

size_t lap_workspace_bytes(const LapGeom &g) { return g.prog_bytes + g.yf_bytes + g.zf_bytes; }

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

template <int M, int NW, bool F16, bool SOP>
static int launch_lap(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                      const LapGeom &g, int32_t *d_scores, void *d_ws, const PencilArgs &pa,
                      hipStream_t stream) {
  auto kfn = lap_kernel<M, NW, F16, SOP>;
  if (g.lds > LDS_MAX) return TSA_EINVAL;
  if (hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)g.lds) != hipSuccess)
    return TSA_EDEVICE;
  int32_t *prog = (int32_t *)d_ws;
  const int64_t wgs = (int64_t)n * g.G * g.GZ;
  uint32_t *err = (uint32_t *)(prog + wgs * LAP_PROG_STRIDE);
  uint8_t *yf = (uint8_t *)d_ws + g.prog_bytes;
  uint8_t *zf = yf + g.yf_bytes;
  unsigned long long *trace = nullptr;
  const char *tpath = getenv("TSA_LAP_TRACE");  // diagnostic: per-WG timestamps to a CSV file
  if (tpath && hipMalloc(&trace, (size_t)g.blocks * 8 * 8) != hipSuccess) return TSA_ENOMEM;
  if (trace && hipMemsetAsync(trace, 0, (size_t)g.blocks * 8 * 8, stream) != hipSuccess)
    return TSA_EDEVICE;
  const uint32_t epoch = lap_next_epoch();
  hipLaunchKernelGGL(kfn, dim3((uint32_t)g.blocks), dim3(64 * NW), g.lds, stream, d_seqs,
                     d_offsets, g.G, g.GZ, g.NC, g.CH, g.YR, g.ZR, yf, zf, prog, err, d_scores, pa, epoch,
                     lap_spin_limit(), trace);
  if (hipGetLastError() != hipSuccess) return TSA_EDEVICE;
  if (trace) {
    std::vector<unsigned long long> h((size_t)g.blocks * 8);
    if (hipMemcpyAsync(h.data(), trace, h.size() * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
      return TSA_EDEVICE;
    (void)hipFree(trace);
    if (FILE *fp = fopen(tpath, "w")) {
      fprintf(fp, "block,tri,lap,tile,start,loop_begin,loop_end,xcc,stalls,bp_waits\n");
      for (int64_t b = 0; b < g.blocks; ++b) {
        if (h[b * 8] == 0) continue;  // padding block
        const int64_t slot = b >> 3, col = (slot % g.CH) * 8 + (b & 7);
        fprintf(fp, "%lld,%lld,%lld,%lld,%llu,%llu,%llu,%llu,%llu,%llu\n", (long long)b,
                (long long)(col / g.GZ), (long long)(slot / g.CH), (long long)(col % g.GZ), h[b * 8],
                h[b * 8 + 1], h[b * 8 + 2], h[b * 8 + 3], h[b * 8 + 4], h[b * 8 + 5]);
      }
      fclose(fp);
    }
  }
  return TSA_OK;
}

int lap_launch(const LapGeom &g, bool f16, bool sop, const uint8_t *d_seqs,
               const int64_t *d_offsets, int32_t n, int32_t *d_scores, void *d_ws,
               const PencilArgs &pa, hipStream_t stream, int32_t **d_err) {
  if (d_err) {  // synchronous caller: clear the error word, it reads it back
    *d_err = (int32_t *)d_ws + (int64_t)n * g.G * g.GZ * LAP_PROG_STRIDE;
    if (hipMemsetAsync(*d_err, 0, sizeof(int32_t), stream) != hipSuccess) return TSA_EDEVICE;
  }
  return TSA_LAP_SHAPES(launch_lap, g.M, g.NW, f16, sop, d_seqs, d_offsets, n, g, d_scores, d_ws,
                        pa, stream);
}

}  // namespace tsa
