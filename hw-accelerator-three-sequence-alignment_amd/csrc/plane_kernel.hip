// plane_kernel.hip -- TSA_KERNEL_PLANE: anti-diagonal plane sweep with the
// RTL's literal arithmetic (49 candidates per cell, each wrapped to
// SCORE_BITS before the 7-way max), one launch per plane q = x+y+z, the
// predecessor planes staged in LDS tiles.
//
// Reference: the recurrence is src/PE_1cyc.v:159-218 (candidates),
// src/PE_1cyc.v:1-32 (MAX7), zero faces src/PE_1cyc.v:164-218 (x=0 gating) and
// src/TriAlign_1cyc.v:155-182 (y=0 / z=0 / corner), final MAX7
// src/TriAlign_1cyc.v:141-142. The RTL's slicing (8x8 pencils + y/z face
// SRAMs, src/TriAlign_1cyc.v:78-98,127-140) becomes a ring of four (y,z)
// planes per triple in HBM: O(N^2) memory for an N^3 cube.
//
// HBM layout per triple: cells ws[slot 0..3][y 0..max_lb][z 0..max_lc], a cell
// = the 7 int16 states {M,Ix,Iy,Iz,Ixy,Iyz,Ixz} + a pad (16 bytes); entry (y,z)
// of the plane in slot q&3 is cell (q-y-z, y, z). Rows y=0 and columns z=0 are
// zeroed once per call (faces); the x=0 entry of each plane is zeroed by that
// plane's own launch; entries with x>LA are never read.
//
// A workgroup takes a TY x 64 tile (rows y0..y0+TY-1, columns z0..z0+63) of
// plane q: it stages the tile plus a one-row / one-column halo of planes q-1,
// q-2 and q-3 -- every predecessor its cells need -- in LDS with coalesced
// 16-byte loads (3 (TY+1) 65 cells, ~4 loads per thread instead of 49 2-byte
// gathers per cell); each cell reads its own column's 5 predecessors from LDS
// and takes the 4 at z-1 from its left lane by DPP (a wave = one tile row).
//
// This kernel is the exact path for every parameter set and length (the
// pencil kernel's factored arithmetic is exact only when nothing wraps).
//
// Traceback (tsa_align_gpu, an extension: the reference's alignment-output
// ports are commented out, src/TriAlign_tb.sv:239-260): the TB instantiation
// also stores, per cell, which source state won each of the 7 MAX7s (3 bits
// each, lowest state index on ties) in a pointer cube tb[y][x+z][z] -- for a
// wave (fixed y and q, consecutive z) x+z is fixed, so the stores coalesce --
// and tb_walk follows the pointers back from cell (LA,LB,LC).

#include "tsa_internal.h"

namespace tsa {

constexpr int PLANE_TY = 4;                   // rows per tile (block = 64 x TY)
constexpr int PLANE_TW = 65;                  // staged columns per row: z0-1 .. z0+63
constexpr int PLANE_TILE = (PLANE_TY + 1) * PLANE_TW;  // staged cells per predecessor plane

PlaneLayout plane_layout(int32_t max_lb, int32_t max_lc) {
  PlaneLayout L;
  L.ldz = plane_ldz(max_lc);
  L.plane = (int64_t)(max_lb + 1) * L.ldz;
  L.per_triple = 4 * L.plane;
  return L;
}

size_t plane_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  (void)max_la;
  const PlaneLayout L = plane_layout(max_lb, max_lc);
  return (size_t)n * (size_t)L.per_triple * sizeof(uint4);
}

// Zero the y=0 row and z=0 column of all 4 planes of every triple.
__global__ __launch_bounds__(256) void plane_face_init(uint4 *__restrict__ ws, PlaneLayout L,
                                                       int32_t max_lb) {
  const int64_t t = blockIdx.y;
  uint4 *base = ws + t * L.per_triple;
  const int64_t nrow = L.ldz, ncol = max_lb + 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 4 * (nrow + ncol);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sp = i / (nrow + ncol), k = i % (nrow + ncol);
    uint4 *pl = base + sp * L.plane;
    if (k < nrow) pl[k] = make_uint4(0u, 0u, 0u, 0u);               // row y = 0
    else pl[(k - nrow) * L.ldz] = make_uint4(0u, 0u, 0u, 0u);       // column z = 0
  }
}

__device__ __forceinline__ int32_t wrapv(int32_t v, int32_t sh) { return (v << sh) >> sh; }

// The 7 states of a staged cell, sign-extended.
__device__ __forceinline__ void unpack7(uint4 c, int32_t (&v)[7]) {
  v[0] = (int16_t)(c.x & 0xFFFF);
  v[1] = (int16_t)(c.x >> 16);
  v[2] = (int16_t)(c.y & 0xFFFF);
  v[3] = (int16_t)(c.y >> 16);
  v[4] = (int16_t)(c.z & 0xFFFF);
  v[5] = (int16_t)(c.z >> 16);
  v[6] = (int16_t)(c.w & 0xFFFF);
}

// Literal MAX7 of one target: max_s wrap(pred[s] - pen[s] + add). With TB,
// arg receives the lowest source index achieving it.
template <int T, bool TB>
__device__ __forceinline__ int32_t max7_literal(const int32_t (&pr)[7], const KParams &kp,
                                               int32_t add, int32_t sh, uint32_t &arg) {
  int32_t m = wrapv(pr[0] - kp.pen[T][0] + add, sh);
  uint32_t a = 0;
#pragma unroll
  for (int s = 1; s < 7; ++s) {
    const int32_t v = wrapv(pr[s] - kp.pen[T][s] + add, sh);
    if constexpr (TB) {
      if (v > m) a = s;
    }
    m = max(m, v);
  }
  arg = a;
  return m;
}

// The same MAX7 on packed int16 pairs (sources 0-1, 2-3, 4-5, 6-6): 2-4
// instructions per pair of candidates instead of 4-5 per candidate. Exact:
// int16 adds are mod 2^16 and SCORE_BITS <= 16, so wrapping their result to
// SCORE_BITS equals wrapping the int32 sum (with no wrap the host bound keeps
// every candidate inside int16). Returns the state in the low half.
typedef short s16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2_t, a) + __builtin_bit_cast(s16x2_t, b));
}
__device__ __forceinline__ uint32_t pk_max16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, a),
                                                                __builtin_bit_cast(s16x2_t, b)));
}
template <int T, bool WRAP, bool ADD>
__device__ __forceinline__ int32_t max7_packed(const uint32_t (&pr)[4], const KParams &kp,
                                              uint32_t add2, uint32_t sh2) {
  uint32_t u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u[i] = pk_add16(pr[i], kp.npen[T][i]);
    if constexpr (ADD) u[i] = pk_add16(u[i], add2);
    if constexpr (WRAP) {
      const s16x2_t sh = __builtin_bit_cast(s16x2_t, sh2);
      u[i] = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(s16x2_t, u[i]) << sh) >> sh);
    }
  }
  const uint32_t m = pk_max16(pk_max16(u[0], u[1]), pk_max16(u[2], u[3]));
  return max((int32_t)(int16_t)(m & 0xFFFF), (int32_t)(int16_t)(m >> 16));
}
// A staged cell as 4 pairs, source 6 duplicated into the pad half.
__device__ __forceinline__ void pairs7(uint4 c, uint32_t (&p)[4]) {
  p[0] = c.x;
  p[1] = c.y;
  p[2] = c.z;
  p[3] = (c.w & 0xFFFFu) * 0x00010001u;
}

// Lane l <- lane l-1 of a 16-byte cell (DPP wave_shr:1); lane 0 keeps `halo`.
__device__ __forceinline__ uint32_t shr1_u32(uint32_t v, uint32_t halo) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)halo, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint4 lane_shr1(uint4 v, uint4 halo) {
  return make_uint4(shr1_u32(v.x, halo.x), shr1_u32(v.y, halo.y), shr1_u32(v.z, halo.z), shr1_u32(v.w, halo.w));
}

// Traceback pointer cube index of cell (x,y,z), 1-based: [y-1][x+z-2][z-1].
__host__ __device__ inline int64_t tb_index(int32_t x, int32_t y, int32_t z, int32_t la,
                                            int32_t lc) {
  return ((int64_t)(y - 1) * (la + lc - 1) + (x + z - 2)) * lc + (z - 1);
}

// One launch = plane q of every triple (blockIdx.z). Block (bx, by) is the
// tile rows y0 = ylo + TY by .. y0+TY-1, columns z0 = zt + 64 bx .. z0+63, where
// zt is the first column any of its rows has on this plane; thread (j, r) owns
// cell (y0 + r, z0 + j) when that cell lies on the plane and in the cube.
template <bool TB, bool WRAP>
__global__ __launch_bounds__(64 * PLANE_TY) void plane_step_kernel(
    const uint8_t *__restrict__ seqs, const int64_t *__restrict__ offs, int32_t q,
    uint4 *__restrict__ ws, PlaneLayout L, KParams kp, int32_t *__restrict__ scores,
    int32_t *__restrict__ final7, uint32_t *__restrict__ tb) {
  __shared__ uint4 tile[3 * PLANE_TILE];  // [plane q-1-p][row y0-1+r][column z0-1+c]
  const int64_t t = blockIdx.z;
  const int64_t o0 = offs[3 * t], o1 = offs[3 * t + 1], o2 = offs[3 * t + 2], o3 = offs[3 * t + 3];
  const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
  if (q > la + lb + lc) return;
  const int32_t ylo = max(1, q - la - lc), yhi = min(lb, q - 1);
  const int32_t y0 = ylo + (int32_t)blockIdx.y * PLANE_TY;
  if (y0 > yhi) return;
  const int32_t zt = max(1, q - la - min(yhi, y0 + PLANE_TY - 1));  // first column of the tile's rows
  const int32_t z0 = zt + (int32_t)blockIdx.x * 64;
  if (z0 > min(lc, q - y0)) return;  // past the last column of the tile's first row

  uint4 *base = ws + t * L.per_triple;
  const int64_t P = L.plane;
  // ---- stage planes q-1, q-2, q-3: rows y0-1 .. y0+TY-1, columns z0-1 .. z0+63
  const int tid = threadIdx.y * 64 + threadIdx.x;
  for (int i = tid; i < 3 * PLANE_TILE; i += 64 * PLANE_TY) {
    const int pl = i / PLANE_TILE, rc = i % PLANE_TILE;
    const int32_t yy = y0 - 1 + rc / PLANE_TW, zz = z0 - 1 + rc % PLANE_TW;
    if (yy <= lb && zz <= lc)
      tile[i] = base[(int64_t)((q - 1 - pl) & 3) * P + (int64_t)yy * L.ldz + zz];
  }
  __syncthreads();

  const int32_t y = y0 + (int32_t)threadIdx.y, z = z0 + (int32_t)threadIdx.x;
  // A wave is one row of the tile (64 consecutive z): each lane reads its own
  // column of the staged planes, and the z-1 predecessors come from lane - 1
  // by DPP (wave_shr:1) -- lane 0 takes the staged halo column z0 - 1. Every
  // lane of the row reads before any returns: a lane whose own cell is off the
  // plane still hands its column to lane + 1.
  const int r = (int)threadIdx.y + 1, c = (int)threadIdx.x + 1;  // staged row / column of (y, z)
  const uint4 *T1 = tile, *T2 = tile + PLANE_TILE, *T3 = tile + 2 * PLANE_TILE;
  const uint4 cX = T1[r * PLANE_TW + c];             // (x-1,y,  z  )  Ix   src/PE_1cyc.v:172-178
  const uint4 cY = T1[(r - 1) * PLANE_TW + c];       // (x,  y-1,z  )  Iy   :180-186
  const uint4 cXY = T2[(r - 1) * PLANE_TW + c];      // (x-1,y-1,z  )  Ixy  :196-202
  const uint4 oXZ = T2[r * PLANE_TW + c];            // lane + 1's Ixz predecessor
  const uint4 oM = T3[(r - 1) * PLANE_TW + c];       // lane + 1's M predecessor
  uint4 hZ = make_uint4(0u, 0u, 0u, 0u), hYZ = hZ, hXZ = hZ, hM = hZ;
  if (threadIdx.x == 0) {  // the halo column
    hZ = T1[r * PLANE_TW];
    hYZ = T2[(r - 1) * PLANE_TW];
    hXZ = T2[r * PLANE_TW];
    hM = T3[(r - 1) * PLANE_TW];
  }
  const uint4 cZ = lane_shr1(cX, hZ);     // (x,  y,  z-1)  Iz   :188-194
  const uint4 cYZ = lane_shr1(cXY, hYZ);  // (x,  y-1,z-1)  Iyz  :204-210
  const uint4 cXZ = lane_shr1(oXZ, hXZ);  // (x-1,y,  z-1)  Ixz  :212-218
  const uint4 cM = lane_shr1(oM, hM);     // (x-1,y-1,z-1)  M    :164-170
  if (y > yhi || z < max(1, q - la - y) || z > min(lc, q - y)) return;
  const int32_t x = q - y - z;
  uint4 *out = base + (int64_t)(q & 3) * P + (int64_t)y * L.ldz + z;
  if (x == 0) {  // the x=0 face entry of this plane (EN_i==1&&EN==0 gating)
    *out = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  const int a = tsa_sym(seqs, o0 + x - 1, kp.packed), b = tsa_sym(seqs, o1 + y - 1, kp.packed),
            cc = tsa_sym(seqs, o2 + z - 1, kp.packed);
  const int32_t sh = kp.wrap_shift;
  const int32_t sab = (a == b) ? kp.match : kp.mismatch;
  const int32_t sbc = (b == cc) ? kp.match : kp.mismatch;
  const int32_t sac = (a == cc) ? kp.match : kp.mismatch;
  int32_t s3;
  if (kp.s3_mode == TSA_S3_SOP) s3 = wrapv(sab + sbc + sac, sh);
  else s3 = (a == b) ? ((b == cc) ? kp.s3_eq : kp.s3_ab) : kp.s3_ne;

  int32_t S[7];
  uint32_t g[7];
  if constexpr (TB) {  // literal int32 candidates with the argmax of each MAX7
    int32_t pM[7], pX[7], pY[7], pZ[7], pXY[7], pYZ[7], pXZ[7];
    unpack7(cM, pM);
    unpack7(cX, pX);
    unpack7(cY, pY);
    unpack7(cZ, pZ);
    unpack7(cXY, pXY);
    unpack7(cYZ, pYZ);
    unpack7(cXZ, pXZ);
    S[SM] = max7_literal<SM, TB>(pM, kp, s3, sh, g[SM]);
    S[SIX] = max7_literal<SIX, TB>(pX, kp, 0, sh, g[SIX]);
    S[SIY] = max7_literal<SIY, TB>(pY, kp, 0, sh, g[SIY]);
    S[SIZ] = max7_literal<SIZ, TB>(pZ, kp, 0, sh, g[SIZ]);
    S[SIXY] = max7_literal<SIXY, TB>(pXY, kp, sab, sh, g[SIXY]);
    S[SIYZ] = max7_literal<SIYZ, TB>(pYZ, kp, sbc, sh, g[SIYZ]);
    S[SIXZ] = max7_literal<SIXZ, TB>(pXZ, kp, sac, sh, g[SIXZ]);
  } else {  // packed int16 pairs
    const uint32_t sh2 = (uint32_t)(16 - kp.bits) * 0x00010001u;
    auto two = [](int32_t v) { return (uint32_t)(uint16_t)v * 0x00010001u; };
    uint32_t p[4];
    pairs7(cM, p);
    S[SM] = max7_packed<SM, WRAP, true>(p, kp, two(s3), sh2);
    pairs7(cX, p);
    S[SIX] = max7_packed<SIX, WRAP, false>(p, kp, 0u, sh2);
    pairs7(cY, p);
    S[SIY] = max7_packed<SIY, WRAP, false>(p, kp, 0u, sh2);
    pairs7(cZ, p);
    S[SIZ] = max7_packed<SIZ, WRAP, false>(p, kp, 0u, sh2);
    pairs7(cXY, p);
    S[SIXY] = max7_packed<SIXY, WRAP, true>(p, kp, two(sab), sh2);
    pairs7(cYZ, p);
    S[SIYZ] = max7_packed<SIYZ, WRAP, true>(p, kp, two(sbc), sh2);
    pairs7(cXZ, p);
    S[SIXZ] = max7_packed<SIXZ, WRAP, true>(p, kp, two(sac), sh2);
  }
  auto pk = [](int32_t lo, int32_t hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); };
  *out = make_uint4(pk(S[0], S[1]), pk(S[2], S[3]), pk(S[4], S[5]), pk(S[6], 0));
  if constexpr (TB) {  // one triple per traceback launch
    uint32_t w = 0;
#pragma unroll
    for (int s = 0; s < NSTATE; ++s) w |= g[s] << (3 * s);
    tb[tb_index(x, y, z, la, lc)] = w;
  }

  if (x == la && y == lb && z == lc) {  // FINAL_MAX, src/TriAlign_1cyc.v:141-142
    int32_t m = S[0];
#pragma unroll
    for (int s = 1; s < NSTATE; ++s) m = max(m, S[s]);
    scores[t] = m;
    if (final7) {
#pragma unroll
      for (int s = 0; s < NSTATE; ++s) final7[t * NSTATE + s] = S[s];
    }
  }
}

// Follow the pointers back from cell (la,lb,lc) (single thread; <= la+lb+lc
// dependent loads). moves[] gets the states from the end backwards; info =
// {moves, x0, y0, z0} where (x0,y0,z0) is the face cell the path leaves.
__global__ void tb_walk(const uint32_t *__restrict__ tb, const int32_t *__restrict__ final7,
                        int32_t la, int32_t lb, int32_t lc, uint8_t *__restrict__ moves,
                        int32_t *__restrict__ info) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  // final MAX7 (src/TriAlign_1cyc.v:141-142): lowest state index on ties
  int32_t T = 0;
  for (int s = 1; s < NSTATE; ++s)
    if (final7[s] > final7[T]) T = s;
  constexpr int DX[7] = {1, 1, 0, 0, 1, 0, 1}, DY[7] = {1, 0, 1, 0, 1, 1, 0},
                DZ[7] = {1, 0, 0, 1, 0, 1, 1};  // predecessor offsets per state
  int32_t x = la, y = lb, z = lc, n = 0;
  for (;;) {
    moves[n++] = (uint8_t)T;
    const int32_t px = x - DX[T], py = y - DY[T], pz = z - DZ[T];
    if (px == 0 || py == 0 || pz == 0 || n >= la + lb + lc) {
      x = px;
      y = py;
      z = pz;
      break;
    }
    T = (int32_t)((tb[tb_index(x, y, z, la, lc)] >> (3 * T)) & 7u);
    x = px;
    y = py;
    z = pz;
  }
  info[0] = n;
  info[1] = x;
  info[2] = y;
  info[3] = z;
}

size_t tb_cube_bytes(int32_t la, int32_t lb, int32_t lc) {
  return (size_t)lb * (size_t)(la + lc - 1) * (size_t)lc * sizeof(uint32_t);
}

int plane_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                       int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                       int32_t *d_scores, int32_t *d_final7, void *d_ws, size_t ws_bytes,
                       hipStream_t stream, uint32_t *d_tb) {
  if (n <= 0) return TSA_OK;
  if (n > 65535) return TSA_EINVAL;  // grid.z limit; callers chunk
  if (d_tb && n != 1) return TSA_EINVAL;  // traceback: one triple, exact lengths
  if (ws_bytes < plane_workspace_bytes(n, max_la, max_lb, max_lc)) return TSA_ENOMEM;
  const PlaneLayout L = plane_layout(max_lb, max_lc);
  uint4 *ws = (uint4 *)d_ws;
  hipLaunchKernelGGL(plane_face_init, dim3(8, n), dim3(256), 0, stream, ws, L, max_lb);
  const int32_t qmax = max_la + max_lb + max_lc;
  // a tile's rows span at most min(LA, LC) + TY columns of a plane
  const int32_t wmax = (max_la < max_lc ? max_la : max_lc) + PLANE_TY;
  const dim3 block(64, PLANE_TY);
  for (int32_t q = 2; q <= qmax; ++q) {
    const int32_t rows = (max_lb < q - 1 ? max_lb : q - 1);
    const dim3 grid((wmax + 63) / 64, (rows + PLANE_TY - 1) / PLANE_TY, n);
    // SCORE_BITS 1..15 wrap in the packed form; 16 is int16 itself; 0 never wraps
    const bool wrap = kp.bits > 0 && kp.bits < 16;
    if (d_tb)
      hipLaunchKernelGGL((plane_step_kernel<true, false>), grid, block, 0, stream, d_seqs, d_offsets,
                         q, ws, L, kp, d_scores, d_final7, d_tb);
    else if (wrap)
      hipLaunchKernelGGL((plane_step_kernel<false, true>), grid, block, 0, stream, d_seqs, d_offsets,
                         q, ws, L, kp, d_scores, d_final7, nullptr);
    else
      hipLaunchKernelGGL((plane_step_kernel<false, false>), grid, block, 0, stream, d_seqs, d_offsets,
                         q, ws, L, kp, d_scores, d_final7, nullptr);
  }
  return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
}

}  // namespace tsa
