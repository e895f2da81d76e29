// plane_kernel.hip -- TSA_KERNEL_PLANE: anti-diagonal plane sweep with the
// RTL's literal arithmetic (49 candidates per cell, each wrapped to
// SCORE_BITS before the 7-way max), one launch per plane q = x+y+z.
//
// Reference: the recurrence is src/PE_1cyc.v:159-218 (candidates),
// src/PE_1cyc.v:1-32 (MAX7), zero faces src/PE_1cyc.v:164-218 (x=0 gating) and
// src/TriAlign_1cyc.v:155-182 (y=0 / z=0 / corner), final MAX7
// src/TriAlign_1cyc.v:141-142. The RTL's slicing (8x8 pencils + y/z face
// SRAMs, src/TriAlign_1cyc.v:78-98,127-140) becomes a ring of four (y,z)
// planes per triple in HBM: O(N^2) memory for an N^3 cube.
//
// HBM layout per triple: int16 ws[slot 0..3][state 0..6][y 0..max_lb][ldz];
// entry (y,z) of the plane in slot q&3 is cell (q-y-z, y, z). Rows y=0 and
// columns z=0 are zeroed once per call (faces); the x=0 entry of each plane is
// zeroed by that plane's own launch; entries with x>LA are never read.
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

PlaneLayout plane_layout(int32_t max_lb, int32_t max_lc) {
  PlaneLayout L;
  L.ldz = plane_ldz(max_lc);
  L.plane = (int64_t)(max_lb + 1) * L.ldz;
  L.per_triple = 4 * NSTATE * L.plane;
  return L;
}

size_t plane_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  (void)max_la;
  const PlaneLayout L = plane_layout(max_lb, max_lc);
  return (size_t)n * (size_t)L.per_triple * sizeof(int16_t);
}

// Zero the y=0 row and z=0 column of all 28 state-planes of every triple.
__global__ __launch_bounds__(256) void plane_face_init(int16_t *__restrict__ ws, PlaneLayout L,
                                                       int32_t max_lb) {
  const int64_t t = blockIdx.y;
  int16_t *base = ws + t * L.per_triple;
  const int64_t nrow = L.ldz, ncol = max_lb + 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 4 * NSTATE * (nrow + ncol);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sp = i / (nrow + ncol), k = i % (nrow + ncol);
    int16_t *pl = base + sp * L.plane;
    if (k < nrow) pl[k] = 0;               // row y = 0
    else pl[(k - nrow) * L.ldz] = 0;       // column z = 0
  }
}

__device__ __forceinline__ int32_t wrapv(int32_t v, int32_t sh) { return (v << sh) >> sh; }

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

// Traceback pointer cube index of cell (x,y,z), 1-based: [y-1][x+z-2][z-1].
__host__ __device__ inline int64_t tb_index(int32_t x, int32_t y, int32_t z, int32_t la,
                                            int32_t lc) {
  return ((int64_t)(y - 1) * (la + lc - 1) + (x + z - 2)) * lc + (z - 1);
}

// One launch = plane q of every triple (blockIdx.z). Thread (j, r) of block
// (bx, by) owns row y = ylo + 4*by + r and column z = zlo(y) + 64*bx + j; the
// 64 lanes of a wave read 64 consecutive z of each predecessor row.
template <bool TB>
__global__ __launch_bounds__(256) void plane_step_kernel(
    const uint8_t *__restrict__ seqs, const int64_t *__restrict__ offs, int32_t q,
    int16_t *__restrict__ ws, PlaneLayout L, KParams kp, int32_t *__restrict__ scores,
    int32_t *__restrict__ final7, uint32_t *__restrict__ tb) {
  const int64_t t = blockIdx.z;
  const int64_t o0 = offs[3 * t], o1 = offs[3 * t + 1], o2 = offs[3 * t + 2], o3 = offs[3 * t + 3];
  const int32_t la = (int32_t)(o1 - o0), lb = (int32_t)(o2 - o1), lc = (int32_t)(o3 - o2);
  if (q > la + lb + lc) return;
  const int32_t ylo = max(1, q - la - lc), yhi = min(lb, q - 1);
  const int32_t y = ylo + (int32_t)blockIdx.y * 4 + (int32_t)threadIdx.y;
  if (y > yhi) return;
  const int32_t zlo = max(1, q - la - y), zend = min(lc, q - y);
  const int32_t z = zlo + (int32_t)blockIdx.x * 64 + (int32_t)threadIdx.x;
  if (z > zend) return;
  const int32_t x = q - y - z;

  int16_t *base = ws + t * L.per_triple;
  const int64_t P = L.plane;
  int16_t *out = base + (int64_t)(q & 3) * NSTATE * P + (int64_t)y * L.ldz + z;
  if (x == 0) {  // the x=0 face entry of this plane (EN_i==1&&EN==0 gating)
#pragma unroll
    for (int s = 0; s < NSTATE; ++s) out[s * P] = 0;
    return;
  }
  const int16_t *q1 = base + (int64_t)((q - 1) & 3) * NSTATE * P;
  const int16_t *q2 = base + (int64_t)((q - 2) & 3) * NSTATE * P;
  const int16_t *q3 = base + (int64_t)((q - 3) & 3) * NSTATE * P;
  const int64_t c00 = (int64_t)y * L.ldz + z;          // (y,  z  )
  const int64_t cm0 = c00 - L.ldz, c0m = c00 - 1;      // (y-1,z  ), (y,  z-1)
  const int64_t cmm = cm0 - 1;                         // (y-1,z-1)

  int32_t pM[7], pX[7], pY[7], pZ[7], pXY[7], pYZ[7], pXZ[7];
#pragma unroll
  for (int s = 0; s < NSTATE; ++s) {
    pM[s] = q3[s * P + cmm];   // (x-1,y-1,z-1)  M    src/PE_1cyc.v:164-170
    pX[s] = q1[s * P + c00];   // (x-1,y,  z  )  Ix   :172-178
    pY[s] = q1[s * P + cm0];   // (x,  y-1,z  )  Iy   :180-186
    pZ[s] = q1[s * P + c0m];   // (x,  y,  z-1)  Iz   :188-194
    pXY[s] = q2[s * P + cm0];  // (x-1,y-1,z  )  Ixy  :196-202
    pYZ[s] = q2[s * P + cmm];  // (x,  y-1,z-1)  Iyz  :204-210
    pXZ[s] = q2[s * P + c0m];  // (x-1,y,  z-1)  Ixz  :212-218
  }
  const int a = tsa_sym(seqs, o0 + x - 1, kp.packed), b = tsa_sym(seqs, o1 + y - 1, kp.packed),
            c = tsa_sym(seqs, o2 + z - 1, kp.packed);
  const int32_t sh = kp.wrap_shift;
  const int32_t sab = (a == b) ? kp.match : kp.mismatch;
  const int32_t sbc = (b == c) ? kp.match : kp.mismatch;
  const int32_t sac = (a == c) ? kp.match : kp.mismatch;
  int32_t s3;
  if (kp.s3_mode == TSA_S3_SOP) s3 = wrapv(sab + sbc + sac, sh);
  else s3 = (a == b) ? ((b == c) ? kp.s3_eq : kp.s3_ab) : kp.s3_ne;

  int32_t S[7];
  uint32_t g[7];
  S[SM] = max7_literal<SM, TB>(pM, kp, s3, sh, g[SM]);
  S[SIX] = max7_literal<SIX, TB>(pX, kp, 0, sh, g[SIX]);
  S[SIY] = max7_literal<SIY, TB>(pY, kp, 0, sh, g[SIY]);
  S[SIZ] = max7_literal<SIZ, TB>(pZ, kp, 0, sh, g[SIZ]);
  S[SIXY] = max7_literal<SIXY, TB>(pXY, kp, sab, sh, g[SIXY]);
  S[SIYZ] = max7_literal<SIYZ, TB>(pYZ, kp, sbc, sh, g[SIYZ]);
  S[SIXZ] = max7_literal<SIXZ, TB>(pXZ, kp, sac, sh, g[SIXZ]);
#pragma unroll
  for (int s = 0; s < NSTATE; ++s) out[s * P] = (int16_t)S[s];
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
  int16_t *ws = (int16_t *)d_ws;
  hipLaunchKernelGGL(plane_face_init, dim3(8, n), dim3(256), 0, stream, ws, L, max_lb);
  const int32_t qmax = max_la + max_lb + max_lc;
  const int32_t wmax = (max_la < max_lc ? max_la : max_lc) + 1;
  const dim3 block(64, 4);
  for (int32_t q = 2; q <= qmax; ++q) {
    const int32_t rows = (max_lb < q - 1 ? max_lb : q - 1);
    const dim3 grid((wmax + 63) / 64, (rows + 3) / 4, n);
    if (d_tb)
      hipLaunchKernelGGL(plane_step_kernel<true>, grid, block, 0, stream, d_seqs, d_offsets, q, ws,
                         L, kp, d_scores, d_final7, d_tb);
    else
      hipLaunchKernelGGL(plane_step_kernel<false>, grid, block, 0, stream, d_seqs, d_offsets, q,
                         ws, L, kp, d_scores, d_final7, nullptr);
  }
  return hipGetLastError() == hipSuccess ? TSA_OK : TSA_EDEVICE;
}

}  // namespace tsa
