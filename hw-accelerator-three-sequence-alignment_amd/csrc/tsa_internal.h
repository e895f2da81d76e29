// tsa_internal.h -- shared host/device definitions of the TriAlign MI355X
// library (not part of the C-ABI; see include/trialign.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/trialign.h"

namespace tsa {

// State order of the RTL SRAM word {M,Ix,Iy,Iz,Ixy,Iyz,Ixz}
// (src/TriAlign_1cyc.v:130,138).
enum { SM = 0, SIX, SIY, SIZ, SIXY, SIYZ, SIXZ, NSTATE = 7 };

// Scoring constants expanded once on the host and passed by value.
struct KParams {
  int32_t pen[7][7];      // P[target][source], src/PE_1cyc.v:164-218
  int32_t match;          // temp_AB/BC/AC arms (src/PE_1cyc.v:159-161), wrapped
  int32_t mismatch;
  int32_t s3_eq;          // temp_ABC arms (src/PE_1cyc.v:162), wrapped:
  int32_t s3_ab;          //   a==b==c / a==b!=c / a!=b   (RTL mode)
  int32_t s3_ne;
  int32_t s3_mode;        // TSA_S3_RTL / TSA_S3_SOP
  int32_t bits;           // SCORE_BITS wrap, 0 = none
  int32_t wrap_shift;     // 32 - bits, or 0 when bits == 0
  int32_t packed;         // input symbols 2-bit packed (tsa_score_batch_async_p2)
  uint32_t npen[7][4];    // -P[T][s] as int16 pairs (s 0-1, 2-3, 4-5, 6-6): PLANE's packed form
};

// Symbol i of a sequence buffer: one byte per symbol, or 2-bit packed (four
// per byte, symbol i at bits 2(i%4) of byte i/4). Either way reduced mod 4,
// as the PE's 2-bit symbol registers do (src/PE_1cyc.v:63-66).
__device__ __forceinline__ uint32_t tsa_sym(const uint8_t *s, int64_t i, int32_t packed) {
  return packed ? (uint32_t)(s[i >> 2] >> (2 * (i & 3))) & 3u : (uint32_t)s[i] & 3u;
}

// Inclusive bounds on every candidate and state value of a (la,lb,lc) cube
// under params p (no wrap). Used to decide whether int16 storage and the
// factored (message) form are exact.
struct Range {
  int64_t lo, hi;
};

int build_kparams(const tsa_params *p, KParams *kp);
Range value_bound(const tsa_params *p, int64_t la, int64_t lb, int64_t lc);
// How far a state can sit below its best predecessor (drop) and a candidate
// below a state (cdrop), for value_bound and the checked kernel.
void bound_drops(const tsa_params *p, int64_t *drop, int64_t *cdrop);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for `fn` on the current
// device, skipped when an earlier call on that device already allowed at
// least `lds` bytes (a per-launch attribute call is host latency on every
// single-cube call). hipSuccess or the HIP error.
hipError_t set_dynamic_lds(const void *fn, size_t lds);
// Drop `fn`'s cached entries (every device): the next set_dynamic_lds sets the
// attribute again.
void forget_dynamic_lds(const void *fn);
// set_dynamic_lds + launch() (a hipLaunchKernelGGL of fn with `lds` dynamic
// bytes). A cached attribute can be stale -- hipDeviceReset drops it while the
// cache still skips the call -- so a failed launch forgets the entry, sets the
// attribute afresh and launches once more. hipSuccess or the HIP error.
template <class F>
hipError_t launch_with_lds(const void *fn, size_t lds, F &&launch) {
  hipError_t rc = set_dynamic_lds(fn, lds);
  if (rc != hipSuccess) return rc;
  launch();
  if ((rc = hipGetLastError()) == hipSuccess) return rc;
  forget_dynamic_lds(fn);
  if ((rc = set_dynamic_lds(fn, lds)) != hipSuccess) return rc;
  launch();
  return hipGetLastError();
}

// Row stride (cells) of a (y,z) plane with lc+1 columns.
inline int64_t plane_ldz(int64_t lc) { return lc + 1; }

// ---- plane kernel (TSA_KERNEL_PLANE) --------------------------------------
// A plane cell is the 7 int16 states + one pad: 16 bytes, one dwordx4.
struct PlaneLayout {
  int64_t ldz;          // row stride of a (y,z) plane, in cells
  int64_t plane;        // cells per plane = (max_lb+1)*ldz
  int64_t per_triple;   // cells per triple = 4 slots * plane
};
PlaneLayout plane_layout(int32_t max_lb, int32_t max_lc);
size_t plane_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc);
int plane_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                       int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                       int32_t *d_scores, int32_t *d_final7, void *d_ws, size_t ws_bytes,
                       hipStream_t stream, uint32_t *d_tb = nullptr);
// ---- literal helix (literal_kernel.hip): TSA_KERNEL_PLANE's batch path -----
// The RTL's literal arithmetic in push form on the helix schedule, LC <= 512.
bool literal_shape_ok(int32_t max_la, int32_t max_lb, int32_t max_lc);
size_t literal_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc);
int literal_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_la,
                         int32_t max_lb, int32_t max_lc, const KParams &kp, int32_t *d_scores,
                         int32_t *d_final7, void *d_ws, size_t ws_bytes, hipStream_t stream);
// Which literal kernel a batch runs (TSA_KERNEL_PLANE): the literal lap
// schedule (a few cubes, lap_kernel LIT), the literal helix (batches the
// helix shape holds) or the plane sweep (the rest; traceback), by a cost
// model. lap: a LapPolicy (LAP_OFF: no lap). TSA_PENCIL_MODE=plane / literal
// / litlap force one (tests).
enum LitKind { LIT_PLANE = 0, LIT_HELIX = 1, LIT_LAP = 2 };
int literal_kind(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop, int lap);
bool literal_helix_chosen(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc);
size_t literal_plan_workspace(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop, int lap);
// d_err (synchronous callers, lap plans only): as pencil_launch_batch's.
// choice_n: the batch size the workspace was sized for.
int literal_plan_launch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n, int32_t max_la, int32_t max_lb,
                        int32_t max_lc, const KParams &kp, int32_t *d_scores, int32_t *d_final7, void *d_ws,
                        size_t ws_bytes, hipStream_t stream, int lap, int32_t **d_err, int32_t choice_n);
void literal_describe(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, bool sop, int lap, char *buf,
                      size_t len);

// Traceback: pointer cube of one (la,lb,lc) triple and the walk kernel.
size_t tb_cube_bytes(int32_t la, int32_t lb, int32_t lc);
__global__ void tb_walk(const uint32_t *tb, const int32_t *final7, int32_t la, int32_t lb,
                        int32_t lc, uint8_t *moves, int32_t *info);

}  // namespace tsa
