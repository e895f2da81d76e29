// pencil_kernel.h -- TSA_KERNEL_PENCIL host interface (see pencil_kernel.hip).
#pragma once

#include "tsa_internal.h"

namespace tsa {

// Headroom (score units) the factored form needs beyond the a-priori bound on
// candidates and states (value_bound): its messages max_s(S[s] - P[T][s]) sit
// one score below a candidate, the f16 form folds the mismatch into them and
// adds the triple score in two parts. Every such intermediate lies within
// [lo - slack, hi + slack], so the carrier (int16, or exact
// f16 integers in [-2048, 2048]) must hold that interval.
int64_t pencil_slack(int32_t match, int32_t mismatch, int32_t gap_open, int32_t gap_extend);

bool pencil_supported(const tsa_params *p);
bool pencil_shape_supported(int32_t max_la, int32_t max_lb, int32_t max_lc);
// Which single-cube (lap) schedules a launch may use:
//   LAP_OFF      -- helix only (no cross-workgroup dependency at all);
//   LAP_RESIDENT -- the lap kernel (async path);
//   LAP_STREAM   -- the same plans on the synchronous paths, which check
//                   *d_err after the launch and rescore with LAP_OFF.
// Both run grids of up to LAP_MAX_WAVES rounds with boundary rings (lap_geom),
// launched as one resident round whose workgroups loop over their later-round
// laps in lap order (any workgroups per CU; every launched workgroup must be
// co-resident); a lap launch that times out reports TSA_SCORE_INVALID.
enum LapPolicy { LAP_OFF = 0, LAP_RESIDENT = 1, LAP_STREAM = 2 };
// Certification limits of the checked kernel (DESIGN.md 1.2 with the observed
// range of best in place of the a-priori one): a triple's scores stand when
// max(best) <= best_max and min(best) >= best_min.
struct CheckLimits {
  int32_t best_max, best_min;
};
size_t pencil_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                              const KParams &kp, const Range &bound, LapPolicy lap,
                              bool checked = false);
// The plan pencil_launch_batch would run, as text (tsa_describe_plan).
void pencil_describe(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                     const Range &bound, LapPolicy lap, char *buf, size_t len, bool checked = false);
int pencil_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                        int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                        const Range &bound, int32_t *d_scores, void *d_ws, size_t ws_bytes,
                        hipStream_t stream, LapPolicy lap, int32_t **d_err,
                        const CheckLimits *chk = nullptr);
// The checked lap kernel (TSA_KERNEL_CHECKED) can run this batch: the lap
// schedule is chosen for it (int16 arithmetic).
bool pencil_checked_plan(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                         const KParams &kp, LapPolicy lap);

}  // namespace tsa
