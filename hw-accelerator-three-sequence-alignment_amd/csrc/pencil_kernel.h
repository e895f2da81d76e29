// pencil_kernel.h -- TSA_KERNEL_PENCIL host interface (see pencil_kernel.hip).
#pragma once

#include "tsa_internal.h"

namespace tsa {

// Headroom (score units) the pencil kernel's int16 lanes keep beyond the
// a-priori value bound: message biases and penalties are applied in int16.
constexpr int64_t PENCIL_MARGIN = 512;

bool pencil_supported(const tsa_params *p);
bool pencil_shape_supported(int32_t max_la, int32_t max_lb, int32_t max_lc);
// stream_ok: the lap kernel may use a grid larger than the resident slots (needs
// in-order block dispatch; the caller must check *d_err after the launch and
// rerun with stream_ok = false if it is set)
size_t pencil_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                              bool stream_ok);
// The plan pencil_launch_batch would run, as text (tsa_describe_plan).
void pencil_describe(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                     const Range &bound, bool stream_ok, char *buf, size_t len);
int pencil_launch_batch(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                        int32_t max_la, int32_t max_lb, int32_t max_lc, const KParams &kp,
                        const Range &bound, int32_t *d_scores, void *d_ws, size_t ws_bytes,
                        hipStream_t stream, bool stream_ok, int32_t **d_err);

}  // namespace tsa
