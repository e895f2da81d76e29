// pencil_kernel.hip -- TSA_KERNEL_PENCIL (placeholder until the systolic
// pencil kernel lands; AUTO dispatch routes every shape to the plane kernel).
#include "pencil_kernel.h"

namespace tsa {

bool pencil_supported(const tsa_params *p) {
  (void)p;
  return false;
}

size_t pencil_workspace_bytes(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc) {
  (void)n; (void)max_la; (void)max_lb; (void)max_lc;
  return 0;
}

int pencil_launch_batch(const uint8_t *, const int64_t *, int32_t, int32_t, int32_t, int32_t,
                        const KParams &, int32_t *, void *, size_t, hipStream_t) {
  return TSA_EINVAL;
}

}  // namespace tsa
