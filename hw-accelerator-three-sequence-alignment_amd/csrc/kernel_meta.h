// Kernel resource table (SGPRs, VGPRs, AGPRs, scratch, static LDS) of every
// gfx950 kernel in libtrialign, generated at build time from the code
// objects' metadata notes by tools/kernel_meta.py (build/kernel_meta.cpp).
// The lap kernel needs the SGPR count: the HIP occupancy API reads one
// workgroup per CU high at .sgpr_count 81-96 / 97-112 (MI355X_MICROARCH.md:463),
// and a lap grid that is not all resident can wait on a workgroup that never
// starts.
#pragma once
#include <algorithm>

namespace tsa {
struct KernelMeta {
  const char *name;  // mangled
  int sgpr, vgpr, agpr, scratch, lds;
};
extern const KernelMeta kKernelMeta[];
extern const int kKernelMetaCount;

// Largest SGPR count over the kernels whose mangled name starts with `prefix`;
// -1 if none.
inline int kernel_sgpr_max(const char *prefix) {
  int best = -1;
  for (int i = 0; i < kKernelMetaCount; ++i) {
    const char *a = kKernelMeta[i].name, *b = prefix;
    while (*b && *a == *b) ++a, ++b;
    if (!*b && kKernelMeta[i].sgpr > best) best = kKernelMeta[i].sgpr;
  }
  return best;
}
// Largest VGPR + AGPR count over those kernels; -1 if none.
inline int kernel_vgpr_max(const char *prefix) {
  int best = -1;
  for (int i = 0; i < kKernelMetaCount; ++i) {
    const char *a = kKernelMeta[i].name, *b = prefix;
    while (*b && *a == *b) ++a, ++b;
    if (!*b && kKernelMeta[i].vgpr + kKernelMeta[i].agpr > best) best = kKernelMeta[i].vgpr + kKernelMeta[i].agpr;
  }
  return best;
}
// Waves per SIMD the VGPR file admits (512 per lane, allocation granule 8).
inline int vgpr_waves_per_simd(int vgpr) {
  const int g = ((vgpr > 0 ? vgpr : 1) + 7) / 8 * 8;
  return std::min(8, 512 / g);
}
// Waves per SIMD the SGPR file admits (800 SGPRs per SIMD, allocation
// granule 16, plus 16 reserved per wave: MI355X_MICROARCH.md:463).
inline int sgpr_waves_per_simd(int sgpr) { return sgpr <= 0 ? 8 : 800 / (((sgpr + 15) / 16) * 16 + 16); }
}  // namespace tsa
