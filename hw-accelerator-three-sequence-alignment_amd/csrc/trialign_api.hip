// trialign_api.hip -- the C-ABI of include/trialign.h: validation, parameter
// expansion, device memory, kernel dispatch and multi-GPU batch sharding.
//
// Boundary mapping (reference file:line -> entry point) is in
// include/trialign.h. There is deliberately no CPU scoring path here: with no
// HIP device every scoring call returns TSA_ENODEV.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "tsa_internal.h"
#include "pencil_kernel.h"
#include "lap_kernel.h"

#ifndef TSA_SRC_HASH  // set by the Makefile: srchash.py over csrc/*.{hip,h} + include/trialign.h
#define TSA_SRC_HASH "unhashed"
#endif

namespace tsa {

static inline int64_t wrap64(int64_t v, int bits) {
  if (bits == 0) return v;
  const uint64_t u = (uint64_t)v << (64 - bits);
  return (int64_t)u >> (64 - bits);
}

static int params_ok(const tsa_params *p) {
  if (!p) return 0;
  if (p->s3_mode != TSA_S3_RTL && p->s3_mode != TSA_S3_SOP) return 0;
  if (p->score_bits != 0 && (p->score_bits < 4 || p->score_bits > 16)) return 0;
  const int32_t lim = 1 << 12;
  if (std::abs(p->match) > lim || std::abs(p->mismatch) > lim || std::abs(p->gap_open) > lim ||
      std::abs(p->gap_extend) > lim)
    return 0;
  return 1;
}

int build_kparams(const tsa_params *p, KParams *kp) {
  if (!params_ok(p) || !kp) return TSA_EINVAL;
  std::memset(kp, 0, sizeof(*kp));
  const int32_t GO = p->gap_open, GE = p->gap_extend;
  const int32_t GO2 = 2 * GO, GE2 = 2 * GE, GOGE = GO + GE;
  const int32_t t[7][7] = {
      {0, 0, 0, 0, 0, 0, 0},                   // M   src/PE_1cyc.v:164-170
      {GO2, GE2, GOGE, GOGE, GOGE, GO2, GOGE}, // Ix  :172-178
      {GO2, GOGE, GE2, GOGE, GOGE, GOGE, GO2}, // Iy  :180-186
      {GO2, GOGE, GOGE, GE2, GO2, GOGE, GOGE}, // Iz  :188-194
      {GO, GE, GE, GO, GE, GO, GO},            // Ixy :196-202
      {GO, GO, GE, GE, GO, GE, GO},            // Iyz :204-210
      {GO, GE, GO, GE, GO, GO, GE},            // Ixz :212-218
  };
  std::memcpy(kp->pen, t, sizeof(t));
  for (int T = 0; T < 7; ++T)
    for (int i = 0; i < 4; ++i) {
      const int32_t lo = -t[T][2 * i], hi = -t[T][std::min(2 * i + 1, 6)];
      kp->npen[T][i] = (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16);
    }
  const int bits = p->score_bits;
  kp->bits = bits;
  kp->wrap_shift = bits ? 32 - bits : 0;
  kp->match = (int32_t)wrap64(p->match, bits);
  kp->mismatch = (int32_t)wrap64(p->mismatch, bits);
  // src/PE_1cyc.v:162 -- '+' binds tighter than '<<' in Verilog
  kp->s3_eq = (int32_t)wrap64(3LL * p->match, bits);
  kp->s3_ab = (int32_t)wrap64(2LL * ((int64_t)p->match + p->mismatch), bits);
  kp->s3_ne = (int32_t)wrap64(3LL * p->mismatch, bits);
  kp->s3_mode = p->s3_mode;
  return TSA_OK;
}

// How far below the best of its predecessor a state (drop) and below a state
// a candidate (cdrop) can sit: penalty minus the smallest score of the target.
void bound_drops(const tsa_params *p, int64_t *drop, int64_t *cdrop) {
  KParams kp;
  build_kparams(p, &kp);
  const int64_t m = p->match, mm = p->mismatch;
  const int64_t s3min = p->s3_mode == TSA_S3_SOP ? std::min({3 * m, m + 2 * mm, 3 * mm})
                                                 : std::min({3 * m, 2 * (m + mm), 3 * mm});
  const int64_t s2min = std::min(m, mm);
  *drop = 0;
  *cdrop = 0;
  for (int T = 0; T < 7; ++T) {
    const int64_t scmin = T == SM ? s3min : T <= SIZ ? 0 : s2min;
    int64_t maxp = kp.pen[T][0];
    for (int s = 0; s < 7; ++s) {
      maxp = std::max<int64_t>(maxp, kp.pen[T][s]);
      *cdrop = std::max<int64_t>(*cdrop, kp.pen[T][s] - scmin);
    }
    *drop = std::max<int64_t>(*drop, maxp - scmin);
  }
}

Range value_bound(const tsa_params *p, int64_t la, int64_t lb, int64_t lc) {
  KParams kp;
  build_kparams(p, &kp);
  const int64_t m = p->match, mm = p->mismatch;
  int64_t s3v[3];
  if (p->s3_mode == TSA_S3_SOP) { s3v[0] = 3 * m; s3v[1] = m + 2 * mm; s3v[2] = 3 * mm; }
  else { s3v[0] = 3 * m; s3v[1] = 2 * (m + mm); s3v[2] = 3 * mm; }
  const int64_t s3max = *std::max_element(s3v, s3v + 3), s3min = *std::min_element(s3v, s3v + 3);
  const int64_t s2max = std::max(m, mm), s2min = std::min(m, mm);
  int64_t scmax[7], scmin[7], dq[7];
  for (int T = 0; T < 7; ++T) {
    if (T == SM) { scmax[T] = s3max; scmin[T] = s3min; dq[T] = 3; }
    else if (T <= SIZ) { scmax[T] = 0; scmin[T] = 0; dq[T] = 1; }
    else { scmax[T] = s2max; scmin[T] = s2min; dq[T] = 2; }
  }
  // upper: best(cell) <= best(pred_T) + inc_T; a path from a zero face to q
  // advances q by dq_T per step, so every value <= q * max_T(inc_T/dq_T)^+.
  double gain = 0.0;
  for (int T = 0; T < 7; ++T)
    for (int s = 0; s < 7; ++s) gain = std::max(gain, (double)(scmax[T] - kp.pen[T][s]) / dq[T]);
  const int64_t hi = (int64_t)std::floor(gain * (double)(la + lb + lc) + 1e-9);
  // lower: best(cell) >= best(diag) + s3 (P[M][*] = 0) -> >= min(l)*min(0,s3min)
  const int64_t mn = std::min(la, std::min(lb, lc));
  const int64_t bestlo = mn * std::min<int64_t>(0, s3min);
  int64_t drop = 0, cdrop = 0;
  bound_drops(p, &drop, &cdrop);
  const int64_t statelo = std::min<int64_t>(0, bestlo - drop);
  Range r;
  r.lo = statelo - std::max<int64_t>(0, cdrop);
  r.hi = std::max<int64_t>(hi, 0);
  return r;
}

}  // namespace tsa

using namespace tsa;

extern "C" {

void tsa_default_params(tsa_params *p) {
  if (!p) return;
  p->match = 1;       // src/PE_1cyc.v:55
  p->mismatch = -1;   // :56
  p->gap_open = 2;    // :57
  p->gap_extend = 1;  // :58
  p->s3_mode = TSA_S3_RTL;
  p->score_bits = 12; // src/TriAlign_tb.sv:56
}

const char *tsa_strerror(int rc) {
  switch (rc) {
    case TSA_OK: return "ok";
    case TSA_EINVAL: return "invalid argument (pointer, length, symbol or parameter)";
    case TSA_ERANGE: return "score range not representable exactly";
    case TSA_ENODEV: return "no HIP device";
    case TSA_EDEVICE: return "HIP runtime error";
    case TSA_ENOMEM: return "out of device memory / workspace too small";
    case TSA_EINTERNAL: return "internal self-check failed";
    default: return "unknown error";
  }
}

const char *tsa_version(void) { return "trialign-mi355x gfx950 src=" TSA_SRC_HASH; }

int tsa_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int tsa_validate(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
                 int32_t lc, const tsa_params *p) {
  if (!a || !b || !c || !params_ok(p)) return TSA_EINVAL;
  if (la < 1 || lb < 1 || lc < 1) return TSA_EINVAL;
  for (int32_t i = 0; i < la; ++i) if (a[i] > 4) return TSA_EINVAL;
  for (int32_t i = 0; i < lb; ++i) if (b[i] > 4) return TSA_EINVAL;
  for (int32_t i = 0; i < lc; ++i) if (c[i] > 4) return TSA_EINVAL;
  if (p->score_bits == 0) {  // int16 state storage must hold the unwrapped range
    const Range r = value_bound(p, la, lb, lc);
    if (r.lo < -32768 || r.hi > 32767) return TSA_ERANGE;
  }
  return TSA_OK;
}

}  // extern "C"

namespace tsa {

namespace {
struct LdsEntry {
  const void *fn;
  int dev;
  size_t lds;
};
std::mutex lds_mu;
std::vector<LdsEntry> lds_done;
}  // namespace

void forget_dynamic_lds(const void *fn) {
  std::lock_guard<std::mutex> g(lds_mu);
  lds_done.erase(std::remove_if(lds_done.begin(), lds_done.end(), [&](const LdsEntry &e) { return e.fn == fn; }),
                 lds_done.end());
}

hipError_t set_dynamic_lds(const void *fn, size_t lds) {
  using Entry = LdsEntry;
  std::mutex &mu = lds_mu;
  std::vector<Entry> &done = lds_done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  {
    std::lock_guard<std::mutex> g(mu);
    for (const Entry &e : done)
      if (e.fn == fn && e.dev == dev && e.lds >= lds) return hipSuccess;
  }
  const hipError_t rc = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (rc == hipSuccess) {
    std::lock_guard<std::mutex> g(mu);
    for (Entry &e : done)
      if (e.fn == fn && e.dev == dev) {
        e.lds = std::max(e.lds, lds);
        return rc;
      }
    done.push_back(Entry{fn, dev, lds});
  }
  return rc;
}

// Is the factored (pencil) arithmetic bit-identical to the literal RTL form
// for every triple of these lengths? Two separate conditions:
//  (1) no candidate can wrap at score_bits -- the bare bound, which already
//      covers every candidate and state (value_bound), against the RTL word;
//  (2) the kernel's carrier holds every intermediate of the factored form:
//      the bound widened by pencil_slack inside int16 (use_f16 applies the
//      same test against the exact-f16 range to pick the f16 arithmetic).
static bool pencil_exact(const tsa_params *p, int64_t la, int64_t lb, int64_t lc) {
  const Range r = value_bound(p, la, lb, lc);
  if (p->score_bits) {
    const int64_t lim_lo = -(1LL << (p->score_bits - 1)), lim_hi = (1LL << (p->score_bits - 1)) - 1;
    if (r.lo < lim_lo || r.hi > lim_hi) return false;
  }
  const int64_t slack = pencil_slack(p->match, p->mismatch, p->gap_open, p->gap_extend);
  return r.lo - slack >= -32768 && r.hi + slack <= 32767 && pencil_supported(p) &&
         pencil_shape_supported((int32_t)la, (int32_t)lb, (int32_t)lc);
}

// Can the checked kernel (TSA_KERNEL_CHECKED) score these lengths? The int16
// carrier holds the a-priori bound (no wrap of its own), only the RTL's
// SCORE_BITS wrap cannot be ruled out a priori.
static bool pencil_checkable(const tsa_params *p, int64_t la, int64_t lb, int64_t lc) {
  if (p->score_bits == 0 || !pencil_supported(p) ||
      !pencil_shape_supported((int32_t)la, (int32_t)lb, (int32_t)lc))
    return false;
  const Range r = value_bound(p, la, lb, lc);
  const int64_t slack = pencil_slack(p->match, p->mismatch, p->gap_open, p->gap_extend);
  return r.lo - slack >= -32768 && r.hi + slack <= 32767;
}

// The checked kernel's certification (DESIGN.md 1.2 with the observed range
// of best in place of the a-priori one): every state lies in
// [min(0, bmin - drop), bmax] and every candidate above that minus cdrop, so
// no candidate wraps at SCORE_BITS when bmax fits and bmin >= lo + drop + cdrop.
static CheckLimits check_limits(const tsa_params *p) {
  const int64_t lim_lo = -(1LL << (p->score_bits - 1)), lim_hi = (1LL << (p->score_bits - 1)) - 1;
  int64_t drop = 0, cdrop = 0;
  bound_drops(p, &drop, &cdrop);
  CheckLimits c;
  c.best_max = (int32_t)lim_hi;
  c.best_min = -std::max<int64_t>(0, cdrop) < lim_lo ? INT32_MAX  // never certifiable
                                                    : (int32_t)(lim_lo + drop + std::max<int64_t>(0, cdrop));
  return c;
}

// TSA_KERNEL_CHECKED is an internal kind too: AUTO upgrades PLANE to it on the
// synchronous paths (upgrade_checked).
static int choose_kernel(int32_t kernel, const tsa_params *p, int64_t la, int64_t lb, int64_t lc) {
  if (kernel == TSA_KERNEL_PLANE) return TSA_KERNEL_PLANE;
  const bool ok = pencil_exact(p, la, lb, lc);
  if (kernel == TSA_KERNEL_PENCIL) return ok ? TSA_KERNEL_PENCIL : -1;
  if (kernel == TSA_KERNEL_CHECKED)
    return ok ? TSA_KERNEL_PENCIL : pencil_checkable(p, la, lb, lc) ? TSA_KERNEL_CHECKED : -1;
  return ok ? TSA_KERNEL_PENCIL : TSA_KERNEL_PLANE;
}
static bool checked_plan(int32_t n, const tsa_params *p, int32_t la, int32_t lb, int32_t lc,
                         LapPolicy lap) {
  KParams kp;
  return build_kparams(p, &kp) == TSA_OK && pencil_checked_plan(std::min(n, 65535), la, lb, lc, kp, lap);
}
static int upgrade_checked(int kind, int32_t kernel, int32_t n, const tsa_params *p, int32_t la,
                           int32_t lb, int32_t lc) {
  if (kind == TSA_KERNEL_PLANE && kernel == TSA_KERNEL_AUTO && pencil_checkable(p, la, lb, lc) &&
      checked_plan(n, p, la, lb, lc, LAP_STREAM))
    return TSA_KERNEL_CHECKED;
  return kind;
}

// lap: LAP_STREAM only on the synchronous paths, which check the lap kernel's
// error word and rescore with LAP_OFF; the async path keeps LAP_RESIDENT
static size_t workspace_for(int kind, int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                            const tsa_params *p, LapPolicy lap = LAP_RESIDENT) {
  if (kind == TSA_KERNEL_PLANE)
    return literal_plan_workspace(n, max_la, max_lb, max_lc, p->s3_mode == TSA_S3_SOP, lap);
  KParams kp;
  if (build_kparams(p, &kp)) return 0;
  return pencil_workspace_bytes(n, max_la, max_lb, max_lc, kp, value_bound(p, max_la, max_lb, max_lc),
                                lap, kind == TSA_KERNEL_CHECKED);
}

// Lap hand-offs that timed out on the synchronous path (each rescored by the
// helix kernel), process-wide; tsa_fallback_count() reads it.
static std::atomic<int64_t> g_lap_fallbacks{0};
// Triples the checked kernel could not certify (rescored by PLANE).
static std::atomic<int64_t> g_check_fallbacks{0};

static int launch_kind(int kind, const uint8_t *d_seqs, const int64_t *d_off, int32_t n,
                       int32_t max_la, int32_t max_lb, int32_t max_lc, const tsa_params *p,
                       int32_t *d_scores, int32_t *d_final7, void *ws, size_t ws_bytes,
                       hipStream_t s, LapPolicy lap = LAP_RESIDENT, int32_t **d_err = nullptr,
                       int32_t packed = 0, int32_t choice_n = -1) {
  // choice_n: the batch size the workspace was sized for (a chunk may be
  // smaller, and must run the kernel that workspace was sized for)
  KParams kp;
  int rc = build_kparams(p, &kp);
  if (rc) return rc;
  kp.packed = packed;
  if (kind == TSA_KERNEL_PLANE)
    return literal_plan_launch(d_seqs, d_off, n, max_la, max_lb, max_lc, kp, d_scores, d_final7, ws, ws_bytes, s,
                               lap, d_err, choice_n);
  const CheckLimits lim = check_limits(p);
  return pencil_launch_batch(d_seqs, d_off, n, max_la, max_lb, max_lc, kp,
                             value_bound(p, max_la, max_lb, max_lc), d_scores, ws, ws_bytes, s,
                             lap, d_err, kind == TSA_KERNEL_CHECKED ? &lim : nullptr);
}

#define HIPCHK(x)                                   \
  do {                                              \
    if ((x) != hipSuccess) { rc = TSA_EDEVICE; goto done; } \
  } while (0)

// Score triples [i0, i1) of a host batch on one device (synchronous).
static int run_host_batch_on_device(int device, const uint8_t *seqs, const int64_t *offsets,
                                    int32_t i0, int32_t i1, const tsa_params *p, int32_t kernel,
                                    int32_t *scores, int32_t *final7) {
  int rc = TSA_OK;
  const int32_t n = i1 - i0;
  if (n <= 0) return TSA_OK;
  int32_t max_la = 0, max_lb = 0, max_lc = 0;
  for (int32_t i = i0; i < i1; ++i) {
    const int64_t *o = offsets + 3 * (int64_t)i;
    max_la = std::max<int32_t>(max_la, (int32_t)(o[1] - o[0]));
    max_lb = std::max<int32_t>(max_lb, (int32_t)(o[2] - o[1]));
    max_lc = std::max<int32_t>(max_lc, (int32_t)(o[3] - o[2]));
  }
  int kind = choose_kernel(kernel, p, max_la, max_lb, max_lc);
  if (kind < 0) return TSA_ERANGE;
  if (!final7) kind = upgrade_checked(kind, kernel, n, p, max_la, max_lb, max_lc);
  // chunk so the workspace stays under ~8 GiB and the grid under 65535
  // triples; the workspace is what the chunk's own plan (lap for a few cubes,
  // the helix ring otherwise) and its fallbacks (the same kind without the lap
  // schedule; the literal kinds for the checked kernel) need
  auto ws_of = [&](int32_t c) {
    size_t w = std::max(workspace_for(kind, c, max_la, max_lb, max_lc, p, LAP_STREAM),
                        workspace_for(kind, c, max_la, max_lb, max_lc, p, LAP_OFF));
    if (kind == TSA_KERNEL_CHECKED)
      w = std::max({w, workspace_for(TSA_KERNEL_PLANE, c, max_la, max_lb, max_lc, p, LAP_STREAM),
                    workspace_for(TSA_KERNEL_PLANE, c, max_la, max_lb, max_lc, p, LAP_OFF)});
    return w;
  };
  const size_t cap = (size_t)8 << 30;
  int32_t chunk = std::min(n, 65535);
  while (chunk > 1 && ws_of(chunk) > cap)
    chunk = std::max<int32_t>(1, std::min<int32_t>(chunk - 1, (int32_t)((double)chunk * cap / ws_of(chunk))));
  const size_t ws_bytes = ws_of(chunk);
  const int64_t base = offsets[3 * (int64_t)i0];
  const int64_t nbytes = offsets[3 * (int64_t)i1] - base;
  uint8_t *d_seqs = nullptr;
  int64_t *d_off = nullptr;
  int32_t *d_scores = nullptr, *d_final = nullptr;
  void *d_ws = nullptr;
  std::vector<int64_t> off((size_t)3 * n + 1);
  hipStream_t s = nullptr;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (size_t k = 0; k < off.size(); ++k) off[k] = offsets[3 * (int64_t)i0 + (int64_t)k] - base;
  if (hipMalloc(&d_seqs, std::max<int64_t>(nbytes, 1)) != hipSuccess ||
      hipMalloc(&d_off, off.size() * sizeof(int64_t)) != hipSuccess ||
      hipMalloc(&d_scores, (size_t)n * sizeof(int32_t)) != hipSuccess ||
      (final7 && hipMalloc(&d_final, (size_t)n * 7 * sizeof(int32_t)) != hipSuccess) ||
      hipMalloc(&d_ws, std::max<size_t>(ws_bytes, 16)) != hipSuccess) {
    rc = TSA_ENOMEM;
    goto done;
  }
  HIPCHK(hipMemcpyAsync(d_seqs, seqs + base, nbytes, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_off, off.data(), off.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(d_ws, 0, ws_bytes, s));
  for (int32_t c0 = 0; c0 < n && rc == TSA_OK; c0 += chunk) {
    // a lap launch whose hand-off timed out (*d_err set) is rescored by the
    // same kind without the lap schedule (no cross-workgroup dependency)
    auto lap_rescue = [&](int k, int32_t cn, int32_t *d_err, int32_t *fin) -> int {
      int32_t herr = 0;
      if (hipMemcpyAsync(&herr, d_err, sizeof(herr), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return TSA_EDEVICE;
      if (!herr) return TSA_OK;
      g_lap_fallbacks.fetch_add(1);
      fprintf(stderr, "trialign: lap hand-off timed out on device %d (%d triples); rescoring "
                      "without the lap schedule\n", device, cn);
      int32_t *d_err2 = nullptr;
      int r = launch_kind(k, d_seqs, d_off + 3 * (int64_t)c0, cn, max_la, max_lb, max_lc, p, d_scores + c0, fin,
                          d_ws, ws_bytes, s, LAP_OFF, &d_err2);
      if (r == TSA_OK && d_err2) r = TSA_EINTERNAL;  // LAP_OFF never plans a lap grid
      return r;
    };
    const int32_t cn = std::min(chunk, n - c0);
    int32_t *d_err = nullptr;
    rc = launch_kind(kind, d_seqs, d_off + 3 * (int64_t)c0, cn, max_la, max_lb, max_lc, p,
                     d_scores + c0, d_final ? d_final + 7 * (int64_t)c0 : nullptr, d_ws,
                     ws_bytes, s, LAP_STREAM, &d_err, 0, chunk);
    if (rc == TSA_OK && kind == TSA_KERNEL_CHECKED) {
      // certified scores stand; a chunk with any other (uncertified, or a
      // timed-out hand-off) is rescored by the literal PLANE kernel
      int32_t herr = 0;
      std::vector<int32_t> hs((size_t)cn);
      HIPCHK(hipMemcpyAsync(&herr, d_err, sizeof(herr), hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(hs.data(), d_scores + c0, (size_t)cn * sizeof(int32_t), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      int64_t bad = 0;
      for (int32_t v : hs) bad += v == TSA_SCORE_UNCERTIFIED || v == TSA_SCORE_INVALID;
      if (herr || bad) {
        g_check_fallbacks.fetch_add(herr ? cn : bad);
        if (herr) g_lap_fallbacks.fetch_add(1);
        int32_t *d_err3 = nullptr;  // the literal kinds (lap, helix or plane)
        rc = launch_kind(TSA_KERNEL_PLANE, d_seqs, d_off + 3 * (int64_t)c0, cn, max_la, max_lb, max_lc,
                         p, d_scores + c0, nullptr, d_ws, ws_bytes, s, LAP_STREAM, &d_err3, 0, chunk);
        if (rc == TSA_OK && d_err3) rc = lap_rescue(TSA_KERNEL_PLANE, cn, d_err3, nullptr);
      }
    } else if (rc == TSA_OK && d_err) {  // lap kernel: a timed-out hand-off invalidates the chunk
      rc = lap_rescue(kind, cn, d_err, d_final ? d_final + 7 * (int64_t)c0 : nullptr);
    }
  }
  if (rc) goto done;
  HIPCHK(hipMemcpyAsync(scores + i0, d_scores, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (final7)
    HIPCHK(hipMemcpyAsync(final7 + 7 * (int64_t)i0, d_final, (size_t)n * 7 * sizeof(int32_t),
                          hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
done:
  if (d_seqs) (void)hipFree(d_seqs);
  if (d_off) (void)hipFree(d_off);
  if (d_scores) (void)hipFree(d_scores);
  if (d_final) (void)hipFree(d_final);
  if (d_ws) (void)hipFree(d_ws);
  if (s) (void)hipStreamDestroy(s);
  return rc;
}

}  // namespace tsa

extern "C" {

int tsa_score_gpu_ex(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
                     int32_t lc, const tsa_params *p, int32_t kernel, int32_t *score,
                     int32_t *final_states, int32_t device) {
  if (!score) return TSA_EINVAL;
  if (kernel < TSA_KERNEL_AUTO || kernel > TSA_KERNEL_CHECKED) return TSA_EINVAL;
  int rc = tsa_validate(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  const int nd = tsa_device_count();
  if (nd <= 0) return TSA_ENODEV;
  if (device < 0 || device >= nd) return TSA_ENODEV;
  std::vector<uint8_t> seqs((size_t)la + lb + lc);
  std::memcpy(seqs.data(), a, la);
  std::memcpy(seqs.data() + la, b, lb);
  std::memcpy(seqs.data() + la + lb, c, lc);
  const int64_t off[4] = {0, la, (int64_t)la + lb, (int64_t)la + lb + lc};
  const int32_t k = final_states ? TSA_KERNEL_PLANE : kernel;
  return run_host_batch_on_device(device, seqs.data(), off, 0, 1, p, k, score, final_states);
}

int64_t tsa_fallback_count(void) { return g_lap_fallbacks.load(); }
int64_t tsa_check_fallback_count(void) { return g_check_fallbacks.load(); }

int tsa_score_gpu(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
                  int32_t lc, const tsa_params *p, int32_t *score, int32_t device) {
  return tsa_score_gpu_ex(a, la, b, lb, c, lc, p, TSA_KERNEL_AUTO, score, nullptr, device);
}

int tsa_score_batch_devices(const uint8_t *seqs, const int64_t *offsets, int32_t n,
                            const tsa_params *p, int32_t *scores, const int32_t *devices,
                            int32_t n_devices) {
  if (!seqs || !offsets || !scores || !devices || n < 0 || n_devices < 1 || n_devices > 1024 ||
      !params_ok(p))
    return TSA_EINVAL;
  for (int32_t i = 0; i < n; ++i) {
    const int64_t *o = offsets + 3 * (int64_t)i;
    if (o[1] < o[0] || o[2] < o[1] || o[3] < o[2]) return TSA_EINVAL;
    int rc = tsa_validate(seqs + o[0], (int32_t)(o[1] - o[0]), seqs + o[1], (int32_t)(o[2] - o[1]),
                          seqs + o[2], (int32_t)(o[3] - o[2]), p);
    if (rc) return rc;
  }
  if (n == 0) return TSA_OK;
  const int nd = tsa_device_count();
  if (nd <= 0) return TSA_ENODEV;
  for (int32_t i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= nd) return TSA_ENODEV;
  // shard s = contiguous triples [n s / ns, n (s+1) / ns) on devices[s]; one
  // host thread per DISTINCT device runs that device's shards in list order
  // (shards sharing a device never run concurrently: a lap grid's residency
  // plan assumes it has the device to itself)
  const int ns = std::min<int32_t>(n_devices, n);
  std::vector<int> dev_of_thread;
  std::vector<std::vector<int>> shards_of_thread;
  for (int s = 0; s < ns; ++s) {
    const int d = devices[s];
    size_t k = 0;
    while (k < dev_of_thread.size() && dev_of_thread[k] != d) ++k;
    if (k == dev_of_thread.size()) {
      dev_of_thread.push_back(d);
      shards_of_thread.emplace_back();
    }
    shards_of_thread[k].push_back(s);
  }
  std::vector<int> rcs(ns, TSA_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < dev_of_thread.size(); ++k) {
    th.emplace_back([&, k] {
      for (int s : shards_of_thread[k]) {
        const int32_t i0 = (int32_t)((int64_t)n * s / ns), i1 = (int32_t)((int64_t)n * (s + 1) / ns);
        rcs[s] = run_host_batch_on_device(dev_of_thread[k], seqs, offsets, i0, i1, p, TSA_KERNEL_AUTO,
                                          scores, nullptr);
        if (rcs[s]) break;
      }
    });
  }
  for (auto &t : th) t.join();
  for (int r : rcs) if (r) return r;
  return TSA_OK;
}

int tsa_score_batch(const uint8_t *seqs, const int64_t *offsets, int32_t n, const tsa_params *p,
                    int32_t *scores, int32_t n_devices) {
  if (!seqs || !offsets || !scores || n < 0 || !params_ok(p)) return TSA_EINVAL;
  const int nd = tsa_device_count();
  if (nd <= 0) {  // validation, then TSA_ENODEV (TSA_OK for n == 0)
    const int32_t d0 = 0;
    return tsa_score_batch_devices(seqs, offsets, n, p, scores, &d0, 1);
  }
  const int use = std::max(1, std::min(n_devices <= 0 ? nd : n_devices, std::max(1, std::min(nd, n))));
  std::vector<int32_t> devs((size_t)use);
  for (int d = 0; d < use; ++d) devs[d] = d;
  return tsa_score_batch_devices(seqs, offsets, n, p, scores, devs.data(), use);
}

int tsa_score_gpu_multi(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                        const uint8_t *c, int32_t lc, const tsa_params *p, const int32_t *devices,
                        int32_t n_devices, int32_t *score, double *wall_us) {
  using namespace tsa;
  if (!score || !devices || n_devices < 1 || n_devices > 64) return TSA_EINVAL;
  int rc = tsa_validate(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  const int nd = tsa_device_count();
  if (nd <= 0) return TSA_ENODEV;
  for (int32_t i = 0; i < n_devices; ++i)
    if (devices[i] < 0 || devices[i] >= nd) return TSA_ENODEV;
  // the factored form where it is exact a priori, else the literal arithmetic
  const bool exact = pencil_exact(p, la, lb, lc);
  KParams kp;
  if ((rc = build_kparams(p, &kp))) return rc;
  const Range bound = value_bound(p, la, lb, lc);
  const LapGeom g = exact ? pencil_split_geom(la, lb, lc, kp, bound, n_devices)
                          : literal_split_geom(la, lb, lc, p->s3_mode == TSA_S3_SOP, n_devices);
  if (!g.ok) return TSA_ERANGE;  // no lap schedule, or fewer laps than parts
  const int np = n_devices;
  const size_t ws_bytes = lap_workspace_bytes(g);
  const int64_t off[4] = {0, la, (int64_t)la + lb, (int64_t)la + lb + lc};
  std::vector<LapPart> parts((size_t)np);
  std::vector<void *> ws((size_t)np, nullptr);
  std::vector<char> own((size_t)np, 0);  // part i created its stream
  int32_t *d_score = nullptr;
  uint32_t *d_err = nullptr;
  int32_t h_score = 0;
  double t0 = 0, t1 = 0;
  bool launched = false;
  auto now_us = [] {
    return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count() * 1e-3;
  };
  for (int i = 0; i < np; ++i) parts[i] = LapPart{devices[i], nullptr, 0, 0, nullptr, nullptr, nullptr};
  // Parts sharing a device run concurrently, each on its own stream, when all
  // their workgroups fit on that device at once (every lap resident: no part's
  // workgroups can hold the CU slots an earlier part's undispatched ones need);
  // otherwise one after another on one stream (below).
  bool concurrent = g.per_cu > 0;
  for (int i = 0; i < np && concurrent; ++i) {
    int64_t blocks = 0;
    for (int j = 0; j < np; ++j)
      if (devices[j] == devices[i])
        blocks += ((int64_t)g.G * (j + 1) / np - (int64_t)g.G * j / np) * g.CH * 8;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, devices[i]) != hipSuccess || cus <= 0 ||
        blocks > (int64_t)cus * g.per_cu)
      concurrent = false;
  }
  if (const char *e = getenv("TSA_SPLIT_SERIAL")) concurrent = concurrent && atoi(e) == 0;  // A/B knob
  // peer access between the distinct devices (each part writes into its
  // neighbours' workspaces, every part into the last one's error word)
  for (int i = 0; i < np; ++i)
    for (int j = 0; j < np; ++j) {
      const int di = devices[i], dj = devices[j];
      if (di == dj) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, di, dj) != hipSuccess || !can) { rc = TSA_EDEVICE; goto done; }
      HIPCHK(hipSetDevice(di));
      const hipError_t e = hipDeviceEnablePeerAccess(dj, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) { rc = TSA_EDEVICE; goto done; }
      (void)hipGetLastError();
    }
  for (int i = 0; i < np; ++i) {
    LapPart &q = parts[i];
    q.L0 = (int32_t)((int64_t)g.G * i / np);
    q.L1 = (int32_t)((int64_t)g.G * (i + 1) / np);
    HIPCHK(hipSetDevice(q.device));
    // unless every part fits at once (concurrent), parts sharing a device run
    // one after another on the first one's stream: launched concurrently, a
    // later part's workgroups can take the CU slots an earlier part's
    // undispatched workgroups need, and wait on them (two 256-workgroup parts
    // of 1024^3 at one workgroup per CU timed out). In lap order with
    // full-length rings an earlier part never waits on a later one.
    for (int j = 0; j < i && !q.stream && !concurrent; ++j)
      if (parts[j].device == q.device) q.stream = parts[j].stream;
    own[i] = q.stream == nullptr;
    if (own[i]) HIPCHK(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
    uint8_t *ds = nullptr;
    int64_t *dof = nullptr;
    // fine-grained: its neighbours' stores land here and are polled here
    if (hipMalloc(&ds, (size_t)off[3]) != hipSuccess || hipMalloc(&dof, sizeof(off)) != hipSuccess ||
        hipExtMallocWithFlags(&ws[i], ws_bytes, hipDeviceMallocFinegrained) != hipSuccess) {
      if (ds) (void)hipFree(ds);
      if (dof) (void)hipFree(dof);
      rc = TSA_ENOMEM;
      goto done;
    }
    q.d_seqs = ds;
    q.d_offsets = dof;
    q.d_ws = ws[i];
    HIPCHK(hipMemcpyAsync(ds, a, la, hipMemcpyHostToDevice, q.stream));
    HIPCHK(hipMemcpyAsync(ds + la, b, lb, hipMemcpyHostToDevice, q.stream));
    HIPCHK(hipMemcpyAsync(ds + la + lb, c, lc, hipMemcpyHostToDevice, q.stream));
    HIPCHK(hipMemcpyAsync(dof, off, sizeof(off), hipMemcpyHostToDevice, q.stream));
    HIPCHK(hipMemsetAsync(ws[i], 0, ws_bytes, q.stream));
    if (i == np - 1) {
      if (hipMalloc(&d_score, sizeof(int32_t)) != hipSuccess) { rc = TSA_ENOMEM; goto done; }
      d_err = lap_err_word(g, 1, ws[i]);
    }
  }
  // every workspace is initialised before any part may store into it
  for (int i = 0; i < np; ++i) {
    HIPCHK(hipSetDevice(parts[i].device));
    HIPCHK(hipStreamSynchronize(parts[i].stream));
  }
  t0 = now_us();
  launched = true;
  rc = exact ? pencil_launch_split(g, kp, bound, parts.data(), np, d_score, d_err)
             : lap_launch_split_lit(g, p->s3_mode == TSA_S3_SOP, kp, parts.data(), np, d_score, d_err);
  if (rc) goto done;
  for (int i = 0; i < np; ++i) {
    HIPCHK(hipSetDevice(parts[i].device));
    HIPCHK(hipStreamSynchronize(parts[i].stream));
  }
  t1 = now_us();
  HIPCHK(hipSetDevice(parts[np - 1].device));
  HIPCHK(hipMemcpy(&h_score, d_score, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (h_score == TSA_SCORE_INVALID) {  // a hand-off timed out: no silent score
    rc = TSA_EINTERNAL;
    goto done;
  }
  *score = h_score;
  if (wall_us) *wall_us = t1 - t0;
done:
  // once any part may be running, every part's stream drains before any
  // allocation goes: a part on another device can still be storing into its
  // neighbours' workspaces (hipFree only synchronises its own device)
  if (launched)
    for (int i = 0; i < np; ++i)
      if (parts[i].stream) {
        (void)hipSetDevice(parts[i].device);
        (void)hipStreamSynchronize(parts[i].stream);
      }
  for (int i = 0; i < np; ++i) {
    (void)hipSetDevice(parts[i].device);
    if (parts[i].d_seqs) (void)hipFree((void *)parts[i].d_seqs);
    if (parts[i].d_offsets) (void)hipFree((void *)parts[i].d_offsets);
    if (ws[i]) (void)hipFree(ws[i]);
    if (i == np - 1 && d_score) (void)hipFree(d_score);
    if (parts[i].stream && own[i]) (void)hipStreamDestroy(parts[i].stream);
  }
  return rc;
}

int tsa_align_gpu(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
                  int32_t lc, const tsa_params *p, int32_t *score, uint8_t *moves, int32_t max_moves,
                  int32_t *n_moves, int32_t *start, int32_t device) {
  if (!score || !moves || !n_moves || !start) return TSA_EINVAL;
  int rc = tsa_validate(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  if ((int64_t)max_moves < (int64_t)la + lb + lc) return TSA_EINVAL;
  const int nd = tsa_device_count();
  if (nd <= 0) return TSA_ENODEV;
  if (device < 0 || device >= nd) return TSA_ENODEV;
  KParams kp;
  if ((rc = build_kparams(p, &kp))) return rc;
  const int64_t len = (int64_t)la + lb + lc;
  const int64_t off[4] = {0, la, (int64_t)la + lb, len};
  const size_t ws_bytes = plane_workspace_bytes(1, la, lb, lc);
  const size_t tb_bytes = tb_cube_bytes(la, lb, lc);
  uint8_t *d_seqs = nullptr, *d_moves = nullptr;
  int64_t *d_off = nullptr;
  int32_t *d_small = nullptr;  // [0] score, [1..7] final states, [8..11] walk info
  uint32_t *d_tb = nullptr;
  void *d_ws = nullptr;
  hipStream_t s = nullptr;
  int32_t h_small[12];
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (hipMalloc(&d_seqs, len) != hipSuccess || hipMalloc(&d_off, sizeof(off)) != hipSuccess ||
      hipMalloc(&d_small, sizeof(h_small)) != hipSuccess ||
      hipMalloc(&d_moves, (size_t)len) != hipSuccess ||
      hipMalloc(&d_ws, std::max<size_t>(ws_bytes, 16)) != hipSuccess ||
      hipMalloc(&d_tb, std::max<size_t>(tb_bytes, 16)) != hipSuccess) {
    rc = TSA_ENOMEM;
    goto done;
  }
  HIPCHK(hipMemcpyAsync(d_seqs, a, la, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_seqs + la, b, lb, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_seqs + la + lb, c, lc, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_off, off, sizeof(off), hipMemcpyHostToDevice, s));
  rc = plane_launch_batch(d_seqs, d_off, 1, la, lb, lc, kp, d_small, d_small + 1, d_ws, ws_bytes,
                          s, d_tb);
  if (rc) goto done;
  hipLaunchKernelGGL(tb_walk, dim3(1), dim3(64), 0, s, d_tb, d_small + 1, la, lb, lc, d_moves,
                     d_small + 8);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(h_small, d_small, sizeof(h_small), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (h_small[8] < 1 || h_small[8] > len) {
    rc = TSA_EINTERNAL;
    goto done;
  }
  {
    std::vector<uint8_t> rev((size_t)h_small[8]);
    HIPCHK(hipMemcpy(rev.data(), d_moves, rev.size(), hipMemcpyDeviceToHost));
    for (size_t k = 0; k < rev.size(); ++k) moves[k] = rev[rev.size() - 1 - k];
  }
  *score = h_small[0];
  *n_moves = h_small[8];
  start[0] = h_small[9];
  start[1] = h_small[10];
  start[2] = h_small[11];
done:
  if (d_seqs) (void)hipFree(d_seqs);
  if (d_off) (void)hipFree(d_off);
  if (d_small) (void)hipFree(d_small);
  if (d_moves) (void)hipFree(d_moves);
  if (d_ws) (void)hipFree(d_ws);
  if (d_tb) (void)hipFree(d_tb);
  if (s) (void)hipStreamDestroy(s);
  return rc;
}

int tsa_describe_plan(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                      const tsa_params *p, int32_t kernel, int32_t sync, char *buf, size_t len) {
  if (!buf || len == 0 || n < 1 || max_la < 1 || max_lb < 1 || max_lc < 1 || !params_ok(p))
    return TSA_EINVAL;
  int kind = choose_kernel(kernel, p, max_la, max_lb, max_lc);
  if (kind < 0) return TSA_ERANGE;
  if (sync) kind = upgrade_checked(kind, kernel, n, p, max_la, max_lb, max_lc);
  const LapPolicy lap = sync ? LAP_STREAM : LAP_RESIDENT;
  if (kind == TSA_KERNEL_PLANE) {
    literal_describe(n, max_la, max_lb, max_lc, p->s3_mode == TSA_S3_SOP, lap, buf, len);
    return TSA_OK;
  }
  if (kind == TSA_KERNEL_CHECKED && !checked_plan(n, p, max_la, max_lb, max_lc, lap)) return TSA_ERANGE;
  KParams kp;
  build_kparams(p, &kp);
  pencil_describe(std::min(n, 65535), max_la, max_lb, max_lc, kp,
                  value_bound(p, max_la, max_lb, max_lc), lap, buf, len, kind == TSA_KERNEL_CHECKED);
  return TSA_OK;
}

int tsa_batch_workspace_size(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                             const tsa_params *p, int32_t kernel, size_t *bytes) {
  if (!bytes || n < 0 || max_la < 1 || max_lb < 1 || max_lc < 1 || !params_ok(p)) return TSA_EINVAL;
  if (kernel < TSA_KERNEL_AUTO || kernel > TSA_KERNEL_CHECKED) return TSA_EINVAL;
  const int kind = choose_kernel(kernel, p, max_la, max_lb, max_lc);
  if (kind < 0) return TSA_ERANGE;
  if (kind == TSA_KERNEL_CHECKED && !checked_plan(n, p, max_la, max_lb, max_lc, LAP_RESIDENT))
    return TSA_ERANGE;
  *bytes = workspace_for(kind, n, max_la, max_lb, max_lc, p);
  return TSA_OK;
}

}  // extern "C"

static int score_batch_async(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                             int32_t max_la, int32_t max_lb, int32_t max_lc, const tsa_params *p,
                             int32_t kernel, int32_t *d_scores, void *d_workspace,
                             size_t workspace_bytes, void *stream, int32_t packed) {
  if (!d_seqs || !d_offsets || !d_scores || !d_workspace || n < 0 || max_la < 1 || max_lb < 1 ||
      max_lc < 1 || !params_ok(p))
    return TSA_EINVAL;
  if (kernel < TSA_KERNEL_AUTO || kernel > TSA_KERNEL_CHECKED) return TSA_EINVAL;
  if (tsa_device_count() <= 0) return TSA_ENODEV;
  if (p->score_bits == 0) {
    const Range r = value_bound(p, max_la, max_lb, max_lc);
    if (r.lo < -32768 || r.hi > 32767) return TSA_ERANGE;
  }
  const int kind = choose_kernel(kernel, p, max_la, max_lb, max_lc);
  if (kind < 0) return TSA_ERANGE;
  if (kind == TSA_KERNEL_CHECKED && !checked_plan(n, p, max_la, max_lb, max_lc, LAP_RESIDENT))
    return TSA_ERANGE;
  if (workspace_bytes < workspace_for(kind, n, max_la, max_lb, max_lc, p)) return TSA_ENOMEM;
  hipStream_t s = (hipStream_t)stream;
  for (int32_t c0 = 0; c0 < n; c0 += 65535) {
    const int32_t cn = std::min<int32_t>(65535, n - c0);
    int rc = launch_kind(kind, d_seqs, d_offsets + 3 * (int64_t)c0, cn, max_la, max_lb, max_lc, p,
                         d_scores + c0, nullptr, d_workspace, workspace_bytes, s, LAP_RESIDENT, nullptr, packed,
                         std::min<int32_t>(n, 65535));
    if (rc) return rc;
  }
  return TSA_OK;
}

extern "C" {

int tsa_score_batch_async(const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                          int32_t max_la, int32_t max_lb, int32_t max_lc, const tsa_params *p,
                          int32_t kernel, int32_t *d_scores, void *d_workspace,
                          size_t workspace_bytes, void *stream) {
  return score_batch_async(d_seqs, d_offsets, n, max_la, max_lb, max_lc, p, kernel, d_scores,
                           d_workspace, workspace_bytes, stream, 0);
}

int tsa_score_batch_async_p2(const uint8_t *d_packed, const int64_t *d_offsets, int32_t n,
                             int32_t max_la, int32_t max_lb, int32_t max_lc, const tsa_params *p,
                             int32_t kernel, int32_t *d_scores, void *d_workspace,
                             size_t workspace_bytes, void *stream) {
  return score_batch_async(d_packed, d_offsets, n, max_la, max_lb, max_lc, p, kernel, d_scores,
                           d_workspace, workspace_bytes, stream, 1);
}

int tsa_pack2(const uint8_t *syms, int64_t n, uint8_t *out) {
  if ((!syms || !out) && n > 0) return TSA_EINVAL;
  if (n < 0) return TSA_EINVAL;
  for (int64_t i = 0; i < n; ++i)
    if (syms[i] > 4) return TSA_EINVAL;
  for (int64_t j = 0; j < (n + 3) / 4; ++j) {
    uint8_t v = 0;
    for (int k = 0; k < 4 && 4 * j + k < n; ++k) v |= (uint8_t)((syms[4 * j + k] & 3) << (2 * k));
    out[j] = v;
  }
  return TSA_OK;
}

}  // extern "C"
