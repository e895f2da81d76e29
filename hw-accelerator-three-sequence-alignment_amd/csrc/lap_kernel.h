// lap_kernel.h -- host interface of the single-cube (lap) schedule
// (lap_kernel.hip), used by the pencil dispatcher (pencil_kernel.hip).
#pragma once

#include "pencil_kernel.h"

namespace tsa {

struct PencilArgs;

// Dispatch rounds of a lap grid (kernel argument): blocks run per XCD in block
// order, SX slots at a time; a producer whose consumer is in a later round
// writes a full-length ring (YRB / ZRB slots) in the boundary regions yb / zb
// (KBY rings per column for y, one per round boundary for z).
struct LapRounds {
  int32_t SX, KBY, YRB, ZRB;
  uint8_t *yb, *zb;
};

struct LapGeom {
  int32_t M, NW;     // packed pairs per lane (tile = 64 M positions), waves (2 NW rows)
  int32_t G, GZ;     // laps, z-tiles
  int32_t NC, CH;    // columns (triple, z-tile) and columns per XCD (blocks = G * CH * 8)
  int32_t YR, ZR;    // slim y / z ring slots per workgroup (powers of 2)
  int32_t SX, KBY, KBZ, YRB, ZRB;  // rounds: slots per XCD, boundary rings (LapRounds)
  int32_t per_cu;    // workgroups a CU holds (per-SIMD register model, occupancy API)
  int64_t blocks;    // logical workgroups (padding blocks for the XCD-aware tile mapping)
  int64_t grid;      // physical grid: one dispatch round (8 SX), each block looping over its rounds
  size_t lds, prog_bytes, yf_bytes, zf_bytes, yb_bytes, zb_bytes;
  int64_t waves;     // dispatch rounds: 1 = every workgroup resident at once
  double est_us;     // estimated latency (lap_geom_chunked: of every launch)
  bool ok;           // feasible and more than one workgroup per triple
  // lap_geom_chunked: a batch runs as launches of `chunk` triples, one after
  // another on the stream (0: one launch); the geometry above is a chunk's
  int32_t chunk;
  int32_t max_la, max_lb, max_lc;
};

// A grid beyond the resident slots runs in rounds: the launch holds one
// round, every workgroup looping over its slots' later rounds in lap order
// (boundary rings keep a producer from waiting on a later round); limited to
// a few (the boundary rings grow with them).
constexpr int64_t LAP_MAX_WAVES = 4;

// Geometry of the lap schedule (M pairs per lane, NW waves) for a batch of n
// triples; full_rings: every ring as long as the cube (no back-pressure: the
// split over devices, whose parts may queue behind each other).
// lit: the literal form (lap_kernel LIT: int16 shifted words, M <= 2).
LapGeom lap_geom(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, int M, int NW,
                 bool full_rings, bool f16, bool sop, bool lit = false);
// A batch of n triples as sequential launches of `chunk` triples each, so
// that every launch's grid keeps to at most LAP_MAX_WAVES rounds: the
// chunk of least total estimated latency (TSA_LAP_CHUNK forces one, tests).
// .ok = false when no chunk size fits.
LapGeom lap_geom_chunked(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc, int M, int NW, bool f16,
                         bool sop, bool lit = false);
size_t lap_workspace_bytes(const LapGeom &g);
// The launch's error word inside a workspace of n triples (set on a hand-off timeout).
uint32_t *lap_err_word(const LapGeom &g, int32_t n, void *d_ws);
// Launch it. d_err (synchronous callers): the error word, cleared before the
// launch, nonzero after it when a hand-off timed out.
// chk (int16 form only): the checked kernel, then a certification pass that
// turns the score of every triple outside *chk into TSA_SCORE_UNCERTIFIED.
int lap_launch(const LapGeom &g, bool f16, bool sop, const uint8_t *d_seqs,
               const int64_t *d_offsets, int32_t n, int32_t *d_scores, void *d_ws,
               const PencilArgs &pa, hipStream_t stream, int32_t **d_err,
               const CheckLimits *chk = nullptr);

// The literal form on a geometry from lap_geom(..., lit = true): the RTL's
// wrapped arithmetic for any parameter set; d_final7 (may be null) receives
// each triple's final 7-tuple {M, Ix, Iy, Iz, Ixy, Iyz, Ixz}. d_err as above.
int lap_launch_lit(const LapGeom &g, bool sop, const uint8_t *d_seqs, const int64_t *d_offsets, int32_t n,
                   int32_t *d_scores, int32_t *d_final7, void *d_ws, const KParams &kp, hipStream_t stream,
                   int32_t **d_err);

// One part of a single cube split over devices by laps (tsa_score_gpu_multi):
// laps [L0, L1) on `device`, with that device's copy of the triple and a
// fine-grained workspace of lap_workspace_bytes(g) (peers write into it).
struct LapPart {
  int device;
  hipStream_t stream;
  int32_t L0, L1;
  const uint8_t *d_seqs;
  const int64_t *d_offsets;
  void *d_ws;
};
// Launch every part (parts in lap order, covering [0, g.G)); d_score and the
// error word d_err (cleared by the caller) are on the last part's device.
int lap_launch_split(const LapGeom &g, bool f16, bool sop, const PencilArgs &pa, const LapPart *parts,
                     int np, int32_t *d_score, uint32_t *d_err);
// The same in the literal arithmetic (lap_kernel LIT, any parameter set), on a
// geometry from literal_split_geom.
int lap_launch_split_lit(const LapGeom &g, bool sop, const KParams &kp, const LapPart *parts, int np,
                         int32_t *d_score, uint32_t *d_err);
LapGeom literal_split_geom(int32_t la, int32_t lb, int32_t lc, bool sop, int np);
// The lap geometry of one (la, lb, lc) cube for an np-way split (.ok = false
// when the factored form has no lap schedule for it or fewer than np laps),
// and its launch (arithmetic chosen as pencil_launch_batch would).
LapGeom pencil_split_geom(int32_t la, int32_t lb, int32_t lc, const KParams &kp, const Range &bound,
                          int np);
int pencil_launch_split(const LapGeom &g, const KParams &kp, const Range &bound, const LapPart *parts,
                        int np, int32_t *d_score, uint32_t *d_err);

}  // namespace tsa
