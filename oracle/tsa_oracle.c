/*
 * tsa_oracle.c -- CPU restatement of the TriAlign RTL arithmetic.
 * TEST INFRASTRUCTURE ONLY (checker + CPU baseline). See tsa_oracle.h.
 *
 * Reference anchors (paths relative to the reference root):
 *   MAX7 signed 7-way max .................. src/PE_1cyc.v:1-32
 *   MATCH/MISMATCH/GO/GE, GO2/GE2/GOGE ...... src/PE_1cyc.v:55-61
 *   2-bit symbol registers (symbols & 3) .... src/PE_1cyc.v:63-66
 *   temp_AB/BC/AC, temp_ABC ................. src/PE_1cyc.v:159-162
 *   M candidates (diag x-1,y-1,z-1, +s3) .... src/PE_1cyc.v:164-170
 *   Ix candidates (x-1,y,z) ................. src/PE_1cyc.v:172-178
 *   Iy candidates (x,y-1,z) ................. src/PE_1cyc.v:180-186
 *   Iz candidates (x,y,z-1) ................. src/PE_1cyc.v:188-194
 *   Ixy candidates (x-1,y-1,z, +s2ab) ....... src/PE_1cyc.v:196-202
 *   Iyz candidates (x,y-1,z-1, +s2bc) ....... src/PE_1cyc.v:204-210
 *   Ixz candidates (x-1,y,z-1, +s2ac) ....... src/PE_1cyc.v:212-218
 *   x = 0 gating (EN_i==1&&EN==0 -> 0) ...... src/PE_1cyc.v:164-178,196-202,212-218
 *   y = 0 / z = 0 / corner faces = 0 ........ src/TriAlign_1cyc.v:155-182
 *   final MAX7 at (LA,LB,LC) ................ src/TriAlign_1cyc.v:141-142,342-345
 *   wordsize = SCORE_BITS = 12 .............. src/TriAlign_tb.sv:56, TriAlign_1cyc.v:6,37
 * Which neighbour feeds which state follows from the PE delay registers
 * (src/PE_1cyc.v:247-299) and the array wiring (src/TriAlign_1cyc.v:118-123);
 * SURVEY.md 3(b) has the derivation and oracle/rtl_model.c re-executes it.
 */
#define _POSIX_C_SOURCE 200809L
#include "tsa_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

double tsao_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* Two's-complement wrap to `bits` (0 = none): the effect of assigning a wider
 * expression to a wordsize-wide wire (src/PE_1cyc.v:127-133). */
static inline int32_t wrapv(int64_t v, int bits) {
  if (bits == 0) return (int32_t)v;
  uint32_t u = (uint32_t)v << (32 - bits);
  return (int32_t)u >> (32 - bits);
}

void tsao_penalty_table(const tsa_params *p, int32_t P[7][7]) {
  const int32_t GO = p->gap_open, GE = p->gap_extend;
  const int32_t GO2 = 2 * GO, GE2 = 2 * GE, GOGE = GO + GE;
  /* columns: source M, Ix, Iy, Iz, Ixy, Iyz, Ixz */
  const int32_t t[7][7] = {
      {0, 0, 0, 0, 0, 0, 0},                 /* M   src/PE_1cyc.v:164-170 */
      {GO2, GE2, GOGE, GOGE, GOGE, GO2, GOGE}, /* Ix  src/PE_1cyc.v:172-178 */
      {GO2, GOGE, GE2, GOGE, GOGE, GOGE, GO2}, /* Iy  src/PE_1cyc.v:180-186 */
      {GO2, GOGE, GOGE, GE2, GO2, GOGE, GOGE}, /* Iz  src/PE_1cyc.v:188-194 */
      {GO, GE, GE, GO, GE, GO, GO},            /* Ixy src/PE_1cyc.v:196-202 */
      {GO, GO, GE, GE, GO, GE, GO},            /* Iyz src/PE_1cyc.v:204-210 */
      {GO, GE, GO, GE, GO, GO, GE},            /* Ixz src/PE_1cyc.v:212-218 */
  };
  memcpy(P, t, sizeof(t));
}

int32_t tsao_s2(int p, int q, const tsa_params *prm) {
  return ((p & 3) == (q & 3)) ? prm->match : prm->mismatch; /* PE_1cyc.v:159-161 */
}

int32_t tsao_s3(int a, int b, int c, const tsa_params *prm) {
  a &= 3;
  b &= 3;
  c &= 3;
  if (prm->s3_mode == TSA_S3_SOP)
    return tsao_s2(a, b, prm) + tsao_s2(b, c, prm) + tsao_s2(a, c, prm);
  /* src/PE_1cyc.v:162: (A==B)?(B==C)?(A==C)?MATCH*3:(MATCH<<1+MISMATCH)
   *                     :(MATCH+MISMATCH<<1):MISMATCH*3
   * Verilog '+' binds tighter than '<<'. The A==C-false arm is unreachable. */
  if (a == b) {
    if (b == c) return 3 * prm->match;
    return (prm->match + prm->mismatch) * 2; /* (MATCH+MISMATCH)<<1 */
  }
  return 3 * prm->mismatch;
}

static int check_args(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                      const uint8_t *c, int32_t lc, const tsa_params *p) {
  if (!a || !b || !c || !p) return TSA_EINVAL;
  if (la < 1 || lb < 1 || lc < 1) return TSA_EINVAL;
  if (p->score_bits != 0 && (p->score_bits < 4 || p->score_bits > 31)) return TSA_EINVAL;
  if (p->s3_mode != TSA_S3_RTL && p->s3_mode != TSA_S3_SOP) return TSA_EINVAL;
  for (int32_t i = 0; i < la; ++i) if (a[i] > 4) return TSA_EINVAL;
  for (int32_t i = 0; i < lb; ++i) if (b[i] > 4) return TSA_EINVAL;
  for (int32_t i = 0; i < lc; ++i) if (c[i] > 4) return TSA_EINVAL;
  return TSA_OK;
}

/* MAX7 over 7 candidates; the RTL's comparator tree (src/PE_1cyc.v:22-28)
 * returns the numeric maximum, so the grouping does not matter here. */
static inline int32_t max7w(const int32_t *s, const int32_t *pen, int32_t add, int bits) {
  int32_t m = wrapv((int64_t)s[0] - pen[0] + add, bits);
  for (int k = 1; k < 7; ++k) {
    int32_t v = wrapv((int64_t)s[k] - pen[k] + add, bits);
    if (v > m) m = v;
  }
  return m;
}

/* One DP cell, literal RTL form. Each pointer is the 7-state tuple of the
 * predecessor the RTL wires into that target. */
static inline void cell_literal(const int32_t *pm, const int32_t *px, const int32_t *py,
                                const int32_t *pz, const int32_t *pxy, const int32_t *pyz,
                                const int32_t *pxz, int32_t sc3, int32_t sab, int32_t sbc,
                                int32_t sac, const int32_t P[7][7], int bits, int32_t *out) {
  out[TSAO_M] = max7w(pm, P[TSAO_M], sc3, bits);
  out[TSAO_IX] = max7w(px, P[TSAO_IX], 0, bits);
  out[TSAO_IY] = max7w(py, P[TSAO_IY], 0, bits);
  out[TSAO_IZ] = max7w(pz, P[TSAO_IZ], 0, bits);
  out[TSAO_IXY] = max7w(pxy, P[TSAO_IXY], sab, bits);
  out[TSAO_IYZ] = max7w(pyz, P[TSAO_IYZ], sbc, bits);
  out[TSAO_IXZ] = max7w(pxz, P[TSAO_IXZ], sac, bits);
}

static inline int32_t best7(const int32_t *s) {
  int32_t m = s[0];
  for (int k = 1; k < 7; ++k) if (s[k] > m) m = s[k];
  return m;
}

int tsao_score_xplane(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                      const uint8_t *c, int32_t lc, const tsa_params *p,
                      int32_t *score, int32_t *final7) {
  int rc = check_args(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  if (!score) return TSA_EINVAL;
  const int bits = p->score_bits;
  int32_t P[7][7];
  tsao_penalty_table(p, P);
  const size_t W = (size_t)lc + 1, H = (size_t)lb + 1;
  const size_t plane = W * H * 7;
  int32_t *prev = (int32_t *)calloc(plane, sizeof(int32_t)); /* x-1; x=0 face = 0 */
  int32_t *cur = (int32_t *)calloc(plane, sizeof(int32_t));  /* y=0/z=0 faces stay 0 */
  if (!prev || !cur) { free(prev); free(cur); return TSA_ENOMEM; }
  /* per-(b,c) pair score, constant over x */
  int32_t s2bc_tab[4][4];
  for (int u = 0; u < 4; ++u)
    for (int v = 0; v < 4; ++v) s2bc_tab[u][v] = wrapv(tsao_s2(u, v, p), bits);
  int32_t s3_tab[4][4][4], s2_tab[4][4];
  for (int u = 0; u < 4; ++u)
    for (int v = 0; v < 4; ++v) {
      s2_tab[u][v] = wrapv(tsao_s2(u, v, p), bits);
      for (int w = 0; w < 4; ++w) s3_tab[u][v][w] = wrapv(tsao_s3(u, v, w, p), bits);
    }
  for (int32_t x = 1; x <= la; ++x) {
    const int ax = a[x - 1] & 3;
    for (int32_t y = 1; y <= lb; ++y) {
      const int by = b[y - 1] & 3;
      const int32_t sab = s2_tab[ax][by];
      const int32_t *prow = prev + (size_t)y * W * 7, *prow1 = prev + (size_t)(y - 1) * W * 7;
      int32_t *crow = cur + (size_t)y * W * 7;
      const int32_t *crow1 = cur + (size_t)(y - 1) * W * 7;
      for (int32_t z = 1; z <= lc; ++z) {
        const int cz = c[z - 1] & 3;
        cell_literal(prow1 + (z - 1) * 7, /* M   (x-1,y-1,z-1) */
                     prow + z * 7,        /* Ix  (x-1,y,  z  ) */
                     crow1 + z * 7,       /* Iy  (x,  y-1,z  ) */
                     crow + (z - 1) * 7,  /* Iz  (x,  y,  z-1) */
                     prow1 + z * 7,       /* Ixy (x-1,y-1,z  ) */
                     crow1 + (z - 1) * 7, /* Iyz (x,  y-1,z-1) */
                     prow + (z - 1) * 7,  /* Ixz (x-1,y,  z-1) */
                     s3_tab[ax][by][cz], sab, s2bc_tab[by][cz], s2_tab[ax][cz], P, bits,
                     crow + z * 7);
      }
    }
    int32_t *t = prev;
    prev = cur;
    cur = t;
  }
  const int32_t *fin = prev + ((size_t)lb * W + (size_t)lc) * 7;
  *score = best7(fin); /* FINAL_MAX, src/TriAlign_1cyc.v:141-142 */
  if (final7) memcpy(final7, fin, 7 * sizeof(int32_t));
  free(prev);
  free(cur);
  return TSA_OK;
}

int tsao_score_diag(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                    const uint8_t *c, int32_t lc, const tsa_params *p,
                    int32_t *score, int32_t *final7) {
  int rc = check_args(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  if (!score) return TSA_EINVAL;
  const int bits = p->score_bits;
  int32_t P[7][7];
  tsao_penalty_table(p, P);
  const size_t W = (size_t)lc + 1, H = (size_t)lb + 1;
  const size_t plane = W * H * 7;
  /* ring of 4 planes indexed by q & 3; entry (y,z) of plane q is cell
   * (q-y-z, y, z). Faces (any coordinate 0) read as the zero tuple. */
  int32_t *ring = (int32_t *)calloc(4 * plane, sizeof(int32_t));
  if (!ring) return TSA_ENOMEM;
  static const int32_t zero7[7] = {0, 0, 0, 0, 0, 0, 0};
#define PL(q) (ring + (size_t)((q) & 3) * plane)
#define AT(q, y, z) (((y) == 0 || (z) == 0 || (q) - (y) - (z) == 0) ? zero7 : PL(q) + ((size_t)(y) * W + (size_t)(z)) * 7)
  const int32_t qmax = la + lb + lc;
  for (int32_t q = 3; q <= qmax; ++q) {
    int32_t *cp = PL(q);
    int32_t ylo = q - la - lc; if (ylo < 1) ylo = 1;
    int32_t yhi = q - 2; if (yhi > lb) yhi = lb;
    for (int32_t y = ylo; y <= yhi; ++y) {
      int32_t zlo = q - la - y; if (zlo < 1) zlo = 1;
      int32_t zhi = q - 1 - y; if (zhi > lc) zhi = lc;
      for (int32_t z = zlo; z <= zhi; ++z) {
        const int32_t x = q - y - z;
        const int ax = a[x - 1] & 3, by = b[y - 1] & 3, cz = c[z - 1] & 3;
        cell_literal(AT(q - 3, y - 1, z - 1), AT(q - 1, y, z), AT(q - 1, y - 1, z),
                     AT(q - 1, y, z - 1), AT(q - 2, y - 1, z), AT(q - 2, y - 1, z - 1),
                     AT(q - 2, y, z - 1), wrapv(tsao_s3(ax, by, cz, p), bits),
                     wrapv(tsao_s2(ax, by, p), bits), wrapv(tsao_s2(by, cz, p), bits),
                     wrapv(tsao_s2(ax, cz, p), bits), P, bits,
                     cp + ((size_t)y * W + (size_t)z) * 7);
      }
    }
  }
  const int32_t *fin = PL(qmax) + ((size_t)lb * W + (size_t)lc) * 7;
  *score = best7(fin);
  if (final7) memcpy(final7, fin, 7 * sizeof(int32_t));
#undef AT
#undef PL
  free(ring);
  return TSA_OK;
}

/* ---- traceback (extension; no RTL counterpart) ------------------------------
 * The path behind the score: the whole cube of literal (wrapped) states is
 * kept, then walked back from (la,lb,lc), recomputing each state's 7 wrapped
 * candidates and taking the lowest source index that achieves it (the final
 * MAX7 likewise). Moves are state indices, forward order; start = the face
 * cell the path leaves. Independent of the GPU's pointer cube by design. */
int tsao_align(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
               int32_t lc, const tsa_params *p, int32_t *score, uint8_t *moves,
               int32_t max_moves, int32_t *n_moves, int32_t *start) {
  int rc = check_args(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  if (!score || !moves || !n_moves || !start) return TSA_EINVAL;
  if ((int64_t)max_moves < (int64_t)la + lb + lc) return TSA_EINVAL;
  const int bits = p->score_bits;
  int32_t P[7][7];
  tsao_penalty_table(p, P);
  const size_t W = (size_t)lc + 1, H = (size_t)lb + 1, D = (size_t)la + 1;
  if (D * H * W > ((size_t)1 << 26)) return TSA_ENOMEM; /* test sizes only */
  int32_t *cube = (int32_t *)calloc(D * H * W * 7, sizeof(int32_t)); /* faces stay 0 */
  if (!cube) return TSA_ENOMEM;
#define CELL(x, y, z) (cube + (((size_t)(x) * H + (size_t)(y)) * W + (size_t)(z)) * 7)
  for (int32_t x = 1; x <= la; ++x)
    for (int32_t y = 1; y <= lb; ++y)
      for (int32_t z = 1; z <= lc; ++z) {
        const int ax = a[x - 1] & 3, by = b[y - 1] & 3, cz = c[z - 1] & 3;
        cell_literal(CELL(x - 1, y - 1, z - 1), CELL(x - 1, y, z), CELL(x, y - 1, z),
                     CELL(x, y, z - 1), CELL(x - 1, y - 1, z), CELL(x, y - 1, z - 1),
                     CELL(x - 1, y, z - 1), wrapv(tsao_s3(ax, by, cz, p), bits),
                     wrapv(tsao_s2(ax, by, p), bits), wrapv(tsao_s2(by, cz, p), bits),
                     wrapv(tsao_s2(ax, cz, p), bits), P, bits, CELL(x, y, z));
      }
  static const int DX[7] = {1, 1, 0, 0, 1, 0, 1}, DY[7] = {1, 0, 1, 0, 1, 1, 0},
                   DZ[7] = {1, 0, 0, 1, 0, 1, 1};
  const int32_t *fin = CELL(la, lb, lc);
  int T = 0;
  for (int s = 1; s < 7; ++s) if (fin[s] > fin[T]) T = s;
  *score = fin[T];
  int32_t x = la, y = lb, z = lc, n = 0;
  for (;;) {
    moves[n++] = (uint8_t)T;
    const int32_t px = x - DX[T], py = y - DY[T], pz = z - DZ[T];
    if (px == 0 || py == 0 || pz == 0) { x = px; y = py; z = pz; break; }
    const int ax = a[x - 1] & 3, by = b[y - 1] & 3, cz = c[z - 1] & 3;
    int32_t add = 0;
    if (T == TSAO_M) add = wrapv(tsao_s3(ax, by, cz, p), bits);
    else if (T == TSAO_IXY) add = wrapv(tsao_s2(ax, by, p), bits);
    else if (T == TSAO_IYZ) add = wrapv(tsao_s2(by, cz, p), bits);
    else if (T == TSAO_IXZ) add = wrapv(tsao_s2(ax, cz, p), bits);
    const int32_t *pr = CELL(px, py, pz), target = CELL(x, y, z)[T];
    int src = -1;
    for (int s = 0; s < 7 && src < 0; ++s)
      if (wrapv((int64_t)pr[s] - P[T][s] + add, bits) == target) src = s;
    if (src < 0) { free(cube); return TSA_EINTERNAL; }
    x = px; y = py; z = pz;
    T = src;
  }
#undef CELL
  for (int32_t k = 0; k < n / 2; ++k) { /* forward order */
    const uint8_t t = moves[k];
    moves[k] = moves[n - 1 - k];
    moves[n - 1 - k] = t;
  }
  *n_moves = n;
  start[0] = x; start[1] = y; start[2] = z;
  free(cube);
  return TSA_OK;
}

/* ---- factored message form ------------------------------------------------
 * A cell with states S sends to each successor target T the value
 *   msg_T = max_s (S[s] - P[T][s]);
 * the successor adds its pair/triple score. With no wrap this equals the
 * literal MAX7 since max_s(S[s]-P+k) = max_s(S[s]-P)+k. Messages kept per
 * cell: [0]=best(->M) [1]=->Ix [2]=->Iy [3]=->Iz [4]=->Ixy [5]=->Iyz [6]=->Ixz.
 */
static inline void make_msgs(const int32_t *S, const int32_t P[7][7], int32_t *m) {
  for (int t = 0; t < 7; ++t) {
    int32_t v = S[0] - P[t][0];
    for (int s = 1; s < 7; ++s) {
      int32_t w = S[s] - P[t][s];
      if (w > v) v = w;
    }
    m[t] = v;
  }
}

static int msg_sweep(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                     const uint8_t *c, int32_t lc, const tsa_params *p, int32_t *score,
                     int32_t *lo_out, int32_t *hi_out) {
  int32_t P[7][7];
  tsao_penalty_table(p, P);
  tsa_params pw = *p;
  pw.score_bits = 0;
  const size_t W = (size_t)lc + 1, H = (size_t)lb + 1;
  const size_t plane = W * H * 7;
  int32_t *prev = (int32_t *)malloc(plane * sizeof(int32_t));
  int32_t *cur = (int32_t *)malloc(plane * sizeof(int32_t));
  if (!prev || !cur) { free(prev); free(cur); return TSA_ENOMEM; }
  int32_t face[7];
  static const int32_t zero7[7] = {0, 0, 0, 0, 0, 0, 0};
  make_msgs(zero7, P, face); /* every face cell has all-zero states */
  for (size_t i = 0; i < W * H; ++i) { memcpy(prev + i * 7, face, sizeof(face)); memcpy(cur + i * 7, face, sizeof(face)); }
  int32_t lo = 0, hi = 0, S[7], lastS[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int32_t x = 1; x <= la; ++x) {
    const int ax = a[x - 1] & 3;
    for (int32_t y = 1; y <= lb; ++y) {
      const int by = b[y - 1] & 3;
      for (int32_t z = 1; z <= lc; ++z) {
        const int cz = c[z - 1] & 3;
        const int32_t *mm = prev + ((size_t)(y - 1) * W + (z - 1)) * 7;
        const int32_t *mx = prev + ((size_t)y * W + z) * 7;
        const int32_t *my = cur + ((size_t)(y - 1) * W + z) * 7;
        const int32_t *mz = cur + ((size_t)y * W + (z - 1)) * 7;
        const int32_t *mxy = prev + ((size_t)(y - 1) * W + z) * 7;
        const int32_t *myz = cur + ((size_t)(y - 1) * W + (z - 1)) * 7;
        const int32_t *mxz = prev + ((size_t)y * W + (z - 1)) * 7;
        S[TSAO_M] = mm[0] + tsao_s3(ax, by, cz, &pw);
        S[TSAO_IX] = mx[1];
        S[TSAO_IY] = my[2];
        S[TSAO_IZ] = mz[3];
        S[TSAO_IXY] = mxy[4] + tsao_s2(ax, by, &pw);
        S[TSAO_IYZ] = myz[5] + tsao_s2(by, cz, &pw);
        S[TSAO_IXZ] = mxz[6] + tsao_s2(ax, cz, &pw);
        for (int k = 0; k < 7; ++k) {
          if (S[k] < lo) lo = S[k];
          if (S[k] > hi) hi = S[k];
        }
        make_msgs(S, P, cur + ((size_t)y * W + z) * 7);
        if (x == la && y == lb && z == lc) memcpy(lastS, S, sizeof(S));
      }
    }
    int32_t *t = prev;
    prev = cur;
    cur = t;
  }
  if (score) *score = best7(lastS);
  if (lo_out) *lo_out = lo;
  if (hi_out) *hi_out = hi;
  free(prev);
  free(cur);
  return TSA_OK;
}

int tsao_score_msg(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                   const uint8_t *c, int32_t lc, const tsa_params *p, int32_t *score) {
  int rc = check_args(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  if (!score) return TSA_EINVAL;
  return msg_sweep(a, la, b, lb, c, lc, p, score, NULL, NULL);
}

int tsao_state_range(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                     const uint8_t *c, int32_t lc, const tsa_params *p, int32_t *lo,
                     int32_t *hi) {
  int rc = check_args(a, la, b, lb, c, lc, p);
  if (rc) return rc;
  if (!lo || !hi) return TSA_EINVAL;
  return msg_sweep(a, la, b, lb, c, lc, p, NULL, lo, hi);
}

/* ---- batch over POSIX threads -------------------------------------------- */
typedef struct {
  const uint8_t *seqs;
  const int64_t *off;
  int32_t n, tid, nthreads;
  const tsa_params *p;
  int32_t *scores;
  int rc;
} batch_job;

static void *batch_worker(void *arg) {
  batch_job *j = (batch_job *)arg;
  j->rc = TSA_OK;
  for (int32_t i = j->tid; i < j->n; i += j->nthreads) {
    const int64_t *o = j->off + 3 * (int64_t)i;
    int rc = tsao_score_xplane(j->seqs + o[0], (int32_t)(o[1] - o[0]), j->seqs + o[1],
                               (int32_t)(o[2] - o[1]), j->seqs + o[2], (int32_t)(o[3] - o[2]),
                               j->p, &j->scores[i], NULL);
    if (rc) { j->rc = rc; break; }
  }
  return NULL;
}

int tsao_score_batch(const uint8_t *seqs, const int64_t *offsets, int32_t n,
                     const tsa_params *p, int32_t *scores, int32_t nthreads) {
  if (!seqs || !offsets || !p || !scores || n < 0) return TSA_EINVAL;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > n && n > 0) nthreads = n;
  batch_job *jobs = (batch_job *)calloc((size_t)nthreads, sizeof(batch_job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!jobs || !th) { free(jobs); free(th); return TSA_ENOMEM; }
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (batch_job){seqs, offsets, n, t, nthreads, p, scores, 0};
    pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  int rc = TSA_OK;
  for (int t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc && !rc) rc = jobs[t].rc;
  }
  free(jobs);
  free(th);
  return rc;
}

/* ---- synthetic inputs ----------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void tsao_gen_uniform(uint64_t seed, uint8_t *out, int32_t len) {
  uint64_t s = seed, w = 0;
  for (int32_t i = 0; i < len; ++i) {
    if ((i & 31) == 0) w = splitmix64(&s);
    out[i] = (uint8_t)((w >> (2 * (i & 31))) & 3);
  }
}
