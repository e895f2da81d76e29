/*
 * rtl_common.h -- pieces shared by the two cycle-level RTL models:
 * oracle/rtl_model.c (TRIALIGN_1cyc + PE_1cyc) and oracle/rtl_model_2cyc.c
 * (TRIALIGN_2cyc + PE_2cyc). TEST INFRASTRUCTURE ONLY.
 *
 * Values carry an X flag (XV): any arithmetic or comparison touching an X
 * yields X, so a score that depends on anything the RTL leaves undefined
 * comes back flagged.
 */
#pragma once
#include <stdint.h>

#define XV INT32_MIN /* the X / z value */
#define PE_LEN 8
#define WS 12 /* SCORE_BITS = wordsize (src/TriAlign_tb.sv:56) */

static inline int32_t w12(int64_t v) {
  uint32_t u = (uint32_t)v << (32 - WS);
  return (int32_t)u >> (32 - WS);
}
static inline int32_t addx(int32_t a, int32_t b) { return (a == XV || b == XV) ? XV : w12((int64_t)a + b); }
static inline int32_t max2x(int32_t a, int32_t b) { return (a == XV || b == XV) ? XV : (a > b ? a : b); }
/* MAX7 with the RTL's port grouping (src/PE_1cyc.v:22-28 == src/PE_2cyc.v:22-28). */
static inline int32_t max7x(int32_t g4, int32_t g2a, int32_t g2b, int32_t g3a, int32_t g1a,
                            int32_t g1b, int32_t g3b) {
  int32_t t1 = max2x(g1a, g1b), t2 = max2x(g2a, g2b), t3 = max2x(g3a, g3b);
  return max2x(max2x(t1, t2), max2x(t3, g4));
}

typedef struct { int32_t s[7]; } st7; /* {M,Ix,Iy,Iz,Ixy,Iyz,Ixz} */
static const st7 ZERO7 = {{0, 0, 0, 0, 0, 0, 0}};
static const st7 X7 = {{XV, XV, XV, XV, XV, XV, XV}};

/* The 49 MAX7 inputs of one PE (src/PE_1cyc.v:159-218; the same expressions
 * in src/PE_2cyc.v:182-241), cand[target][port] in MAX7 port order
 * {G4, G2_A, G2_B, G3_A, G1_A, G1_B, G3_B} of the MAX7 instance of each
 * target. own = the PE's state registers, d12 = *_1_d2, d11 = *_1_d1,
 * d21 = *_2_d1, d31 = *_3_d1, i2 / i3 = the (y-1) / (z-1) neighbour outputs,
 * gate = (EN_i == 1 && EN == 0). */
static inline void pe_cands(int32_t A, int32_t B, int32_t C, int gate, const st7 *own,
                            const st7 *d12, const st7 *d11, const st7 *d21, const st7 *d31,
                            const st7 *i2, const st7 *i3, int32_t cand[7][7]) {
  const int32_t MATCH = 1, MISMATCH = -1, GO = 2, GE = 1; /* src/PE_1cyc.v:55-61 */
  const int32_t GO2 = GO << 1, GE2 = GE << 1, GOGE = GO + GE;
  int32_t tAB, tBC, tAC, tABC;
  if (A == XV || B == XV) tAB = XV; else tAB = (A == B) ? MATCH : MISMATCH;
  if (B == XV || C == XV) tBC = XV; else tBC = (B == C) ? MATCH : MISMATCH;
  if (A == XV || C == XV) tAC = XV; else tAC = (A == C) ? MATCH : MISMATCH;
  /* `+` binds tighter than `<<`: 3 / 0 / -3 (src/PE_1cyc.v:162) */
  if (A == XV || B == XV || C == XV) tABC = XV;
  else if (A == B) tABC = (B == C) ? ((A == C) ? MATCH * 3 : (MATCH << (1 + MISMATCH))) : w12((int64_t)(MATCH + MISMATCH) * 2);
  else tABC = w12(MISMATCH * 3);
#define C0(pen, sc) addx(-(pen), (sc))
#define CV(v, pen, sc) addx(addx((v), -(pen)), (sc))
#define G(v, pen, sc) (gate ? C0(pen, sc) : CV(v, pen, sc))
  /* M: G4=M G2=Ixy,Iyz G3=Iz,Ixz G1=Ix,Iy; all from *_1_d2 + temp_ABC */
  int32_t *m = cand[0];
  m[0] = G(d12->s[0], 0, tABC); m[1] = G(d12->s[4], 0, tABC); m[2] = G(d12->s[5], 0, tABC);
  m[3] = G(d12->s[3], 0, tABC); m[4] = G(d12->s[1], 0, tABC); m[5] = G(d12->s[2], 0, tABC);
  m[6] = G(d12->s[6], 0, tABC);
  /* Ix: G4=Ix G2=Ixy,Ixz G3=Iy,Iz G1=M,Iyz; own state */
  int32_t *x = cand[1];
  x[0] = G(own->s[1], GE2, 0); x[1] = G(own->s[4], GOGE, 0); x[2] = G(own->s[6], GOGE, 0);
  x[3] = G(own->s[2], GOGE, 0); x[4] = G(own->s[0], GO2, 0); x[5] = G(own->s[5], GO2, 0);
  x[6] = G(own->s[3], GOGE, 0);
  /* Iy: G4=Iy G2=Ixy,Iyz G3=Ix,Iz G1=M,Ixz; (y-1) outputs, never gated */
  int32_t *y = cand[2];
  y[0] = CV(i2->s[2], GE2, 0); y[1] = CV(i2->s[4], GOGE, 0); y[2] = CV(i2->s[5], GOGE, 0);
  y[3] = CV(i2->s[1], GOGE, 0); y[4] = CV(i2->s[0], GO2, 0); y[5] = CV(i2->s[6], GO2, 0);
  y[6] = CV(i2->s[3], GOGE, 0);
  /* Iz: G4=Iz G2=Ixz,Iyz G3=Ix,Iy G1=M,Ixy; (z-1) outputs, never gated */
  int32_t *z = cand[3];
  z[0] = CV(i3->s[3], GE2, 0); z[1] = CV(i3->s[6], GOGE, 0); z[2] = CV(i3->s[5], GOGE, 0);
  z[3] = CV(i3->s[1], GOGE, 0); z[4] = CV(i3->s[0], GO2, 0); z[5] = CV(i3->s[4], GO2, 0);
  z[6] = CV(i3->s[2], GOGE, 0);
  /* Ixy: G4=Iy G2=Ixy,Ix G3=Iyz,Iz G1=M,Ixz; *_2_d1 + temp_AB */
  int32_t *a = cand[4];
  a[0] = G(d21->s[2], GE, tAB); a[1] = G(d21->s[4], GE, tAB); a[2] = G(d21->s[1], GE, tAB);
  a[3] = G(d21->s[5], GO, tAB); a[4] = G(d21->s[0], GO, tAB); a[5] = G(d21->s[6], GO, tAB);
  a[6] = G(d21->s[3], GO, tAB);
  /* Iyz: G4=Iz G2=Ixz,Ix G3=Iyz,Iy G1=M,Ixy; *_1_d1 + temp_BC, never gated */
  int32_t *b = cand[5];
  b[0] = CV(d11->s[3], GE, tBC); b[1] = CV(d11->s[6], GO, tBC); b[2] = CV(d11->s[1], GO, tBC);
  b[3] = CV(d11->s[5], GE, tBC); b[4] = CV(d11->s[0], GO, tBC); b[5] = CV(d11->s[4], GO, tBC);
  b[6] = CV(d11->s[2], GE, tBC);
  /* Ixz: G4=Iz G2=Ixy,Iyz G3=Ixz,Iy G1=M,Ix; *_3_d1 + temp_AC */
  int32_t *c = cand[6];
  c[0] = G(d31->s[3], GE, tAC); c[1] = G(d31->s[4], GO, tAC); c[2] = G(d31->s[5], GO, tAC);
  c[3] = G(d31->s[6], GE, tAC); c[4] = G(d31->s[0], GO, tAC); c[5] = G(d31->s[1], GE, tAC);
  c[6] = G(d31->s[2], GO, tAC);
#undef G
#undef CV
#undef C0
}

/* The seven MAX7 outputs of a candidate set (state order). */
static inline st7 pe_max(const int32_t cand[7][7]) {
  st7 r;
  for (int t = 0; t < 7; ++t)
    r.s[t] = max7x(cand[t][0], cand[t][1], cand[t][2], cand[t][3], cand[t][4], cand[t][5], cand[t][6]);
  return r;
}

/* Testbench symbol RAM (src/TriAlign_tb.sv:149-169,391-397): defined only
 * where the caller wrote a symbol; 4-bit symbols. */
static inline int32_t tb_symbol(const uint8_t *s, int len, uint32_t addr) {
  if ((int64_t)addr >= len) return XV;
  return (int32_t)(s[addr] & 0xF);
}
