/*
 * rtl_model_2cyc.c -- cycle-level C model of the reference's TRIALIGN_2cyc +
 * PE_2cyc + sram_1024x8_t13 + the testbench's registered symbol RAM (the
 * variant behind the paper's ASIC numbers). TEST INFRASTRUCTURE ONLY: with
 * oracle/rtl_model.c (the 1-cycle variant) it pins the restatement in
 * tsa_oracle.c and records where the two RTL variants agree.
 *
 * Same method as rtl_model.c: every `always @(*)` block is evaluated from the
 * current register values, then every `always @(posedge clk)` block commits at
 * once, SRAMs included; values carry an X flag (rtl_common.h).
 *
 * What differs from the 1-cycle design, and is modelled here:
 *  - PE: the 49 MAX7 inputs are registered (`*_max_*_d`, src/PE_2cyc.v:
 *    134-148,389-491) and the MAX7 reads the registers, so a state is the
 *    MAX7 of inputs two clocks old; A and EN pass two registers (A_d -> A,
 *    EN_d -> EN, :377-384,530-545); the neighbour delay registers latch only
 *    when pp_counter == 1 (:549-640);
 *  - controller: every compute step is a COMPUTE clock followed by a WAIT
 *    clock (src/TriAlign_2cyc.v:364-482); pp_counter is 1 on the WAIT clock;
 *    A_start registers the A symbol (:360,469);
 *  - SRAM control registers shift only on COMPUTE clocks and hold on WAIT
 *    clocks (:520-631); the SRAMs themselves read or write on every clock
 *    with CEN low (:684-712), so a write port writes twice per step;
 *  - the y-face store is 3 groups x 2 x 8 SRAMs (:85-92,141-157): groups 0/1
 *    have 13-bit addresses (index bits [9:5] select a 512-word page), group
 *    2 has 9 (the page bits fall off); an index goes to group 2 when one of
 *    its bits 6..9 is also set in B_idx (:176-180), otherwise to group
 *    idx[4]; idx[3] selects the SRAM pair. The read index starts at 16, the
 *    write index at 0, and both advance by 8 per pencil, wrapping at
 *    A_idx + 8 (:448-450,650-651).
 *
 * Mapping (reference file:line):
 *   MAX7, PE arithmetic ............... src/PE_2cyc.v:1-32,182-241
 *   PE registers ...................... src/PE_2cyc.v:245-640
 *   PE array wiring, borders, A/EN flow src/TriAlign_2cyc.v:119-229
 *   controller ........................ src/TriAlign_2cyc.v:231-484,633-680
 *   SRAM control registers ............ src/TriAlign_2cyc.v:494-631
 *   sram_1024x8_t13 ................... src/TriAlign_2cyc.v:684-712
 *   testbench symbol RAM / start / finish src/TriAlign_tb.sv:149-169,279-353,391-397
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rtl_common.h"
#include "tsa_oracle.h"

enum { IDLE = 0, INITIAL = 1, COMPUTE = 2, OUT = 3, WAIT = 5 };
#define YG 3                       /* y SRAM groups */
#define YDEPTH01 8192              /* 2**(SRAM_ADDR_BITS+4) */
#define ZDEPTH 512                 /* 2**SRAM_ADDR_BITS */
#define YAMASK 0x1FFFu             /* y_A_i is 13 bits */

typedef struct {
  int32_t A, A_d, B, C;            /* 2-bit symbol registers, XV when z/x */
  int EN, EN_d;
  st7 S;                           /* M..Ixz registers */
  st7 d11, d12, d21, d31;          /* *_1_d1, *_1_d2, *_2_d1, *_3_d1 */
  int32_t cd[7][7];                /* registered MAX7 inputs */
} pe2_t;

typedef struct {
  int WEN, CEN;
  uint32_t A;
  st7 Q;
} sram_ctl;

typedef struct {
  const uint8_t *sa, *sb, *sc;
  int la, lb, lc;
  int32_t a_sym, b_sym, c_sym;     /* testbench registered RAM outputs */
  int state;
  uint32_t input_counter, compute_counter, pp_counter, slice_y, slice_z;
  int32_t Bi[PE_LEN + 1][PE_LEN + 1], Ci[PE_LEN + 1][PE_LEN + 1];
  int32_t A_start;
  int EN_start;
  uint32_t y_read_idx, y_write_idx;
  int32_t score_reg;
  int finish;
  uint32_t A_addr, B_addr, C_addr;
  sram_ctl y[YG][2][PE_LEN + 1];   /* [group][pair][k]; SRAMs exist for k = 1..8 */
  sram_ctl z[2][PE_LEN + 1];
  st7 *ymem[YG][2][PE_LEN + 1];
  st7 *zmem[2][PE_LEN + 1];
  pe2_t pe[PE_LEN + 1][PE_LEN + 1];
} rtl2_t;

/* bits 6..9 of an index shared with B_idx select group 2 (src/TriAlign_2cyc.v:178-180) */
static inline int grp_bool(uint32_t idx, uint32_t B_idx) { return (idx & B_idx & 0x3C0u) != 0; }
static inline int grp_of(uint32_t idx, int b) { return b ? 2 : (int)((idx >> 4) & 1u); }
static inline uint32_t page_of(uint32_t idx) { return ((idx >> 5) & 0x1Fu) << 9; }

static void free_rtl2(rtl2_t *R) {
  if (!R) return;
  for (int g = 0; g < YG; ++g)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k <= PE_LEN; ++k) free(R->ymem[g][j][k]);
  for (int g = 0; g < 2; ++g)
    for (int k = 0; k <= PE_LEN; ++k) free(R->zmem[g][k]);
  free(R);
}

int tsao_rtl2_run(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
                  int32_t lc, int32_t *score, int32_t *score_is_x, int64_t *cycles_out) {
  if (!a || !b || !c || !score || la < 1 || lb < 1 || lc < 1) return TSA_EINVAL;
  if (la > ZDEPTH) return TSA_EINVAL;
  rtl2_t *R = (rtl2_t *)calloc(1, sizeof(rtl2_t));
  if (!R) return TSA_ENOMEM;
  R->sa = a; R->sb = b; R->sc = c; R->la = la; R->lb = lb; R->lc = lc;
  for (int g = 0; g < YG; ++g)
    for (int j = 0; j < 2; ++j)
      for (int k = 1; k <= PE_LEN; ++k) {
        const int depth = g < 2 ? YDEPTH01 : ZDEPTH;
        R->ymem[g][j][k] = (st7 *)malloc(sizeof(st7) * depth);
        if (!R->ymem[g][j][k]) { free_rtl2(R); return TSA_ENOMEM; }
        for (int i = 0; i < depth; ++i) R->ymem[g][j][k][i] = X7;
      }
  for (int g = 0; g < 2; ++g)
    for (int k = 1; k <= PE_LEN; ++k) {
      R->zmem[g][k] = (st7 *)malloc(sizeof(st7) * ZDEPTH);
      if (!R->zmem[g][k]) { free_rtl2(R); return TSA_ENOMEM; }
      for (int i = 0; i < ZDEPTH; ++i) R->zmem[g][k][i] = X7;
    }
  /* ---- reset (src/TriAlign_2cyc.v:496-519,634-656; src/PE_2cyc.v:389-439,494-514,540-578) */
  for (int g = 0; g < YG; ++g)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k <= PE_LEN; ++k) R->y[g][j][k] = (sram_ctl){1, 1, 0u, X7};
  for (int g = 0; g < 2; ++g)
    for (int k = 0; k <= PE_LEN; ++k) R->z[g][k] = (sram_ctl){1, 1, 0u, X7};
  for (int y = 0; y <= PE_LEN; ++y)
    for (int z = 0; z <= PE_LEN; ++z) {
      pe2_t *p = &R->pe[y][z];
      p->A = p->A_d = p->B = p->C = XV;
      p->EN = p->EN_d = 0;
      p->S = p->d11 = p->d12 = p->d21 = p->d31 = ZERO7;
      memset(p->cd, 0, sizeof(p->cd));
      R->Bi[y][z] = 0; R->Ci[y][z] = 0;
    }
  R->state = IDLE;
  R->A_start = XV;
  R->y_read_idx = 16;
  R->a_sym = R->b_sym = R->c_sym = XV;
  const uint32_t A_idx = (uint32_t)la, B_idx = (uint32_t)lb, C_idx = (uint32_t)lc;
  const uint32_t slice_y_max_idx = (B_idx / PE_LEN - 1) & 0xFF; /* 8-bit wires :43-47 */
  const uint32_t slice_z_max_idx = (C_idx / PE_LEN - 1) & 0xFF;
  int start_pulse = 1;
  int64_t cyc = 0;
  const int64_t max_cycles = 100000000LL;
  int32_t final_score = XV;
  int done = 0;

  st7 Mo[PE_LEN + 1][PE_LEN + 1];
  int ENo[PE_LEN + 1][PE_LEN + 1];
  int32_t Ao[PE_LEN + 1][PE_LEN + 1];
  pe2_t npe[PE_LEN + 1][PE_LEN + 1];
  sram_ctl ny[YG][2][PE_LEN + 1], nz[2][PE_LEN + 1];

  while (!done && cyc < max_cycles) {
    /* ---------------- combinational ---------------- */
    const uint32_t rd = R->y_read_idx, wr = R->y_write_idx;
    const uint32_t b00 = ((rd == 0) ? (A_idx + 2 * PE_LEN - 1) : (rd - 1)) & 0xFFFu; /* 12-bit wire :72,177 */
    const int b00_b = grp_bool(b00, B_idx), rd_b = grp_bool(rd, B_idx), wr_b = grp_bool(wr, B_idx);
    const int rd_g = grp_of(rd, rd_b), wr_g = grp_of(wr, wr_b), b00_g = grp_of(b00, b00_b);
    const int rd_j = (rd >> 3) & 1, wr_j = (wr >> 3) & 1, b00_j = (b00 >> 3) & 1;
    for (int y = 1; y <= PE_LEN; ++y)
      for (int z = 1; z <= PE_LEN; ++z) {
        const pe2_t *p = &R->pe[y][z];
        Mo[y][z] = p->S;
        if (!p->EN) Mo[y][z].s[0] = XV; /* M_o = EN ? M : z (src/PE_2cyc.v:171) */
        ENo[y][z] = p->EN;
        Ao[y][z] = p->A;
      }
    ENo[1][0] = R->EN_start; /* :183 */
    for (int gi = 1; gi <= PE_LEN; ++gi) { /* z border (:187-196) */
      if (R->slice_y == 0) Mo[0][gi] = ZERO7;
      else Mo[0][gi] = (R->slice_y % 2 == 1) ? R->z[0][gi].Q : R->z[1][gi].Q;
      ENo[0][gi] = ENo[1][gi - 1];
    }
    for (int ge = 1; ge <= PE_LEN; ++ge) /* y border (:197-212) */
      Mo[ge][0] = (R->slice_z == 0) ? ZERO7 : R->y[rd_g][rd_j][ge].Q;
    Mo[0][0] = (R->slice_y == 0 || R->slice_z == 0) ? ZERO7 : R->y[b00_g][b00_j][PE_LEN].Q; /* :213-219 */
    Ao[0][1] = R->A_start; /* :225-228 */
    for (int ge = 2; ge <= PE_LEN; ++ge) Ao[0][ge] = Ao[1][ge - 1];

    /* PE combinational + next state (src/PE_2cyc.v:182-385) */
    for (int ge = 1; ge <= PE_LEN; ++ge)
      for (int gi = 1; gi <= PE_LEN; ++gi) {
        const pe2_t *p = &R->pe[ge][gi];
        pe2_t *n = &npe[ge][gi];
        const int EN_i = ENo[ge - 1][gi];
        const st7 i1 = Mo[ge - 1][gi - 1], i2 = Mo[ge - 1][gi], i3 = Mo[ge][gi - 1];
        pe_cands(p->A, p->B, p->C, EN_i == 1 && p->EN == 0, &p->S, &p->d12, &p->d11, &p->d21,
                 &p->d31, &i2, &i3, n->cd);       /* -> *_max_*_d */
        n->S = pe_max(p->cd);                     /* MAX7 of the registered inputs */
        if (R->pp_counter == 1) {                 /* :580-608 */
          n->d11 = i1; n->d12 = p->d11; n->d21 = i2; n->d31 = i3;
        } else {
          n->d11 = p->d11; n->d12 = p->d12; n->d21 = p->d21; n->d31 = p->d31;
        }
        const int32_t ai = Ao[ge - 1][gi];
        n->A = p->A_d;
        n->A_d = (ai == XV) ? XV : (ai & 3);
        n->B = (R->Bi[ge][gi] == XV) ? XV : (R->Bi[ge][gi] & 3);
        n->C = (R->Ci[ge][gi] == XV) ? XV : (R->Ci[ge][gi] & 3);
        n->EN = p->EN_d;
        n->EN_d = EN_i;
      }
    /* FINAL_MAX on PE(8,8) outputs (:167-168) */
    const st7 f = Mo[PE_LEN][PE_LEN];
    const int32_t final_max_out = max7x(f.s[6], f.s[2], f.s[3], f.s[4], f.s[0], f.s[1], f.s[5]);

    /* ---------------- controller combinational (:231-484) ---------------- */
    int n_state = R->state;
    uint32_t n_ic = R->input_counter, n_cc = R->compute_counter, n_sy = R->slice_y, n_sz = R->slice_z;
    uint32_t n_pp = R->pp_counter;
    int32_t nBi[PE_LEN + 1][PE_LEN + 1], nCi[PE_LEN + 1][PE_LEN + 1];
    memcpy(nBi, R->Bi, sizeof(nBi));
    memcpy(nCi, R->Ci, sizeof(nCi));
    int32_t n_Astart = R->A_start;
    int n_EN_start = R->EN_start;
    memcpy(ny, R->y, sizeof(ny));
    memcpy(nz, R->z, sizeof(nz));
    uint32_t n_yr = rd, n_yw = wr;
    int32_t n_score = R->score_reg;
    int n_finish = R->finish;
    uint32_t nA = R->A_addr, nB = R->B_addr, nC = R->C_addr;
    switch (R->state) {
      case IDLE:
        if (start_pulse) {
          n_state = INITIAL;
          n_ic = 0;
          nz[0][0].A = 0; nz[1][0].A = 0;
          nA = 0; nB = 0; nC = 0;
        }
        break;
      case INITIAL: {
        const uint32_t ic = R->input_counter;
        if (ic >= 1) {
          nBi[(ic - 1) % PE_LEN + 1][(ic - 1) / PE_LEN + 1] = R->b_sym;
          nCi[(ic - 1) % PE_LEN + 1][(ic - 1) / PE_LEN + 1] = R->c_sym;
        }
        for (int j = 1; j <= PE_LEN; ++j) {
          nz[0][j].WEN = (R->slice_y % 2 == 1) ? 1 : 0;
          nz[1][j].WEN = (R->slice_y % 2 == 1) ? 0 : 1;
          nz[0][j].CEN = 0; nz[1][j].CEN = 0;
          nz[0][j].A = 0; nz[1][j].A = 0;
        }
        for (int k = 1; k <= PE_LEN; ++k) {
          ny[rd_g][rd_j][k].WEN = 1; ny[rd_g][rd_j][k].CEN = 0;
          ny[wr_g][wr_j][k].WEN = 0; ny[wr_g][wr_j][k].CEN = 0;
        }
        ny[b00_g][b00_j][PE_LEN].WEN = 1; ny[b00_g][b00_j][PE_LEN].CEN = 0;
        if (ic < PE_LEN * PE_LEN - 1) {
          for (int k = 0; k <= PE_LEN; ++k) ny[rd_g][rd_j][k].A = page_of(rd);
        } else {
          ny[b00_g][b00_j][PE_LEN].A = page_of(b00);
        }
        n_state = (ic == PE_LEN * PE_LEN) ? COMPUTE : INITIAL;
        n_ic = (ic == PE_LEN * PE_LEN) ? 0 : ic + 1;
        nC = (R->B_addr == (R->slice_y + 1) * PE_LEN - 1)
                 ? ((R->C_addr == (R->slice_z + 1) * PE_LEN - 1) ? R->slice_z * PE_LEN : R->C_addr + 1)
                 : R->C_addr;
        nB = (R->B_addr == (R->slice_y + 1) * PE_LEN - 1) ? R->slice_y * PE_LEN : R->B_addr + 1;
        nA = (ic >= PE_LEN * PE_LEN - 1) ? 1 : 0;
        n_cc = 0;
        n_Astart = R->a_sym;
        n_pp = (R->pp_counter == 1) ? 0 : R->pp_counter + 1;
        break;
      }
      case COMPUTE: {
        const uint32_t cc = R->compute_counter;
        if (cc < A_idx - 1) { /* read addresses (:368-390) */
          ny[rd_g][rd_j][1].A = cc + page_of(rd);
          ny[b00_g][b00_j][PE_LEN].A = cc + 1 + page_of(b00);
          if (R->slice_y % 2 == 1) nz[0][1].A = cc; else nz[1][1].A = cc;
        } else if (cc >= A_idx - 1 && cc < A_idx + PE_LEN) {
          ny[rd_g][rd_j][1].A = A_idx - 1 + page_of(rd);
          nz[0][1].A = A_idx - 1;
          nz[1][1].A = A_idx - 1;
        }
        if (cc >= PE_LEN && cc < PE_LEN + A_idx) { /* write addresses (:405-418) */
          if (R->slice_y % 2 == 1) nz[1][1].A = cc - PE_LEN; else nz[0][1].A = cc - PE_LEN;
          ny[wr_g][wr_j][1].A = cc - PE_LEN + page_of(wr);
        } else if (cc >= PE_LEN + A_idx && cc < 2 * PE_LEN + A_idx - 1) { /* :419-429 */
          nz[0][1].CEN = 1;
          nz[1][1].CEN = 1;
          ny[wr_g][wr_j][1].CEN = 1;
        }
        n_state = WAIT;
        n_pp = 1;
        break;
      }
      case WAIT: {
        const uint32_t cc = R->compute_counter;
        n_cc = (cc == 2 * PE_LEN + A_idx - 1) ? 0 : cc + 1;
        n_pp = 0;
        if (cc == 2 * PE_LEN + A_idx - 1) { /* next pencil (:444-465) */
          n_sy = (R->slice_y == slice_y_max_idx) ? 0 : R->slice_y + 1;
          n_sz = (R->slice_y == slice_y_max_idx) ? ((R->slice_z == slice_z_max_idx) ? 0 : R->slice_z + 1) : R->slice_z;
          n_yw = (wr == A_idx + PE_LEN) ? 0 : wr + PE_LEN;
          n_yr = (rd >= A_idx + PE_LEN) ? 0 : rd + PE_LEN;
          n_state = (R->slice_y == slice_y_max_idx && R->slice_z == slice_z_max_idx) ? OUT : INITIAL;
          nA = 0;
          nB = (R->slice_y == slice_y_max_idx) ? 0 : (R->slice_y + 1) * PE_LEN;
          nC = (R->slice_y == slice_y_max_idx) ? ((R->slice_z == slice_z_max_idx) ? 0 : (R->slice_z + 1) * PE_LEN) : R->C_addr;
          if (R->slice_z == slice_z_max_idx && R->slice_y == slice_y_max_idx) {
            n_score = final_max_out;
            n_finish = 1;
          }
        } else {
          if (cc < A_idx - 1) {
            n_Astart = R->a_sym;
            nA = R->A_addr + 1;
          }
          n_state = COMPUTE;
          if (cc == 0) n_EN_start = 1;
          if (cc == A_idx) n_EN_start = 0;
        }
        break;
      }
      default: break; /* OUT */
    }

    /* ---------------- clock edge ---------------- */
    /* SRAMs sample the pre-edge control and data (:704-711) */
    for (int g = 0; g < YG; ++g)
      for (int j = 0; j < 2; ++j)
        for (int k = 1; k <= PE_LEN; ++k) {
          sram_ctl *s = &R->y[g][j][k];
          if (s->CEN != 0) continue;
          const uint32_t addr = g < 2 ? (s->A & YAMASK) : (s->A & (ZDEPTH - 1));
          if (s->WEN == 0) R->ymem[g][j][k][addr] = Mo[k][PE_LEN]; /* y_D_i = PE(k, 8) (:159-165) */
          else s->Q = R->ymem[g][j][k][addr];
        }
    for (int g = 0; g < 2; ++g)
      for (int k = 1; k <= PE_LEN; ++k) {
        sram_ctl *s = &R->z[g][k];
        if (s->CEN != 0) continue;
        const uint32_t addr = s->A & (ZDEPTH - 1);
        if (s->WEN == 0) R->zmem[g][k][addr] = Mo[PE_LEN][k]; /* z_D_wire = PE(8, k) (:136) */
        else s->Q = R->zmem[g][k][addr];
      }
    /* SRAM control registers (:520-631) */
    if (R->state == COMPUTE) {
      sram_ctl old[YG][2][PE_LEN + 1];
      memcpy(old, R->y, sizeof(old));
      for (int g = 0; g < YG; ++g)
        for (int j = 0; j < 2; ++j)
          for (int k = 0; k <= PE_LEN; ++k) {
            sram_ctl *s = &R->y[g][j][k];
            if (g < 2) s->WEN = ny[g][j][k].WEN; /* group 2's WEN holds (:524-529) */
            const int wr_here = k > 1 && (wr_b ? (g == 2 && wr_j == j) : (g == wr_g && wr_j == j));
            const int rd_here = k > 1 && (rd_b ? (g == 2 && rd_j == j) : (g == rd_g && rd_j == j));
            s->CEN = wr_here ? old[g][j][k - 1].CEN : ny[g][j][k].CEN;
            if (wr_b && wr_here) s->A = old[g][j][k - 1].A;
            else if (rd_b && rd_here) s->A = old[g][j][k - 1].A;
            else if (!wr_b && wr_here) s->A = old[g][j][k - 1].A;
            else if (!rd_b && rd_here) s->A = old[g][j][k - 1].A;
            else s->A = ny[g][j][k].A;
            s->A &= YAMASK;
          }
      for (int g = 0; g < 2; ++g) {
        sram_ctl o[PE_LEN + 1];
        memcpy(o, R->z[g], sizeof(o));
        for (int j = 0; j <= PE_LEN; ++j) R->z[g][j].WEN = nz[g][j].WEN;
        R->z[g][1].A = nz[g][1].A & (ZDEPTH - 1);
        R->z[g][1].CEN = nz[g][1].CEN;
        for (int j = 2; j <= PE_LEN; ++j) { R->z[g][j].A = o[j - 1].A; R->z[g][j].CEN = o[j - 1].CEN; }
      }
    } else {
      for (int g = 0; g < YG; ++g)
        for (int j = 0; j < 2; ++j)
          for (int k = 0; k <= PE_LEN; ++k) {
            R->y[g][j][k].WEN = ny[g][j][k].WEN;
            R->y[g][j][k].CEN = ny[g][j][k].CEN;
            R->y[g][j][k].A = ny[g][j][k].A & YAMASK;
          }
      for (int g = 0; g < 2; ++g)
        for (int j = 0; j <= PE_LEN; ++j) {
          R->z[g][j].WEN = nz[g][j].WEN;
          R->z[g][j].CEN = nz[g][j].CEN;
          R->z[g][j].A = nz[g][j].A & (ZDEPTH - 1);
        }
    }
    /* PE registers */
    for (int y = 1; y <= PE_LEN; ++y)
      for (int z = 1; z <= PE_LEN; ++z) R->pe[y][z] = npe[y][z];
    /* testbench registered symbol RAM read (tb:391-397, 163-169) */
    R->a_sym = tb_symbol(R->sa, R->la, R->A_addr);
    R->b_sym = tb_symbol(R->sb, R->lb, R->B_addr);
    R->c_sym = tb_symbol(R->sc, R->lc, R->C_addr);
    /* controller registers (:657-679) */
    R->state = n_state;
    R->input_counter = n_ic & 0xFFF;
    R->compute_counter = n_cc & 0xFFF;
    R->pp_counter = n_pp & 7;
    R->slice_y = n_sy & 0x1FF;
    R->slice_z = n_sz & 0x1FF;
    memcpy(R->Bi, nBi, sizeof(nBi));
    memcpy(R->Ci, nCi, sizeof(nCi));
    R->A_start = n_Astart;
    R->EN_start = n_EN_start;
    R->y_read_idx = n_yr & 0x3FF;
    R->y_write_idx = n_yw & 0x3FF;
    R->score_reg = n_score;
    R->finish = n_finish;
    R->A_addr = nA & 0x7FFF;
    R->B_addr = nB & 0x7FFF;
    R->C_addr = nC & 0x7FFF;
    start_pulse = 0;
    ++cyc;
    if (R->finish) { final_score = R->score_reg; done = 1; }
  }
  *score = (final_score == XV) ? 0 : final_score;
  if (score_is_x) *score_is_x = (final_score == XV) || !done;
  if (cycles_out) *cycles_out = cyc;
  free_rtl2(R);
  return done ? TSA_OK : TSA_EINTERNAL;
}
