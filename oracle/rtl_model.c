/*
 * rtl_model.c -- cycle-level C model of the reference's TRIALIGN_1cyc +
 * PE_1cyc + sram_1024x8_t13 + the testbench's registered symbol RAM.
 * TEST INFRASTRUCTURE ONLY: it pins the restatement in tsa_oracle.c.
 *
 * No Verilog simulator exists in this image, so the RTL cannot
 * be executed as-is. This model re-executes its register transfers one clock
 * at a time: every `always @(*)` block is evaluated from the current register
 * values (blocking order preserved), then every `always @(posedge clk)` block
 * commits at once, SRAMs included. Values carry an X flag: reset-z registers,
 * unwritten SRAM words, symbols outside the caller's sequence, and the PE's
 * `M_o = (EN==1) ? M : 'z` (src/PE_1cyc.v:148) are X, and any arithmetic or
 * comparison touching an X yields X -- so a score that depends on anything the
 * RTL leaves undefined comes back flagged instead of silently agreeing.
 *
 * Mapping (reference file:line):
 *   MAX7 .............................. src/PE_1cyc.v:1-32
 *   PE combinational (scores, 49 cands) src/PE_1cyc.v:159-218
 *   PE state / delay / input registers  src/PE_1cyc.v:222-347,369-430
 *   PE array wiring, borders, A/EN flow src/TriAlign_1cyc.v:115-125,145-190
 *   controller FSM (IDLE/INITIAL/COMPUTE) src/TriAlign_1cyc.v:193-349
 *   SRAM control shift registers ...... src/TriAlign_1cyc.v:361-423
 *   controller registers .............. src/TriAlign_1cyc.v:426-468
 *   sram_1024x8_t13 ................... src/TriAlign_1cyc.v:472-501
 *   testbench symbol RAM (1-cycle pull) src/TriAlign_tb.sv:149-169,391-397
 *   start pulse / finish .............. src/TriAlign_tb.sv:279-333,339-353
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rtl_common.h"
#include "tsa_oracle.h"

typedef struct {
  int32_t A, B, C; /* 2-bit symbol regs, XV when z/x */
  int EN;
  st7 S;                      /* M..Ixz registers */
  st7 d1_1, d2_1, d1_2, d1_3; /* _1_d1, _1_d2, _2_d1, _3_d1 delay registers */
} pe_t;

typedef struct {
  int la, lb, lc, a_total;
  const uint8_t *sa, *sb, *sc;
  /* testbench symbol path: registered RAM word + mux (1-cycle latency) */
  int32_t a_sym, b_sym, c_sym;
  /* controller registers */
  int state;
  uint32_t input_counter, compute_counter, slice_y, slice_z;
  int32_t Bi[PE_LEN + 1][PE_LEN + 1], Ci[PE_LEN + 1][PE_LEN + 1];
  int EN_start;
  uint32_t y_read_idx, y_write_idx;
  int32_t score_reg;
  int finish;
  uint32_t A_addr, B_addr, C_addr;
  /* SRAM control + arrays */
  int ny;                      /* TOTAL_SRAM_Y_LENGTH */
  int *y_WEN, *y_CEN;
  uint32_t *y_A;
  st7 *y_Q, *y_mem;            /* [ny], [ny][512] */
  int z_WEN[2][PE_LEN + 1], z_CEN[2][PE_LEN + 1];
  uint32_t z_A[2][PE_LEN + 1];
  st7 z_Q[2][PE_LEN + 1];
  st7 *z_mem;                  /* [2][PE_LEN+1][512] */
  pe_t pe[PE_LEN + 1][PE_LEN + 1];
} rtl_t;

enum { IDLE = 0, INITIAL = 1, COMPUTE = 2 };
#define SRAM_DEPTH 512 /* 2**SRAM_ADDR_BITS, SRAM_ADDR_BITS = 9 */
#define AMASK 511u

/* PE wire outputs (M_o is z when EN==0, src/PE_1cyc.v:148) */
static inline st7 pe_out(const pe_t *p) {
  st7 o = p->S;
  if (!p->EN) o.s[0] = XV;
  return o;
}

int tsao_rtl_run(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                 const uint8_t *c, int32_t lc, int32_t a_total_len, int32_t *score,
                 int32_t *score_is_x, int64_t *cycles_out) {
  if (!a || !b || !c || !score || la < 1 || lb < 1 || lc < 1) return TSA_EINVAL;
  if (a_total_len < la || a_total_len > SRAM_DEPTH) return TSA_EINVAL;
  rtl_t *R = (rtl_t *)calloc(1, sizeof(rtl_t));
  if (!R) return TSA_ENOMEM;
  R->la = la; R->lb = lb; R->lc = lc; R->a_total = a_total_len;
  R->sa = a; R->sb = b; R->sc = c;
  R->ny = a_total_len + 2 * PE_LEN; /* A_TOTAL_LENGTH + B_LENGTHX2 (src/TriAlign_1cyc.v:44) */
  R->y_WEN = (int *)malloc(sizeof(int) * R->ny);
  R->y_CEN = (int *)malloc(sizeof(int) * R->ny);
  R->y_A = (uint32_t *)malloc(sizeof(uint32_t) * R->ny);
  R->y_Q = (st7 *)malloc(sizeof(st7) * R->ny);
  R->y_mem = (st7 *)malloc(sizeof(st7) * (size_t)R->ny * SRAM_DEPTH);
  R->z_mem = (st7 *)malloc(sizeof(st7) * 2 * (PE_LEN + 1) * SRAM_DEPTH);
  int *nyWEN = (int *)malloc(sizeof(int) * R->ny), *nyCEN = (int *)malloc(sizeof(int) * R->ny);
  uint32_t *nyA = (uint32_t *)malloc(sizeof(uint32_t) * R->ny);
  if (!R->y_WEN || !R->y_CEN || !R->y_A || !R->y_Q || !R->y_mem || !R->z_mem || !nyWEN ||
      !nyCEN || !nyA) {
    free(R->y_WEN); free(R->y_CEN); free(R->y_A); free(R->y_Q); free(R->y_mem);
    free(R->z_mem); free(nyWEN); free(nyCEN); free(nyA); free(R);
    return TSA_ENOMEM;
  }
  /* ---- reset (src/TriAlign_1cyc.v:361-375,426-446; PE_1cyc.v:303-324,369-398) */
  for (int i = 0; i < R->ny; ++i) { R->y_WEN[i] = 1; R->y_CEN[i] = 1; R->y_A[i] = 0; R->y_Q[i] = X7; }
  for (size_t i = 0; i < (size_t)R->ny * SRAM_DEPTH; ++i) R->y_mem[i] = X7;
  for (size_t i = 0; i < 2u * (PE_LEN + 1) * SRAM_DEPTH; ++i) R->z_mem[i] = X7;
  for (int g = 0; g < 2; ++g)
    for (int j = 0; j <= PE_LEN; ++j) { R->z_WEN[g][j] = 1; R->z_CEN[g][j] = 1; R->z_A[g][j] = 0; R->z_Q[g][j] = X7; }
  for (int y = 0; y <= PE_LEN; ++y)
    for (int z = 0; z <= PE_LEN; ++z) {
      R->Bi[y][z] = 0; R->Ci[y][z] = 0;
      pe_t *p = &R->pe[y][z];
      p->A = XV; p->B = XV; p->C = XV; p->EN = 0;
      p->S = ZERO7; p->d1_1 = ZERO7; p->d2_1 = ZERO7; p->d1_2 = ZERO7; p->d1_3 = ZERO7;
    }
  R->state = IDLE;
  R->a_sym = R->b_sym = R->c_sym = XV; /* A_r_RAM not reset in the testbench */
  const uint32_t A_idx = (uint32_t)la, B_idx = (uint32_t)lb, C_idx = (uint32_t)lc;
  const uint32_t slice_y_max_idx = (B_idx / PE_LEN - 1) & 0xFF; /* 8-bit wires :47-51 */
  const uint32_t slice_z_max_idx = (C_idx / PE_LEN - 1) & 0xFF;
  int start_pulse = 1; /* testbench S_IDLE pulses start_ABSW_r once (tb:314-318) */
  int64_t cyc = 0;
  const int64_t max_cycles = 50000000LL;
  int32_t final_score = XV;
  int done = 0;

  st7 Mo[PE_LEN + 1][PE_LEN + 1]; /* PE wire outputs incl. borders */
  int ENo[PE_LEN + 1][PE_LEN + 1];
  int32_t Ao[PE_LEN + 1][PE_LEN + 1];
  pe_t npe[PE_LEN + 1][PE_LEN + 1];

  while (!done && cyc < max_cycles) {
    /* ---------------- combinational evaluation ---------------- */
    const uint32_t border_00 = ((R->y_read_idx == 0) ? (A_idx + 2 * PE_LEN - 1) : (R->y_read_idx - 1)) & 0xFFF;
    for (int y = 1; y <= PE_LEN; ++y)
      for (int z = 1; z <= PE_LEN; ++z) {
        Mo[y][z] = pe_out(&R->pe[y][z]);
        ENo[y][z] = R->pe[y][z].EN;
        Ao[y][z] = R->pe[y][z].A;
      }
    /* borders (src/TriAlign_1cyc.v:152-190) */
    ENo[1][0] = R->EN_start;
    for (int gi = 1; gi <= PE_LEN; ++gi) {
      if (R->slice_y == 0) Mo[0][gi] = ZERO7;
      else Mo[0][gi] = (R->slice_y % 2 == 1) ? R->z_Q[0][gi] : R->z_Q[1][gi];
      ENo[0][gi] = ENo[1][gi - 1];
    }
    for (int ge = 1; ge <= PE_LEN; ++ge) {
      if (R->slice_z == 0) Mo[ge][0] = ZERO7;
      else {
        uint32_t idx = R->y_read_idx + (uint32_t)ge - 1;
        Mo[ge][0] = (idx < (uint32_t)R->ny) ? R->y_Q[idx] : X7;
      }
    }
    if (R->slice_y == 0 || R->slice_z == 0) Mo[0][0] = ZERO7;
    else Mo[0][0] = (border_00 < (uint32_t)R->ny) ? R->y_Q[border_00] : X7;
    Ao[0][1] = R->a_sym;
    for (int ge = 2; ge <= PE_LEN; ++ge) Ao[0][ge] = Ao[1][ge - 1];

    /* PE combinational + next state (src/PE_1cyc.v:159-299) */
    for (int ge = 1; ge <= PE_LEN; ++ge)
      for (int gi = 1; gi <= PE_LEN; ++gi) {
        const pe_t *p = &R->pe[ge][gi];
        pe_t *n = &npe[ge][gi];
        const int EN_i = ENo[ge - 1][gi];
        const st7 i1 = Mo[ge - 1][gi - 1], i2 = Mo[ge - 1][gi], i3 = Mo[ge][gi - 1];
        int32_t cand[7][7];
        pe_cands(p->A, p->B, p->C, EN_i == 1 && p->EN == 0, &p->S, &p->d2_1, &p->d1_1, &p->d1_2,
                 &p->d1_3, &i2, &i3, cand);
        n->S = pe_max(cand);
        /* delay + input registers (247-299) */
        n->d2_1 = p->d1_1;
        n->d1_1 = i1;
        n->d1_2 = i2;
        n->d1_3 = i3;
        n->A = (Ao[ge - 1][gi] == XV) ? XV : (Ao[ge - 1][gi] & 3);
        n->B = (R->Bi[ge][gi] == XV) ? XV : (R->Bi[ge][gi] & 3);
        n->C = (R->Ci[ge][gi] == XV) ? XV : (R->Ci[ge][gi] & 3);
        n->EN = EN_i;
      }
    /* FINAL_MAX on PE(8,8) wires (src/TriAlign_1cyc.v:141-142) */
    const st7 f = Mo[PE_LEN][PE_LEN];
    const int32_t final_max_out = max7x(f.s[6], f.s[2], f.s[3], f.s[4], f.s[0], f.s[1], f.s[5]);

    /* SRAM data inputs (src/TriAlign_1cyc.v:130,138) */
    /* y_D_i[gi*8+ge] = PE(ge+1, 8) outputs; z_D_wire[g][gsz] = PE(8, gsz) outputs */

    /* ---------------- controller combinational (193-349) ---------------- */
    int n_state = R->state;
    uint32_t n_ic = R->input_counter, n_cc = R->compute_counter, n_sy = R->slice_y, n_sz = R->slice_z;
    int32_t nBi[PE_LEN + 1][PE_LEN + 1], nCi[PE_LEN + 1][PE_LEN + 1];
    memcpy(nBi, R->Bi, sizeof(nBi));
    memcpy(nCi, R->Ci, sizeof(nCi));
    int n_EN_start = R->EN_start;
    memcpy(nyWEN, R->y_WEN, sizeof(int) * R->ny);
    memcpy(nyCEN, R->y_CEN, sizeof(int) * R->ny);
    memcpy(nyA, R->y_A, sizeof(uint32_t) * R->ny);
    int nzWEN[2][PE_LEN + 1], nzCEN[2][PE_LEN + 1];
    uint32_t nzA[2][PE_LEN + 1];
    memcpy(nzWEN, R->z_WEN, sizeof(nzWEN));
    memcpy(nzCEN, R->z_CEN, sizeof(nzCEN));
    memcpy(nzA, R->z_A, sizeof(nzA));
    uint32_t n_yr = R->y_read_idx, n_yw = R->y_write_idx;
    int32_t n_score = R->score_reg;
    int n_finish = R->finish;
    uint32_t nA = R->A_addr, nB = R->B_addr, nC = R->C_addr;
#define YSET(arr, idx, val) do { uint32_t _i = (idx); if (_i < (uint32_t)R->ny) (arr)[_i] = (val); } while (0)
    switch (R->state) {
      case IDLE:
        if (start_pulse) {
          n_state = INITIAL;
          n_ic = 0;
          nyA[0] = 0;
          nzA[0][0] = 0;
          nzA[1][0] = 0;
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
          nzWEN[0][j] = (R->slice_y % 2 == 1) ? 1 : 0;
          nzWEN[1][j] = (R->slice_y % 2 == 1) ? 0 : 1;
          nzCEN[0][j] = 0; nzCEN[1][j] = 0;
          nzA[0][j] = 0; nzA[1][j] = 0;
        }
        for (uint32_t i = 0; i < PE_LEN; ++i) {
          YSET(nyWEN, i + R->y_read_idx, 1);
          YSET(nyCEN, i + R->y_read_idx, 0);
          YSET(nyCEN, i + R->y_write_idx, 0);
          YSET(nyWEN, i + R->y_write_idx, 0);
          YSET(nyCEN, border_00, 0);
        }
        if (ic < PE_LEN * PE_LEN) {
          for (int i = 0; i < R->ny; ++i) nyA[i] = 0;
        } else {
          YSET(nyA, border_00, 1u);
        }
        n_state = (ic == PE_LEN * PE_LEN) ? COMPUTE : INITIAL;
        n_ic = (ic == PE_LEN * PE_LEN) ? 0 : ic + 1;
        nC = (R->B_addr == (R->slice_y + 1) * PE_LEN - 1)
                 ? ((R->C_addr == (R->slice_z + 1) * PE_LEN - 1) ? R->slice_z * PE_LEN : R->C_addr + 1)
                 : R->C_addr;
        nB = (R->B_addr == (R->slice_y + 1) * PE_LEN - 1) ? R->slice_y * PE_LEN : R->B_addr + 1;
        nA = (ic == PE_LEN * PE_LEN) ? 1 : 0;
        n_cc = 0;
        break;
      }
      case COMPUTE: {
        const uint32_t cc = R->compute_counter;
        if (cc == 0) n_EN_start = 1;
        if (cc == A_idx) n_EN_start = 0;
        if (cc < A_idx - 1) nA = R->A_addr + 1;
        if (cc < A_idx - 2) {
          YSET(nyA, border_00, (cc + 2) & AMASK);
          YSET(nyA, R->y_read_idx, (cc + 1) & AMASK);
          if (R->slice_y % 2 == 1) nzA[0][1] = (cc + 1) & AMASK;
          else nzA[1][1] = (cc + 1) & AMASK;
        } else if (cc >= A_idx - 2 && cc < A_idx - 1 + PE_LEN) {
          YSET(nyA, R->y_read_idx, (A_idx - 1) & AMASK);
          nzA[0][1] = (A_idx - 1) & AMASK;
          nzA[1][1] = (A_idx - 1) & AMASK;
        }
        if (cc >= PE_LEN && cc < PE_LEN + A_idx) {
          if (R->slice_y % 2 == 1) nzA[1][1] = (cc - PE_LEN) & AMASK;
          else nzA[0][1] = (cc - PE_LEN) & AMASK;
          YSET(nyA, R->y_write_idx, (cc - PE_LEN) & AMASK);
        } else if (cc >= PE_LEN + A_idx && cc < 2 * PE_LEN + A_idx - 1) {
          nzCEN[0][1] = 1;
          nzCEN[1][1] = 1;
          YSET(nyCEN, R->y_write_idx, 1);
        }
        n_cc = (cc == 2 * PE_LEN + A_idx - 1) ? 0 : cc + 1;
        if (cc == 2 * PE_LEN + A_idx - 1) {
          n_sy = (R->slice_y == slice_y_max_idx) ? 0 : R->slice_y + 1;
          n_sz = (R->slice_y == slice_y_max_idx) ? ((R->slice_z == slice_z_max_idx) ? 0 : R->slice_z + 1) : R->slice_z;
          n_yw = ((R->y_write_idx == A_idx + PE_LEN) ? 0 : R->y_write_idx + PE_LEN) & 0x3FF;
          if (R->slice_z > 0) n_yr = ((R->y_read_idx >= A_idx + PE_LEN) ? 0 : R->y_read_idx + PE_LEN) & 0x3FF;
          else n_yr = R->y_read_idx;
          n_state = (R->slice_y == slice_y_max_idx && R->slice_z == slice_z_max_idx) ? 3 /*OUT*/ : INITIAL;
          nA = 0;
          nB = (R->slice_y == slice_y_max_idx) ? 0 : (R->slice_y + 1) * PE_LEN;
          nC = (R->slice_y == slice_y_max_idx) ? ((R->slice_z == slice_z_max_idx) ? 0 : (R->slice_z + 1) * PE_LEN) : R->C_addr;
          if (R->slice_z == slice_z_max_idx && R->slice_y == slice_y_max_idx) {
            n_score = final_max_out;
            n_finish = 1;
          }
        }
        break;
      }
      default: break;
    }

    /* ---------------- clock edge: commit ---------------- */
    /* SRAMs sample the pre-edge control and data (sram_1024x8_t13, 493-500) */
    for (int i = 0; i < R->ny; ++i) {
      if (R->y_CEN[i] != 0) continue;
      const uint32_t addr = R->y_A[i] & AMASK;
      if (R->y_WEN[i] == 0) {
        const int ge = i % PE_LEN; /* y_D_i[gi*8+ge] = PE(ge+1, 8) */
        R->y_mem[(size_t)i * SRAM_DEPTH + addr] = Mo[ge + 1][PE_LEN];
      } else {
        R->y_Q[i] = R->y_mem[(size_t)i * SRAM_DEPTH + addr];
      }
    }
    for (int g = 0; g < 2; ++g)
      for (int j = 1; j <= PE_LEN; ++j) {
        if (R->z_CEN[g][j] != 0) continue;
        const uint32_t addr = R->z_A[g][j] & AMASK;
        st7 *m = R->z_mem + ((size_t)g * (PE_LEN + 1) + j) * SRAM_DEPTH + addr;
        if (R->z_WEN[g][j] == 0) *m = Mo[PE_LEN][j];
        else R->z_Q[g][j] = *m;
      }
    /* SRAM control registers with the shift functions (361-423) */
    {
      int *oCEN = (int *)malloc(sizeof(int) * R->ny);
      uint32_t *oA = (uint32_t *)malloc(sizeof(uint32_t) * R->ny);
      memcpy(oCEN, R->y_CEN, sizeof(int) * R->ny);
      memcpy(oA, R->y_A, sizeof(uint32_t) * R->ny);
      for (int i = 0; i < R->ny; ++i) R->y_WEN[i] = nyWEN[i];
      const uint32_t yw = R->y_write_idx, yr = R->y_read_idx;
      for (uint32_t i = 0; i < (uint32_t)R->ny; ++i) {
        if (i > yw && i < yw + PE_LEN && i >= 1) { R->y_A[i] = oA[i - 1]; R->y_CEN[i] = oCEN[i - 1]; }
        else if (i == yr) { R->y_A[i] = nyA[i] & AMASK; R->y_CEN[i] = nyCEN[i]; }
        else if (i == yw) { R->y_A[i] = nyA[i] & AMASK; R->y_CEN[i] = nyCEN[i]; }
        else if (i == border_00) { R->y_A[i] = nyA[i] & AMASK; R->y_CEN[i] = nyCEN[i]; }
        else if (i > yr && i < yr + PE_LEN && i >= 1) { R->y_A[i] = oA[i - 1]; R->y_CEN[i] = nyCEN[i]; }
        else { R->y_A[i] = nyA[i] & AMASK; R->y_CEN[i] = nyCEN[i]; }
      }
      free(oCEN);
      free(oA);
      for (int g = 0; g < 2; ++g) {
        for (int j = 0; j <= PE_LEN; ++j) R->z_WEN[g][j] = nzWEN[g][j];
        uint32_t oa[PE_LEN + 1];
        int oc[PE_LEN + 1];
        memcpy(oa, R->z_A[g], sizeof(oa));
        memcpy(oc, R->z_CEN[g], sizeof(oc));
        R->z_A[g][1] = nzA[g][1] & AMASK;
        R->z_CEN[g][1] = nzCEN[g][1];
        for (int j = 2; j <= PE_LEN; ++j) { R->z_A[g][j] = oa[j - 1]; R->z_CEN[g][j] = oc[j - 1]; }
      }
    }
    /* PE registers */
    for (int y = 1; y <= PE_LEN; ++y)
      for (int z = 1; z <= PE_LEN; ++z) R->pe[y][z] = npe[y][z];
    /* testbench registered symbol RAM read (tb:391-397, 163-169) */
    R->a_sym = tb_symbol(R->sa, R->la, R->A_addr);
    R->b_sym = tb_symbol(R->sb, R->lb, R->B_addr);
    R->c_sym = tb_symbol(R->sc, R->lc, R->C_addr);
    /* controller registers (448-466) */
    R->state = n_state;
    R->input_counter = n_ic & 0xFFF;
    R->compute_counter = n_cc & 0xFFF;
    R->slice_y = n_sy & 0x1FF;
    R->slice_z = n_sz & 0x1FF;
    memcpy(R->Bi, nBi, sizeof(nBi));
    memcpy(R->Ci, nCi, sizeof(nCi));
    R->EN_start = n_EN_start;
    R->y_read_idx = n_yr;
    R->y_write_idx = n_yw;
    R->score_reg = n_score;
    R->finish = n_finish;
    R->A_addr = nA & 0x7FFF;
    R->B_addr = nB & 0x7FFF;
    R->C_addr = nC & 0x7FFF;
    start_pulse = 0;
    ++cyc;
    if (R->finish) { final_score = R->score_reg; done = 1; }
  }
#undef YSET
  *score = (final_score == XV) ? 0 : final_score;
  if (score_is_x) *score_is_x = (final_score == XV) || !done;
  if (cycles_out) *cycles_out = cyc;
  free(R->y_WEN); free(R->y_CEN); free(R->y_A); free(R->y_Q); free(R->y_mem); free(R->z_mem);
  free(nyWEN); free(nyCEN); free(nyA);
  free(R);
  return done ? TSA_OK : TSA_EINTERNAL;
}
