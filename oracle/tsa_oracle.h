/*
 * tsa_oracle.h -- CPU oracle for the TriAlign hot path. TEST INFRASTRUCTURE.
 *
 * This is a plain-C restatement of the reference RTL's arithmetic
 * (timmy139710/HW-Accelerator-Three-Sequence-Alignment, src/PE_1cyc.v and
 * src/TriAlign_1cyc.v). It is the checker for the HIP product path and the
 * CPU baseline of bench.py; nothing in the product library links, loads or
 * calls it (only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg do).
 *
 * Parity pinning (see DESIGN.md section "Oracle"): the reference ships no
 * golden vector or expected score. The oracle is pinned by (1) the analytic
 * known answer of the reference testbench's own input (all-A 64^3 -> 192,
 * src/TriAlign_tb.sv:423-1960), (2) the family all-A n^3 -> 3n, (3) a
 * cycle-level C model of TRIALIGN_1cyc + PE_1cyc (oracle/rtl_model.c) that
 * executes the RTL's register transfers -- face SRAMs, delay registers and
 * pencil FSM included -- and must agree with this restatement on every
 * in-envelope input, and (4) the survey-time values (dat triple -> 1, etc.).
 */
#ifndef TSA_ORACLE_H
#define TSA_ORACLE_H

#include <stdint.h>

#include "../include/trialign.h"

#ifdef __cplusplus
extern "C" {
#endif

/* State order of the RTL SRAM word {M,Ix,Iy,Iz,Ixy,Iyz,Ixz}
 * (src/TriAlign_1cyc.v:130,138). */
enum { TSAO_M = 0, TSAO_IX, TSAO_IY, TSAO_IZ, TSAO_IXY, TSAO_IYZ, TSAO_IXZ };

/* Penalty subtracted on the transition source -> target, P[target][source]
 * (src/PE_1cyc.v:164-218; see tsa_oracle.c for the per-line mapping). */
void tsao_penalty_table(const tsa_params *p, int32_t P[7][7]);

/* Pair / triple scores of the PE (src/PE_1cyc.v:159-162), on symbols & 3. */
int32_t tsao_s2(int p, int q, const tsa_params *prm);
int32_t tsao_s3(int a, int b, int c, const tsa_params *prm);

/* Literal restatement, x-plane order (two (LB+1)x(LC+1) planes of 7 states).
 * 49 candidates per cell, each wrapped to score_bits before MAX7, exactly as
 * the RTL's wordsize-wide candidate wires (src/PE_1cyc.v:127-133).
 * final7 (nullable) receives the 7 states of cell (la,lb,lc). */
int tsao_score_xplane(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                      const uint8_t *c, int32_t lc, const tsa_params *p,
                      int32_t *score, int32_t *final7);

/* Same arithmetic in anti-diagonal plane order (q = x+y+z), with a ring of
 * four (y,z) planes -- the traversal the GPU plane kernel uses. Self-check. */
int tsao_score_diag(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                    const uint8_t *c, int32_t lc, const tsa_params *p,
                    int32_t *score, int32_t *final7);

/* Factored "message" form (each cell sends 7 max-reduced messages to its 7
 * successors), unbounded arithmetic. Equal to the literal form whenever no
 * candidate wraps; used to validate the factoring the pencil kernel uses. */
int tsao_score_msg(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                   const uint8_t *c, int32_t lc, const tsa_params *p,
                   int32_t *score);

/* Traceback of the literal form (extension: the RTL outputs only the score):
 * moves[] = state index per alignment column, forward order; start = face
 * cell the path leaves; ties to the lowest state index. Cubes up to 2^26
 * cells (full state cube in memory). Mirrors tsa_align_gpu's contract. */
int tsao_align(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb, const uint8_t *c,
               int32_t lc, const tsa_params *p, int32_t *score, uint8_t *moves,
               int32_t max_moves, int32_t *n_moves, int32_t *start);

/* Min / max over every state value of the cube (unbounded arithmetic), for
 * range checks of the int16 GPU state storage. */
int tsao_state_range(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                     const uint8_t *c, int32_t lc, const tsa_params *p,
                     int32_t *lo, int32_t *hi);

/* n triples laid out as in tsa_score_batch(); nthreads POSIX threads, one
 * triple at a time per thread (tsao_score_xplane). */
int tsao_score_batch(const uint8_t *seqs, const int64_t *offsets, int32_t n,
                     const tsa_params *p, int32_t *scores, int32_t nthreads);

/* Synthetic DNA: splitmix64(seed) words, 32 two-bit symbols per word, low
 * bits first. Seed of triple i, sequence s in {0,1,2}:
 * TSAO_SEED_BASE + 3*i + s. */
#define TSAO_SEED_BASE 0x7A1A11670000ULL
void tsao_gen_uniform(uint64_t seed, uint8_t *out, int32_t len);

/* Cycle-level model of TRIALIGN_1cyc (oracle/rtl_model.c). a_total_len is
 * the A_TOTAL_LEN parameter (sizes the y-face SRAM ring; <= 512). score_is_x
 * is set when the score depends on an undefined (x/z) value. */
int tsao_rtl_run(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                 const uint8_t *c, int32_t lc, int32_t a_total_len, int32_t *score,
                 int32_t *score_is_x, int64_t *cycles_out);

/* Cycle-level model of TRIALIGN_2cyc + PE_2cyc (oracle/rtl_model_2cyc.c),
 * A_TOTAL_LEN 512 (la <= 512). Same outputs as tsao_rtl_run. */
int tsao_rtl2_run(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                  const uint8_t *c, int32_t lc, int32_t *score, int32_t *score_is_x,
                  int64_t *cycles_out);

/* Monotonic wall clock in seconds (clock_gettime(CLOCK_MONOTONIC)). */
double tsao_now(void);

#ifdef __cplusplus
}
#endif
#endif
