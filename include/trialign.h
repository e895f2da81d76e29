/*
 * trialign.h -- C-ABI of the MI355X-native three-sequence 3-D DP scorer.
 *
 * This is the drop-in boundary for the reference's one hot path: the TRIALIGN
 * module (timmy139710/HW-Accelerator-Three-Sequence-Alignment), which maps
 * (seqA, seqB, seqC) -> optimal 7-state affine-gap 3-D DP score.
 *
 *   reference interface                        replaced by
 *   ------------------------------------------ ---------------------------------
 *   TRIALIGN ports + parameters                tsa_score_gpu()
 *     src/TriAlign_1cyc.v:1-22                   (lengths A_idx/B_idx/C_idx ->
 *     (start_align pulse, A/B/C_symbol pull,      la/lb/lc; symbol pull protocol
 *      A/B/C_idx lengths, Score, finish)          -> caller-owned byte arrays;
 *                                                 Score/finish -> *score + rc)
 *   PE localparams MATCH/MISMATCH/GO/GE        tsa_params + tsa_default_params()
 *     src/PE_1cyc.v:55-61 (compile-time)         (runtime; defaults = RTL values)
 *   SCORE_BITS parameter (12)                  tsa_params.score_bits
 *     src/TriAlign_tb.sv:56, TriAlign_1cyc.v:6
 *   temp_ABC triple score                      tsa_params.s3_mode (RTL literal by
 *     src/PE_1cyc.v:162                           default; sum-of-pairs optional)
 *   testbench one-shot start/finish FSM        tsa_score_batch(): many triples,
 *     src/TriAlign_tb.sv:279-333                  sharded over the node's GPUs
 *   (no reference equivalent: the reference    tsa_score_batch_async(): device
 *    has one alignment in flight)                 pointers + caller stream, for
 *                                                 in-HBM throughput runs
 *   alignment-output ports (commented out,     tsa_align_gpu(): the optimal path
 *    src/TriAlign_tb.sv:239-260)                  as alignment columns
 *
 * Conventions
 *   - Symbols are one byte each, 0..4 = A,T,C,G,N (src/TriAlign_tb.sv:42-46).
 *     Values > 4 -> TSA_EINVAL. Symbols are reduced mod 4 exactly as the 2-bit
 *     PE symbol registers do (src/PE_1cyc.v:63-66), so N aliases A.
 *   - Lengths >= 1. There is no RTL length envelope here (multiples of 8,
 *     LB <= LA <= 512): results outside it follow the recurrence.
 *   - Return 0 (TSA_OK) or a negative TSA_E* code. Functions are thread-safe
 *     and retain no caller pointer. GPU calls other than *_async are
 *     synchronous.
 *   - Every GPU entry point fails with TSA_ENODEV when no HIP device is
 *     present: there is no CPU fallback in this library.
 */
#ifndef TRIALIGN_H
#define TRIALIGN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSA_OK 0
#define TSA_EINVAL (-1)    /* bad pointer, length, symbol or parameter        */
#define TSA_ERANGE (-2)    /* score range cannot be represented exactly       */
#define TSA_ENODEV (-3)    /* no HIP device / device index out of range       */
#define TSA_EDEVICE (-4)   /* HIP runtime error                               */
#define TSA_ENOMEM (-5)    /* device allocation failed / workspace too small  */
#define TSA_EINTERNAL (-6) /* kernel self-check failed                        */

/* Score reported for a triple the device could not score (a lap-kernel
 * hand-off timed out on tsa_score_batch_async): rescore it. Never a valid
 * score -- every valid score fits 16 bits. The synchronous entry points
 * rescore such triples themselves (tsa_fallback_count counts it). */
#define TSA_SCORE_INVALID INT32_MIN

/* Score reported by TSA_KERNEL_CHECKED for a triple whose values may have
 * left the SCORE_BITS range (so the RTL's wrapped result may differ): rescore
 * it with TSA_KERNEL_PLANE. The synchronous entry points do that themselves
 * (tsa_check_fallback_count counts it). */
#define TSA_SCORE_UNCERTIFIED (INT32_MIN + 1)

#define TSA_S3_RTL 0 /* temp_ABC as the RTL evaluates it (src/PE_1cyc.v:162) */
#define TSA_S3_SOP 1 /* sum of the three pair scores                          */

/* Kernel selection for tsa_score_*; TSA_KERNEL_AUTO picks per shape. */
#define TSA_KERNEL_AUTO 0
/* The literal RTL arithmetic (every candidate wrapped at SCORE_BITS) for any
 * parameter set. Its plan by a cost model: the literal lap schedule for a few
 * cubes, the literal helix for batches of LC <= 512, else the anti-diagonal
 * plane sweep (tsa_describe_plan names it). */
#define TSA_KERNEL_PLANE 1
#define TSA_KERNEL_PENCIL 2 /* register-systolic pencil sweep (factored form)    */
/* The pencil lap kernel in int16 with a range monitor, for cubes whose a-priori
 * bound exceeds SCORE_BITS (beyond ~680 per side with the RTL constants) but
 * whose values may well stay inside it: the factored form is exact whenever
 * no value of the literal recurrence wraps, and the monitor proves that per
 * triple (every real cell's best, then the candidate bound of DESIGN.md 1.2)
 * or reports TSA_SCORE_UNCERTIFIED. TSA_KERNEL_AUTO uses it on the
 * synchronous entry points (rescoring uncertified triples with PLANE); the
 * async path only runs it when asked. Single cubes / small batches (the lap
 * schedule) only: TSA_ERANGE otherwise. */
#define TSA_KERNEL_CHECKED 3

typedef struct tsa_params {
  int32_t match;      /* MATCH      (src/PE_1cyc.v:55), default  1 */
  int32_t mismatch;   /* MISMATCH   (src/PE_1cyc.v:56), default -1 */
  int32_t gap_open;   /* GO         (src/PE_1cyc.v:57), default  2 */
  int32_t gap_extend; /* GE         (src/PE_1cyc.v:58), default  1 */
  int32_t s3_mode;    /* TSA_S3_RTL (default) or TSA_S3_SOP          */
  int32_t score_bits; /* 12 = RTL SCORE_BITS wrap (default); 0 = no wrap
                         (int16 range); any of 4..16 is accepted      */
} tsa_params;

/* Fill *p with the RTL's effective constants (1, -1, 2, 1, RTL s3, 12 bits). */
void tsa_default_params(tsa_params *p);

/* Host-side validation of one triple + params (no device work). */
int tsa_validate(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                 const uint8_t *c, int32_t lc, const tsa_params *p);

/* Score one triple on HIP device `device` (synchronous). Host buffers. */
int tsa_score_gpu(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                  const uint8_t *c, int32_t lc, const tsa_params *p,
                  int32_t *score, int32_t device);

/* As tsa_score_gpu with an explicit kernel choice and optional final states:
 * final_states (nullable) receives the 7 states {M,Ix,Iy,Iz,Ixy,Iyz,Ixz} of
 * cell (la,lb,lc) -- the 84-bit SRAM word of src/TriAlign_1cyc.v:130,138; a
 * non-null final_states runs the literal kernels (TSA_KERNEL_PLANE). */
int tsa_score_gpu_ex(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                     const uint8_t *c, int32_t lc, const tsa_params *p,
                     int32_t kernel, int32_t *score, int32_t *final_states,
                     int32_t device);

/* Score n independent triples held back to back in host memory:
 * triple i is seqs[offsets[3i] .. offsets[3i+1]) = A,
 * [offsets[3i+1] .. offsets[3i+2]) = B, [offsets[3i+2] .. offsets[3i+3]) = C.
 * offsets has 3n+1 entries. Triples are sharded over min(n_devices, visible
 * devices) GPUs (n_devices <= 0: all visible), one host thread per device. */
int tsa_score_batch(const uint8_t *seqs, const int64_t *offsets, int32_t n,
                    const tsa_params *p, int32_t *scores, int32_t n_devices);

/* tsa_score_batch over an explicit device list: the batch is cut into
 * min(n_devices, n) contiguous shards, shard s (triples [n*s/ns, n*(s+1)/ns))
 * on devices[s]. A device may be listed more than once ({0,0,0} shards a
 * batch three ways on one GPU): one host thread per distinct device runs its
 * shards one after another. Same replacement of the testbench's one-shot
 * caller (src/TriAlign_tb.sv:279-333) as tsa_score_batch, which is this call
 * with devices {0..n_devices-1}. TSA_ENODEV for a device index out of range. */
int tsa_score_batch_devices(const uint8_t *seqs, const int64_t *offsets, int32_t n,
                            const tsa_params *p, int32_t *scores,
                            const int32_t *devices, int32_t n_devices);

/* Device-resident batch. d_seqs/d_offsets/d_scores are device pointers on the
 * current device; stream is a hipStream_t (NULL = default stream). The
 * workspace must hold tsa_batch_workspace_size() bytes. max_l* bound every
 * triple's lengths. Launches only; no host synchronisation. Validation of
 * symbols is the caller's job on this path (tsa_validate on the host copy).
 * For a few large cubes this path may run the single-cube (lap) schedule --
 * the factored lap kernel, or for TSA_KERNEL_PLANE the literal lap kernel --
 * whose workgroups hand data to each other. The launched grid is one
 * resident round (8 x SX workgroups, at any workgroups per CU); a cube or
 * batch with more laps than resident slots runs up to LAP_MAX_WAVES (4)
 * rounds as each workgroup's loop over its later-round laps, in lap order.
 * Forward progress needs every launched workgroup co-resident, so a
 * concurrent kernel holding CUs of the device can delay some of them; every
 * hand-off wait is bounded, and if one times out the affected triples read
 * TSA_SCORE_INVALID once the stream has synchronised -- check for it on every
 * kernel choice, TSA_KERNEL_PLANE included. */
int tsa_batch_workspace_size(int32_t n, int32_t max_la, int32_t max_lb,
                             int32_t max_lc, const tsa_params *p,
                             int32_t kernel, size_t *bytes);
int tsa_score_batch_async(const uint8_t *d_seqs, const int64_t *d_offsets,
                          int32_t n, int32_t max_la, int32_t max_lb,
                          int32_t max_lc, const tsa_params *p, int32_t kernel,
                          int32_t *d_scores, void *d_workspace,
                          size_t workspace_bytes, void *stream);

/* tsa_score_batch_async on 2-bit packed sequences: d_packed holds symbol i of
 * the batch buffer at bits [2(i%4)+1 : 2(i%4)] of byte i/4 (tsa_pack2);
 * offsets count symbols, as above. The RTL keeps symbols in 2-bit registers
 * (src/PE_1cyc.v:63-66: N = 4 scores as A), so packing loses nothing; the
 * input is a quarter of the bytes. Same kernels, workspace and semantics. */
int tsa_score_batch_async_p2(const uint8_t *d_packed, const int64_t *d_offsets,
                             int32_t n, int32_t max_la, int32_t max_lb,
                             int32_t max_lc, const tsa_params *p, int32_t kernel,
                             int32_t *d_scores, void *d_workspace,
                             size_t workspace_bytes, void *stream);
/* Pack n symbols (0..4) four to a byte for tsa_score_batch_async_p2; out must
 * hold (n + 3) / 4 bytes. TSA_EINVAL on a symbol above 4. Host only. */
int tsa_pack2(const uint8_t *syms, int64_t n, uint8_t *out);

/* Score ONE triple with its cube split over several GPUs (synchronous): the
 * reference's slicing of the (y,z) plane into pencils chained through face
 * SRAMs (src/TriAlign_1cyc.v:78-98,127-140, pic/Memory.png), distributed --
 * the cube's laps (2*NW rows of y each) are cut into
 * n_devices contiguous runs, part i on devices[i]; the last lap of part i
 * hands its y records to part i+1 by system-scope stores into part i+1's
 * fine-grained workspace over xGMI (peer access is enabled between the listed
 * devices). A device may be listed more than once: its parts then run
 * concurrently on streams of their own when all their workgroups fit on the
 * device at once, else one after another on one stream of that device (a
 * part that waited for CU slots held by a later part could never finish).
 * The factored arithmetic where
 * it is exact a priori, else the RTL's literal wrapped arithmetic (any
 * parameter set); TSA_ERANGE with fewer laps than n_devices (or no lap
 * schedule). A timed-out hand-off returns TSA_EINTERNAL (never a silent
 * score). wall_us (nullable): host wall time from the first launch to the last
 * part's completion. */
int tsa_score_gpu_multi(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                        const uint8_t *c, int32_t lc, const tsa_params *p,
                        const int32_t *devices, int32_t n_devices, int32_t *score,
                        double *wall_us);

/* Optimal alignment of one triple (synchronous, HIP device `device`): the
 * path behind the score, as one move per alignment column. This has no RTL
 * counterpart -- the testbench's alignment-output ports are commented out
 * (src/TriAlign_tb.sv:239-260) -- so it is an extension, defined by the same
 * recurrence (src/PE_1cyc.v:164-218) and computed by the literal PLANE
 * arithmetic. moves[k], k < *n_moves, in forward order, is the state of the
 * k-th column, which says which sequences it consumes:
 *   TSA_MOVE_M (a,b,c) _IX (a) _IY (b) _IZ (c) _IXY (a,b) _IYZ (b,c) _IXZ (a,c).
 * start[3] receives the face cell (x0,y0,z0) the path leaves: the zero faces
 * make the start free, so symbols before a[x0], b[y0], c[z0] are not aligned
 * (0-based: the first aligned symbols are a[x0], b[y0], c[z0] as consumed).
 * Ties go to the lowest state index, at the final MAX7 and at every cell.
 * max_moves must be >= la + lb + lc. The pointer cube needs 4*lb*(la+lc-1)*lc
 * bytes of device memory (TSA_ENOMEM when it cannot be allocated). */
#define TSA_MOVE_M 0
#define TSA_MOVE_IX 1
#define TSA_MOVE_IY 2
#define TSA_MOVE_IZ 3
#define TSA_MOVE_IXY 4
#define TSA_MOVE_IYZ 5
#define TSA_MOVE_IXZ 6
int tsa_align_gpu(const uint8_t *a, int32_t la, const uint8_t *b, int32_t lb,
                  const uint8_t *c, int32_t lc, const tsa_params *p, int32_t *score,
                  uint8_t *moves, int32_t max_moves, int32_t *n_moves, int32_t *start,
                  int32_t device);

/* Which kernel, arithmetic and schedule a batch of these sizes would run, as a
 * short text such as "pencil lap f16 rtl M=1 NW=16 laps=16 tiles=1 waves=1"
 * or "plane" (sync = 1: the synchronous tsa_score_batch path, which may stream
 * the lap kernel). Host-only, no device needed. A diagnostic with no reference
 * counterpart (the RTL has one fixed datapath). */
int tsa_describe_plan(int32_t n, int32_t max_la, int32_t max_lb, int32_t max_lc,
                      const tsa_params *p, int32_t kernel, int32_t sync, char *buf,
                      size_t len);

/* Lap-kernel hand-offs that timed out on the synchronous entry points since
 * the library was loaded; each was rescored without the lap schedule (the
 * helix, or for the literal arithmetic the literal helix / plane sweep) and
 * logged to stderr. 0 in a healthy run. */
int64_t tsa_fallback_count(void);

/* Triples the checked kernel could not certify on the synchronous entry points
 * since the library was loaded; each was rescored in the literal arithmetic
 * (TSA_KERNEL_PLANE's plan). */
int64_t tsa_check_fallback_count(void);

/* Number of visible HIP devices (0 when none), or a negative code. */
int tsa_device_count(void);

/* Short description of a return code. */
const char *tsa_strerror(int rc);

/* Library build id, "trialign-mi355x gfx950 src=<hash>": the first 16 hex
 * digits of a SHA-256 over the library's sources (csrc .hip and .h files and
 * this header; srchash.py), so a run names the sources its binary came from. */
const char *tsa_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TRIALIGN_H */
