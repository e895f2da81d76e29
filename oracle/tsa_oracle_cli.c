/* tsa_oracle_cli -- TEST INFRASTRUCTURE: CPU oracle counterpart of the tsa
 * CLI. Prints the testbench line "TriAlign Score: <n>" (src/TriAlign_tb.sv:341)
 * from the restatement (default) or the cycle-level RTL model (--rtl).
 *   tsa_oracle_cli A B C [--rtl] [--s3 rtl|sop] [--bits B] */
#include <stdio.h>
#include <string.h>

#include "../hw-accelerator-three-sequence-alignment_amd/tools/seqio.h"
#include "tsa_oracle.h"

int main(int argc, char **argv) {
  const char *f[3];
  int nf = 0, rtl = 0;
  tsa_params p = {1, -1, 2, 1, TSA_S3_RTL, 12};
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--rtl")) rtl = 1;
    else if (!strcmp(argv[i], "--s3") && i + 1 < argc) p.s3_mode = !strcmp(argv[++i], "sop");
    else if (!strcmp(argv[i], "--bits") && i + 1 < argc) p.score_bits = atoi(argv[++i]);
    else if (nf < 3) f[nf++] = argv[i];
  }
  if (nf != 3) { fprintf(stderr, "usage: tsa_oracle_cli A B C [--rtl] [--s3 rtl|sop] [--bits B]\n"); return 2; }
  uint8_t *s[3];
  int64_t n[3];
  for (int k = 0; k < 3; ++k)
    if ((n[k] = tsa_read_sequence(f[k], &s[k])) < 0) { fprintf(stderr, "cannot read %s\n", f[k]); return 1; }
  int32_t score = 0, isx = 0, fin[7];
  int rc;
  if (rtl) rc = tsao_rtl_run(s[0], (int32_t)n[0], s[1], (int32_t)n[1], s[2], (int32_t)n[2], 512, &score, &isx, NULL);
  else rc = tsao_score_xplane(s[0], (int32_t)n[0], s[1], (int32_t)n[1], s[2], (int32_t)n[2], &p, &score, fin);
  if (rc) { fprintf(stderr, "error %d\n", rc); return 1; }
  printf("TriAlign Score:        \t%d%s\n", score, isx ? " (x)" : "");
  if (!rtl) printf("final states {M,Ix,Iy,Iz,Ixy,Iyz,Ixz}: %d %d %d %d %d %d %d\n", fin[0], fin[1], fin[2], fin[3], fin[4], fin[5], fin[6]);
  return 0;
}
