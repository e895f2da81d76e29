// tsa -- score one triple on the GPU and print the testbench's line
// "TriAlign Score: <n>" (src/TriAlign_tb.sv:339-341).
//   tsa A.dat B.dat C.dat [--kernel auto|plane|pencil] [--device N]
//       [--s3 rtl|sop] [--bits B] [--match M --mismatch X --go O --ge E]
//       [--states] [--align]
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/trialign.h"
#include "seqio.h"

static int usage() {
  fprintf(stderr,
          "usage: tsa A B C [--kernel auto|plane|pencil] [--device N] [--s3 rtl|sop]\n"
          "           [--bits B] [--match M] [--mismatch X] [--go O] [--ge E] [--states]\n"
          "           [--align]   (also print the optimal alignment; tsa_align_gpu)\n"
          "A/B/C: dat files (one symbol 0..4 per line) or FASTA (A=0 T=1 C=2 G=3 N=4)\n");
  return 2;
}

int main(int argc, char **argv) {
  const char *files[3];
  int nf = 0, device = 0, kernel = TSA_KERNEL_AUTO, states = 0, align = 0;
  tsa_params p;
  tsa_default_params(&p);
  for (int i = 1; i < argc; ++i) {
    const char *a = argv[i];
    auto next = [&](void) -> const char * { return (i + 1 < argc) ? argv[++i] : nullptr; };
    if (!strcmp(a, "--kernel")) {
      const char *v = next();
      if (!v) return usage();
      kernel = !strcmp(v, "plane") ? TSA_KERNEL_PLANE : !strcmp(v, "pencil") ? TSA_KERNEL_PENCIL : TSA_KERNEL_AUTO;
    } else if (!strcmp(a, "--device")) { const char *v = next(); if (!v) return usage(); device = atoi(v); }
    else if (!strcmp(a, "--s3")) { const char *v = next(); if (!v) return usage(); p.s3_mode = !strcmp(v, "sop") ? TSA_S3_SOP : TSA_S3_RTL; }
    else if (!strcmp(a, "--bits")) { const char *v = next(); if (!v) return usage(); p.score_bits = atoi(v); }
    else if (!strcmp(a, "--match")) { const char *v = next(); if (!v) return usage(); p.match = atoi(v); }
    else if (!strcmp(a, "--mismatch")) { const char *v = next(); if (!v) return usage(); p.mismatch = atoi(v); }
    else if (!strcmp(a, "--go")) { const char *v = next(); if (!v) return usage(); p.gap_open = atoi(v); }
    else if (!strcmp(a, "--ge")) { const char *v = next(); if (!v) return usage(); p.gap_extend = atoi(v); }
    else if (!strcmp(a, "--states")) states = 1;
    else if (!strcmp(a, "--align")) align = 1;
    else if (a[0] == '-' && a[1] == '-') return usage();
    else if (nf < 3) files[nf++] = a;
    else return usage();
  }
  if (nf != 3) return usage();
  uint8_t *s[3];
  int64_t n[3];
  for (int k = 0; k < 3; ++k) {
    n[k] = tsa_read_sequence(files[k], &s[k]);
    if (n[k] < 0) { fprintf(stderr, "tsa: cannot read %s\n", files[k]); return 1; }
  }
  int32_t score = 0, fin[7];
  int rc = tsa_score_gpu_ex(s[0], (int32_t)n[0], s[1], (int32_t)n[1], s[2], (int32_t)n[2], &p,
                            states ? TSA_KERNEL_PLANE : kernel, &score, states ? fin : nullptr, device);
  if (rc) { fprintf(stderr, "tsa: %s (%d)\n", tsa_strerror(rc), rc); return 1; }
  printf("TriAlign Score:        \t%d\n", score);
  if (states)
    printf("final states {M,Ix,Iy,Iz,Ixy,Iyz,Ixz}: %d %d %d %d %d %d %d\n", fin[0], fin[1], fin[2],
           fin[3], fin[4], fin[5], fin[6]);
  if (align) {
    const int64_t cap = n[0] + n[1] + n[2];
    uint8_t *mv = (uint8_t *)malloc((size_t)cap);
    int32_t nm = 0, st[3], sc = 0;
    rc = mv ? tsa_align_gpu(s[0], (int32_t)n[0], s[1], (int32_t)n[1], s[2], (int32_t)n[2], &p, &sc,
                            mv, (int32_t)cap, &nm, st, device)
            : TSA_ENOMEM;
    if (rc) { fprintf(stderr, "tsa: %s (%d)\n", tsa_strerror(rc), rc); free(mv); return 1; }
    static const int use[7][3] = {{1, 1, 1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1, 1, 0}, {0, 1, 1}, {1, 0, 1}};
    static const char *letters = "ATCGN";
    printf("alignment start (x0,y0,z0) = (%d,%d,%d), %d columns\n", st[0], st[1], st[2], nm);
    for (int k = 0; k < 3; ++k) {
      int64_t pos = st[k];
      putchar("ABC"[k]);
      putchar(' ');
      for (int32_t j = 0; j < nm; ++j) putchar(use[mv[j]][k] ? letters[s[k][pos++]] : '-');
      putchar('\n');
    }
    free(mv);
  }
  return 0;
}
