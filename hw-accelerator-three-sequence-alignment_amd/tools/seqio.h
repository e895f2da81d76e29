// seqio.h -- sequence readers shared by the CLIs: the reference's dat format
// (one decimal symbol per line, CRLF, dat/A_seq.dat) and FASTA with the
// testbench's encoding A=0 T=1 C=2 G=3 N=4 (src/TriAlign_tb.sv:42-46).
#pragma once
#include <ctype.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

// Returns the number of symbols read into *out (malloc'd), or -1 on error.
static inline int64_t tsa_read_sequence(const char *path, uint8_t **out) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (sz < 0) { fclose(f); return -1; }
  char *buf = (char *)malloc((size_t)sz + 1);
  if (!buf) { fclose(f); return -1; }
  size_t got = fread(buf, 1, (size_t)sz, f);
  fclose(f);
  buf[got] = 0;
  uint8_t *seq = (uint8_t *)malloc(got + 1);
  int64_t n = 0;
  // skip leading whitespace to sniff the format
  const char *p = buf;
  while (*p && isspace((unsigned char)*p)) ++p;
  if (*p == '>') {  // FASTA: first record only
    const char *q = strchr(p, '\n');
    q = q ? q + 1 : p + strlen(p);
    for (; *q && *q != '>'; ++q) {
      char ch = (char)toupper((unsigned char)*q);
      if (isspace((unsigned char)ch)) continue;
      int v;
      switch (ch) {
        case 'A': v = 0; break;
        case 'T': case 'U': v = 1; break;
        case 'C': v = 2; break;
        case 'G': v = 3; break;
        case 'N': v = 4; break;
        default: free(buf); free(seq); return -1;
      }
      seq[n++] = (uint8_t)v;
    }
  } else {  // dat: decimal tokens separated by whitespace (CRLF tolerant)
    char *q = (char *)p;
    while (*q) {
      while (*q && isspace((unsigned char)*q)) ++q;
      if (!*q) break;
      char *end;
      long v = strtol(q, &end, 10);
      if (end == q || v < 0 || v > 4) { free(buf); free(seq); return -1; }
      seq[n++] = (uint8_t)v;
      q = end;
    }
  }
  free(buf);
  *out = seq;
  return n;
}
