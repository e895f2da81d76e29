#!/bin/bash
# Round 4j: single-cube A/B of the lap kernel's register budget (M = 1 at 6 or
# 4 waves per EU, the per-lap index launder on or off) against the r4b build,
# the round-loop geometries, and the helix per-cell rate of the M = 4 form
# (LC 512, one workgroup per CU) against M = 2 (LC 256), plain f16 arithmetic.
# The GPU suite runs separately (scripts/gpu_round.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4j}; O=gpurun_out/$TAG; mkdir -p $O
TAG=$TAG LENS="64 256 512" PKGS="variants/r4b hw-accelerator-three-sequence-alignment_amd variants/flatnl variants/flatw4" HPKGS="" \
  bash scripts/gpu_ab.sh > /dev/null || exit 1
for i in 1 2; do
  echo "== helix M" >> $O/helix_m.jsonl
  timeout -k 10 150 python tools/bench_variants.py --n 512 --L 256 --rounds 5 \
    --variants "TSA_PENCIL_MODE=helix" "TSA_PENCIL_MODE=helix,TSA_PENCIL_ARITH=f16" >> $O/helix_m.jsonl 2>> $O/helix_m.err || exit 1
  timeout -k 10 150 python tools/bench_variants.py --n 256 --L 512 --rounds 3 \
    --variants "TSA_PENCIL_MODE=helix,TSA_PENCIL_ARITH=f16" >> $O/helix_m.jsonl 2>> $O/helix_m.err || exit 1
done
run() { echo "== $*" >> $O/lapab.jsonl; timeout -k 10 300 python tools/bench_variants.py "$@" >> $O/lapab.jsonl 2>> $O/lapab.err; }
run --n 8 --L 512 --rounds 5 --check --variants "TSA_LAP_M=1" "TSA_LAP_M=2" || exit 1
run --n 16 --L 256 --rounds 5 --check --variants "TSA_LAP_M=1" "TSA_LAP_M=2" || exit 1
run --n 1 --L 1024 --rounds 5 --score-bits 16 --preload --variants "TSA_NONE=0" || exit 1
cat $O/single_ab.jsonl $O/helix_m.jsonl $O/lapab.jsonl
