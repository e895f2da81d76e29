#!/bin/bash
# Same-box A/B of variant libraries (scripts/build_variant.sh -> variants/<name>):
# single cubes (spin preload) over PKGS, then the helix batch over HPKGS.
# KERNEL (pencil) and BITS (12) select the single cubes' kernel and words
# (e.g. KERNEL=checked LENS=1024 for the checked 1024^3 form); HKERNEL the
# batch's (plane: the literal helix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}; O=gpurun_out/$TAG; mkdir -p $O
for i in 1 2; do
  for pk in $PKGS; do
    for L in ${LENS:-64 256 512}; do
      echo "== $pk $L" >> $O/single_ab.jsonl
      TSA_PKG_DIR=$GRAFT_REPO_ROOT/$pk timeout -k 10 120 python tools/bench_variants.py --n 1 --L $L --rounds ${ROUNDS:-9} --preload --kernel ${KERNEL:-pencil} --score-bits ${BITS:-12} --variants "TSA_NONE=0" >> $O/single_ab.jsonl 2>> $O/single_ab.err || exit 1
    done
  done
  for pk in $HPKGS; do
    echo "== helix $pk" >> $O/helix_ab.jsonl
    TSA_PKG_DIR=$GRAFT_REPO_ROOT/$pk timeout -k 10 120 python tools/bench_variants.py --n 512 --L 256 --rounds 5 --kernel ${HKERNEL:-pencil} --variants "TSA_NONE=0" >> $O/helix_ab.jsonl 2>> $O/helix_ab.err || exit 1
  done
done
cat $O/single_ab.jsonl; [ -z "$HPKGS" ] || cat $O/helix_ab.jsonl
