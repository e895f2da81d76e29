#!/bin/bash
# Lap-schedule A/B on one box (tools/bench_variants.py, interleaved rounds):
# geometries of single large cubes and batches under the round loop. Each
# line: median ms, and whether the variants agree (and none timed out).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-lapab}; mkdir -p $O
run() { echo "== $*" >> $O/lapab.jsonl; timeout -k 10 300 python tools/bench_variants.py "$@" >> $O/lapab.jsonl 2>> $O/lapab.err; }
run --n 1 --L 1024 --score-bits 16 --rounds 5 --variants "TSA_LAP_M=2,TSA_LAP_NW=8" "TSA_LAP_M=1,TSA_LAP_NW=8" "TSA_LAP_M=1,TSA_LAP_NW=4" || exit 1
run --n 1 --L 1024 --score-bits 12 --kernel plane --rounds 3 --variants "TSA_LAP_M=2,TSA_LAP_NW=8" "TSA_LAP_M=1,TSA_LAP_NW=8" || exit 1
run --n 1 --L 768 --score-bits 16 --rounds 5 --variants "TSA_LAP_M=2,TSA_LAP_NW=8" "TSA_LAP_M=1,TSA_LAP_NW=8" || exit 1
run --n 8 --L 512 --rounds 5 --check --variants "TSA_LAP_CHUNK=4" "TSA_LAP_CHUNK=8" || exit 1
run --n 16 --L 256 --rounds 5 --check --variants "TSA_LAP_CHUNK=8" "TSA_LAP_CHUNK=16" "TSA_PENCIL_MODE=helix" || exit 1
run --n 4 --L 1024 --score-bits 16 --rounds 3 --variants "TSA_LAP_CHUNK=1" "TSA_LAP_CHUNK=2" "TSA_LAP_CHUNK=4" || exit 1
cat $O/lapab.jsonl
