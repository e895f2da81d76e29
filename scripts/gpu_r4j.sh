#!/bin/bash
# Round 4j: the GPU suite on the flat-parameter lap kernel, the single-cube A/B
# against the r4b build (and a variant without the per-lap index launder, 4
# waves per EU for M = 1), the round-loop geometries, and the helix per-cell
# rate of the M = 4 form (LC 512) against M = 2 (LC 256), plain f16 arithmetic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TSA_EXPECT_GPU=1
TAG=${TAG:-r4j}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG LENS="64 256 512" PKGS="variants/r4b hw-accelerator-three-sequence-alignment_amd variants/flatnl" HPKGS="" \
  bash scripts/gpu_ab.sh > /dev/null || exit 1
run() { echo "== $*" >> $O/lapab.jsonl; timeout -k 10 300 python tools/bench_variants.py "$@" >> $O/lapab.jsonl 2>> $O/lapab.err; }
run --n 8 --L 512 --rounds 5 --check --variants "TSA_LAP_M=1" "TSA_LAP_M=2" || exit 1
run --n 16 --L 256 --rounds 5 --check --variants "TSA_LAP_M=1" "TSA_LAP_M=2" || exit 1
run --n 1 --L 1024 --rounds 5 --score-bits 16 --preload --variants "TSA_NONE=0" || exit 1
for i in 1 2; do
  echo "== helix M" >> $O/helix_m.jsonl
  timeout -k 10 150 python tools/bench_variants.py --n 512 --L 256 --rounds 5 \
    --variants "TSA_PENCIL_MODE=helix" "TSA_PENCIL_MODE=helix,TSA_PENCIL_ARITH=f16" >> $O/helix_m.jsonl 2>> $O/helix_m.err || exit 1
  timeout -k 10 150 python tools/bench_variants.py --n 256 --L 512 --rounds 3 \
    --variants "TSA_PENCIL_MODE=helix,TSA_PENCIL_ARITH=f16" >> $O/helix_m.jsonl 2>> $O/helix_m.err || exit 1
done
cat $O/single_ab.jsonl $O/lapab.jsonl $O/helix_m.jsonl
