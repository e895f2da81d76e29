#!/bin/bash
# Round 3: literal helix M = 4 (LC <= 512): literal GPU tests, then timing
# literal vs PLANE on 512^3-class batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "literal or golden or plane" --timeout 120 --timeout-method thread > gpurun_out/pytest_r3k.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r3k.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r3k.log | head; exit $rc; }
BV="python tools/bench_variants.py --kernel plane --check"
for spec in "64 512" "16 384" "4 512"; do
  set -- $spec
  timeout -k 10 300 $BV --n $1 --L $2 --rounds 3 --variants TSA_PENCIL_MODE=literal TSA_PENCIL_MODE=plane >> gpurun_out/r3k_lit4.jsonl 2>> gpurun_out/r3k_lit4.err || exit 1
done
cat gpurun_out/r3k_lit4.jsonl
