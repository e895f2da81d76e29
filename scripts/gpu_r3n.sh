#!/bin/bash
# Round 3: PLANE sweep with DPP z-1 exchange -- plane/traceback/golden GPU
# tests, then plane-sweep timings (compare profiles/r3l_literal_lap_vs_plane.jsonl).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "plane or align or golden or wrap or params or edge or ragged" \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_r3n.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r3n.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r3n.log | head -20; exit $rc; }
BV="python tools/bench_variants.py --kernel plane --check --rounds 5 --variants TSA_PENCIL_MODE=plane"
for spec in "1 256" "16 256" "1 1024" "512 256"; do
  set -- $spec
  timeout -k 10 300 $BV --n $1 --L $2 >> gpurun_out/r3n_plane.jsonl 2>> gpurun_out/r3n_plane.err || { tail -5 gpurun_out/r3n_plane.err; exit 1; }
done
cat gpurun_out/r3n_plane.jsonl
