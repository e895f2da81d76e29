#!/bin/bash
# Round 3: literal lap (lap_kernel LIT) -- parity tests, then literal lap vs
# literal helix vs PLANE sweep on single cubes / small batches, then the bench
# line (the split-over-devices leg with parts serialised per device).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "literal_lap or split_cube or literal_helix or golden_final" \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_r3l.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r3l.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r3l.log | head -20; exit $rc; }
BV="python tools/bench_variants.py --kernel plane --check --rounds 5"
for spec in "1 64" "1 128" "1 256" "4 256" "16 256" "1 512" "1 1024"; do
  set -- $spec
  V="TSA_PENCIL_MODE=litlap TSA_PENCIL_MODE=plane"
  [ $2 -le 512 ] && V="$V TSA_PENCIL_MODE=literal"
  timeout -k 10 300 $BV --n $1 --L $2 --variants $V >> gpurun_out/r3l_litlap.jsonl 2>> gpurun_out/r3l_litlap.err || { tail -5 gpurun_out/r3l_litlap.err; exit 1; }
done
cat gpurun_out/r3l_litlap.jsonl
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['parity']['mismatches'], d['single_cube'].get('split over devices'))"
exit $rc
