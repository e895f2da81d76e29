#!/bin/bash
# Round 3: chunked lap launches -- chunk GPU tests + lap/literal tests, then
# lap (chunked) vs helix on batches of mid-size and large cubes, factored and
# literal, to fit the cost model.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "chunk or lap or literal or checked" \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_r3o.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r3o.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r3o.log | head -20; exit $rc; }
for spec in "4 256" "16 256" "32 256" "64 256" "128 256" "8 512" "4 1024"; do
  set -- $spec
  timeout -k 10 300 python tools/bench_variants.py --kernel pencil --check --rounds 3 --n $1 --L $2 --score-bits 16 \
    --variants TSA_PENCIL_MODE=lap TSA_PENCIL_MODE=helix >> gpurun_out/r3o_chunk.jsonl 2>> gpurun_out/r3o.err || { tail -5 gpurun_out/r3o.err; exit 1; }
done
for spec in "4 256" "16 256" "64 256" "8 512" "2 1024"; do
  set -- $spec
  V="TSA_PENCIL_MODE=litlap TSA_PENCIL_MODE=plane"; [ $2 -le 512 ] && V="$V TSA_PENCIL_MODE=literal"
  timeout -k 10 300 python tools/bench_variants.py --kernel plane --check --rounds 3 --n $1 --L $2 \
    --variants $V >> gpurun_out/r3o_chunk.jsonl 2>> gpurun_out/r3o.err || { tail -5 gpurun_out/r3o.err; exit 1; }
done
cat gpurun_out/r3o_chunk.jsonl
