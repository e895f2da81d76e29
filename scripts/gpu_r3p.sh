#!/bin/bash
# Round 3 final-tree check after chunked lap launches: every GPU test, the
# bench line, the helix rocprof + PMC passes (TAG=r3p), and the new plan
# points (chunked factored lap at 64 x 256^3, literal lap vs helix at 512 x 64^3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
NOPROF=1 bash scripts/gpu_round.sh || exit $?
TAG=r3p KERNELS=pencil bash scripts/gpu_profile.sh || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_variants.py --kernel pencil --check --rounds 5 --n 64 --L 256 --score-bits 16 \
  --variants TSA_PENCIL_MODE=lap TSA_PENCIL_MODE=helix >> gpurun_out/r3p_plan.jsonl 2>> gpurun_out/r3p.err || exit 1
timeout -k 10 300 python tools/bench_variants.py --kernel plane --check --rounds 5 --n 512 --L 64 \
  --variants TSA_PENCIL_MODE=litlap TSA_PENCIL_MODE=literal >> gpurun_out/r3p_plan.jsonl 2>> gpurun_out/r3p.err || exit 1
timeout -k 10 300 python tools/bench_variants.py --kernel plane --check --rounds 5 --n 128 --L 256 \
  --variants TSA_PENCIL_MODE=litlap TSA_PENCIL_MODE=literal >> gpurun_out/r3p_plan.jsonl 2>> gpurun_out/r3p.err || exit 1
cat gpurun_out/r3p_plan.jsonl
