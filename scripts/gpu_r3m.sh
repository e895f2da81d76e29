#!/bin/bash
# Round 3 final-tree check: every GPU test, the bench line, the rocprof trace +
# PMC passes of the helix batch kernel (gpu_profile.sh, TAG=r3m), and a
# rocprof kernel trace of the literal lap at 1024^3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
NOPROF=1 bash scripts/gpu_round.sh || exit $?
TAG=r3m KERNELS=pencil bash scripts/gpu_profile.sh || exit $?
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_r3m_litlap"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/tools/bench_variants.py" --kernel plane --n 1 --L 1024 --rounds 9 \
  --variants TSA_PENCIL_MODE=litlap > "$OUT/bv.json" 2> "$OUT/bv.err"
rc=$?; echo "litlap trace rc=$rc"; cat "$OUT/bv.json"; exit $rc
