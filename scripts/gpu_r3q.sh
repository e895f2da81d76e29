#!/bin/bash
# Round 3: literal split over devices (LIT + SYS lap) -- split, literal-lap and
# chunk GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu -k "split or literal_lap or chunk" \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_r3q.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r3q.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r3q.log | head -20; exit $rc; }
timeout -k 10 200 python tools/split_cube.py --devices 0,0 --lengths 1024,1024r --reps 3 > gpurun_out/r3q_split.json 2> gpurun_out/r3q_split.err; rc=$?
cat gpurun_out/r3q_split.json; exit $rc
