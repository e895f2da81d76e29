#!/bin/bash
# scratch: GPU tests of the lap / checked kernels, then the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "checked or lap or 512 or 1024 or async or geometries" > gpurun_out/pytest_chk.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_chk.log | tail -40; tail -3 gpurun_out/pytest_chk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
