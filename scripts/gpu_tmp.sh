#!/bin/bash
# scratch: lap GPU tests, then lap A/B (LIBS) on single cubes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "lap or single_cube or 512 or timeout or 1024 or async or geometries or checked or packed" > gpurun_out/pytest_lap.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_lap.log | tail -10; tail -2 gpurun_out/pytest_lap.log; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS}" SPECS="${SPECS:-64 128 256 512}" bash scripts/gpu_lapvar.sh
