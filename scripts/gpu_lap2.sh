#!/bin/bash
# Lap-kernel bring-up: its GPU parity tests, then tools/lap_trace.py diagnostics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "${TESTS:-lap or single_cube or 512 or timeout or 1024 or async or geometries}" \
  > gpurun_out/pytest_lap.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_lap.log | tail -40; tail -3 gpurun_out/pytest_lap.log; [ $rc -eq 0 ] || exit $rc
S=${SPECS:-"64:TSA_LAP_M=1,TSA_LAP_NW=8 64:TSA_LAP_M=1,TSA_LAP_NW=4 64x16x64:TSA_LAP_M=1,TSA_LAP_NW=8,TSA_LAP_SINGLE=1 64x8x64:TSA_LAP_M=1,TSA_LAP_NW=4,TSA_LAP_SINGLE=1 128 128:TSA_LAP_M=1,TSA_LAP_NW=4 256 256:TSA_LAP_M=1,TSA_LAP_NW=4 512"}
timeout -k 10 300 python tools/lap_trace.py $S > gpurun_out/lapdiag.jsonl 2> gpurun_out/lapdiag.err
rc=$?; cat gpurun_out/lapdiag.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/lapdiag.err; exit $rc; }
