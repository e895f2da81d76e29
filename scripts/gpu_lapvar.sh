#!/bin/bash
# Lap diagnostics (tools/lap_trace.py) for the in-tree package and each
# variants/<name> variant in $LIBS (scripts/build_variant.sh; timing-only
# experiment builds allowed). TESTS=1 first runs the lap kernel's GPU parity
# tests on the in-tree package.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  TSA_EXPECT_GPU=1 timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    -k "lap or single_cube or 512 or timeout or 1024 or async or geometries or checked or packed" > gpurun_out/pytest_lap.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_lap.log; [ $rc -eq 0 ] || exit $rc
fi
S=${SPECS:-"64x16x64:TSA_LAP_M=1,TSA_LAP_NW=8,TSA_LAP_SINGLE=1 64x8x64:TSA_LAP_M=1,TSA_LAP_NW=4,TSA_LAP_SINGLE=1 64:TSA_LAP_M=1,TSA_LAP_NW=8 64:TSA_LAP_M=1,TSA_LAP_NW=4"}
for which in cur ${LIBS}; do
  if [ $which = cur ]; then unset TSA_PKG_DIR; else export TSA_PKG_DIR=$GRAFT_REPO_ROOT/variants/$which; fi
  timeout -k 10 200 python tools/lap_trace.py $S > gpurun_out/lapvar_$which.jsonl 2> gpurun_out/lapvar_$which.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/lapvar_$which.err; exit $rc; }
  echo "== $which"; python -c "
import json,sys
for l in open('gpurun_out/lapvar_$which.jsonl'):
    r=json.loads(l); print(r['spec'], r['us_median'], r.get('step_clk'), r.get('stalls'))"
done
