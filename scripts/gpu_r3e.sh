#!/bin/bash
# Round 3: ring-lag census of the lap kernel (TSA_DIAG build, full rings: no
# back-pressure) at 512^3 / 768^3 / 1024^3 (16-bit words), and 1024^3 with the
# default rings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TSA_PKG_DIR=$GRAFT_REPO_ROOT/variants/diag timeout -k 10 300 python tools/lap_trace.py --bits 16 --reps 3 \
  512:TSA_LAP_FULL_RINGS=1 768:TSA_LAP_FULL_RINGS=1 1024:TSA_LAP_FULL_RINGS=1 1024 > gpurun_out/lap_lag.jsonl 2> gpurun_out/lap_lag.err
rc=$?; python3 -c "
import json,sys
for l in open('gpurun_out/lap_lag.jsonl'):
    r=json.loads(l); print(r['spec'], r['plan'], r['us_median'], r.get('bp_waits'), r.get('lag_y'), r.get('lag_z'))"
exit $rc
