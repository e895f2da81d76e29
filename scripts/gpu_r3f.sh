#!/bin/bash
# Round 3: the M = 2 lap kernel at 80 VGPRs (two 9-wave workgroups per CU) vs
# 96 (variants/wpe5), single cubes 768^3 / 1024^3 (16-bit) and 1024^3 checked
# 12-bit, interleaved; the residency census of the diag build; lap parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "lap or 1024 or checked or split or 512_cube or configs4" \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r3f.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in cur wpe5; do
    if [ $v = cur ]; then unset TSA_PKG_DIR; else export TSA_PKG_DIR=$GRAFT_REPO_ROOT/variants/$v; fi
    timeout -k 10 200 python tools/lap_trace.py --bits 16 --reps 5 768 1024 > gpurun_out/wpe_${v}_$rep.jsonl 2> gpurun_out/wpe_$v.err || exit 1
    timeout -k 10 200 python tools/lap_trace.py --bits 12 --reps 5 --kernel checked 1024 >> gpurun_out/wpe_${v}_$rep.jsonl 2>> gpurun_out/wpe_$v.err
    python3 -c "
import json
for l in open('gpurun_out/wpe_${v}_$rep.jsonl'):
    r=json.loads(l); print('$v', r['spec'], r['plan'], r['us_median'], r.get('bp_waits'), r.get('lap_end_lag_us'))"
  done
done
unset TSA_PKG_DIR
TSA_PKG_DIR=$GRAFT_REPO_ROOT/variants/diag timeout -k 10 200 python tools/lap_trace.py --bits 16 --reps 3 \
  1024:TSA_LAP_FULL_RINGS=1 768:TSA_LAP_FULL_RINGS=1 > gpurun_out/lap_lag_wpe6.jsonl 2> gpurun_out/lap_lag_wpe6.err || exit 1
python3 -c "
import json,csv,collections
for l in open('gpurun_out/lap_lag_wpe6.jsonl'):
    r=json.loads(l); print(r['spec'], r['us_median'], r.get('lag_y'), r.get('lag_z'))
for fn in ['gpurun_out/lap_trace_1024_TSA_LAP_FULL_RINGS=1.csv']:
    rows=list(csv.DictReader(open(fn))); t0=min(int(r['start']) for r in rows)
    st=collections.defaultdict(list)
    for r in rows: st[int(r['lap'])].append((int(r['start'])-t0)/100.0)
    print('start us per lap', [round(max(v),1) for k,v in sorted(st.items())][::4])"
