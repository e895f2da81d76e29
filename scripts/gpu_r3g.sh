#!/bin/bash
# Round 3: lap grids in dispatch rounds with boundary rings -- timings and
# start stamps per M (TSA_LAP_M) at 768^3 / 1024^3, small cubes, checked
# 1024^3; then the lap parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
summ() { python3 -c "
import json,csv,collections,re,os
for l in open('$1'):
    r=json.loads(l)
    fn='gpurun_out/lap_trace_'+re.sub(r'[^0-9A-Za-z_=.-]','_',r['spec'])+'.csv'
    late=''
    if os.path.exists(fn):
        rows=list(csv.DictReader(open(fn))); t0=min(int(x['start']) for x in rows)
        st=sorted(((int(x['block'])>>3),(int(x['start'])-t0)/100) for x in rows if int(x['xcc'])==0)
        lt=[s for s,t in st if t>50]; late='first late slot %s of %d'%(lt[0] if lt else None, len(st))
    print(r['spec'], r['plan'], r['score'], r['us_median'], 'bp', r.get('bp_waits'), 'stalls', r.get('stalls'), late)"; }
timeout -k 10 300 python tools/lap_trace.py --bits 16 --reps 5 768 1024 > gpurun_out/r3g_lap.jsonl 2> gpurun_out/r3g_lap.err; rc=$?; summ gpurun_out/r3g_lap.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/r3g_lap.err; exit $rc; }
timeout -k 10 200 python tools/lap_trace.py --bits 12 --reps 5 64 128 256 512 > gpurun_out/r3g_small.jsonl 2> gpurun_out/r3g_small.err; rc=$?; summ gpurun_out/r3g_small.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/lap_trace.py --bits 12 --reps 5 --kernel checked 1024 > gpurun_out/r3g_chk.jsonl 2> gpurun_out/r3g_chk.err; rc=$?; summ gpurun_out/r3g_chk.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_r3g.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r3g.log; exit $rc
