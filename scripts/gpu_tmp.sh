#!/bin/bash
# scratch: full GPU tests, then PLANE timings (batch 512 x 256^3, single 1024^3 12-bit)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_all.log | tail -10; tail -2 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --kernel plane --steps 2 --warmup 1 --no-cpu-baseline --no-extra-configs > gpurun_out/bench_plane.json 2> gpurun_out/bench_plane.err
rc=$?; echo "plane bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_plane.err; exit $rc; }
python -c "import json; r=json.load(open('gpurun_out/bench_plane.json')); print('plane batch', r['value'], 'GCUPS', r['ms_per_step'], 'ms')"
timeout -k 10 200 python tools/bench_variants.py --n 1 --L 1024 --kernel plane --rounds 3 --variants TSA_NOOP=1 > gpurun_out/plane1024.json 2> gpurun_out/plane1024.err
rc=$?; cat gpurun_out/plane1024.json; exit $rc
