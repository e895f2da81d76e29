#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_variants.py --check --n 1 --rounds 20 --variants TSA_LAP_ZT=128 TSA_LAP_ZT=256 "TSA_LAP_ZT=128,TSA_LAP_NW=8" > gpurun_out/single.json 2> gpurun_out/single.err
rc=$?; echo "single rc=$rc"; cat gpurun_out/single.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_variants.py --check --n 1 --L 1024 --rounds 3 --score-bits 16 --variants TSA_LAP_ZT=128 TSA_LAP_ZT=256 TSA_LAP_ZT=1024 "TSA_LAP_ZT=128,TSA_LAP_NW=8" > gpurun_out/c4.json 2> gpurun_out/c4.err
rc=$?; echo "c4 rc=$rc"; cat gpurun_out/c4.json; exit $rc
