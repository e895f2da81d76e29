#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_variants.py --check --n 1 --rounds 20 --variants TSA_LAP_NW=16 TSA_LAP_NW=8 TSA_LAP_NW=4 TSA_PENCIL_MODE=helix > gpurun_out/single.json 2> gpurun_out/single.err
rc=$?; echo "single rc=$rc"; cat gpurun_out/single.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_variants.py --check --n 512 --rounds 5 --variants TSA_PENCIL_NW=8 TSA_PENCIL_NW=16 > gpurun_out/batch.json 2> gpurun_out/batch.err
rc=$?; echo "batch rc=$rc"; cat gpurun_out/batch.json; exit $rc
