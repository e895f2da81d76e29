#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "pencil or golden" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_variants.py --check --n 512 --rounds 4 --variants TSA_PENCIL_NW=16 TSA_PENCIL_NW=8 "TSA_PENCIL_NW=8,TSA_PENCIL_STAGGER=14" "TSA_PENCIL_NW=8,TSA_PENCIL_STAGGER=28" > gpurun_out/batch.json 2> gpurun_out/batch.err
rc=$?; echo "batch rc=$rc"; cat gpurun_out/batch.json; exit $rc
