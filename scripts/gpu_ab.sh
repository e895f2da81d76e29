#!/bin/bash
# Parity (full GPU suite) then an A/B of pencil variants given in $VARIANTS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_variants.py --check --n ${N:-512} --variants ${VARIANTS} > gpurun_out/variants.json 2> gpurun_out/variants.err
rc=$?; echo "variants rc=$rc"; cat gpurun_out/variants.json; [ $rc -eq 0 ] || tail -20 gpurun_out/variants.err; exit $rc
