#!/bin/bash
# One GPU call: parity tests, the bench line, then the rocprof trace + PMC
# passes of the pencil batch kernel (scripts/gpu_profile.sh). Stops at the
# first failure; every GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
[ -n "$NOPROF" ] && exit 0
KERNELS=${KERNELS:-pencil} bash scripts/gpu_profile.sh
