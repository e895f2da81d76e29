#!/bin/bash
# GPU box recipe: parity tests, then the bench (one JSON line), each under
# its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for k in ${BENCH_KERNELS:-auto}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --kernel $k ${BENCH_ARGS} > gpurun_out/bench_$k.json 2> gpurun_out/bench_$k.err
  rc=$?; echo "bench $k rc=$rc"; cat gpurun_out/bench_$k.json
  [ $rc -eq 0 ] || exit $rc
done
