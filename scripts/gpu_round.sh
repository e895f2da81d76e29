#!/bin/bash
# One GPU call: the parity tests, the bench line (which runs its own rocprofv3
# kernel-trace child on the same box), then the PMC passes of the bench's
# profiled child (scripts/gpu_profile.sh). Stops at the first failure; every
# GPU step has its own time limit. Results under gpurun_out/<TAG>/.
#   TAG=r4b bash scripts/gpu_round.sh          (NOTEST=1 / NOPROF=1 skip steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${TAG:-r4}; O=gpurun_out/$TAG; mkdir -p $O
export TSA_EXPECT_GPU=1
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py --profile-dir "$GRAFT_REPO_ROOT/$O/bench_profile" ${BENCH_ARGS} \
  > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
[ -n "$NOPROF" ] && exit 0
TAG=$TAG KERNELS=${KERNELS:-pencil} bash scripts/gpu_profile.sh
