#!/bin/bash
# rocprofv3 of the bench's profiled child (bench.py --profile-child: the batch
# launches, then the configs[2] single cube): one kernel-trace + stats pass,
# then the PMC passes -- FETCH_SIZE and WRITE_SIZE in separate runs for HBM
# bytes (MI355X_MICROARCH.md's recipe) and SQ_INSTS_VALU for VALU
# instructions. Outputs under gpurun_out/prof_<TAG>/<kernel>/; summarise with
# python3 tools/pmc_traffic.py <TAG> (writes profiles/pmc_*.json, stamped).
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${TAG:-r4}
cd /tmp && export TMPDIR=/tmp
for k in ${KERNELS:-pencil}; do
  OUT="$R/gpurun_out/prof_${TAG}/$k"
  mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$R/bench.py" --profile-child --steps 10 --warmup 3 --kernel $k ${BENCH_ARGS} \
    > "$OUT/child.out" 2> "$OUT/child.err"
  rc=$?; echo "trace $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv \
      -- python3 "$R/bench.py" --profile-child --steps 2 --warmup 1 --kernel $k ${BENCH_ARGS} \
      > "$OUT/pmc_$c.out" 2> "$OUT/pmc_$c.err"
    rc=$?; echo "pmc $c $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
