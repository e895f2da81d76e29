#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench, one pass per kernel, then the
# PMC passes for HBM bytes (FETCH_SIZE and WRITE_SIZE in separate runs, as
# MI355X_MICROARCH.md prescribes) and for VALU instructions (SQ_INSTS_VALU). Outputs under gpurun_out/prof_<tag>/.
set -o pipefail
R="$GRAFT_REPO_ROOT"
TAG=${TAG:-r2}
cd /tmp && export TMPDIR=/tmp
for k in ${KERNELS:-pencil plane}; do
  OUT="$R/gpurun_out/prof_${TAG}/$k"
  mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --kernel $k --no-cpu-baseline --no-extra-configs ${BENCH_ARGS} \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "trace $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps 1 --warmup 0 --kernel $k --no-cpu-baseline --no-extra-configs ${BENCH_ARGS} \
      > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
    rc=$?; echo "pmc $c $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
