#!/bin/bash
# Lap-kernel bring-up: its parity tests, then single-cube timings over the
# (M, NW) knobs and the helix, then a lap trace of the default 256^3 plan.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -k "${TESTS:-lap or single_cube or 512 or timeout or 1024 or wide or two or full_shard or ragged or async or geometries}" \
  > gpurun_out/pytest_lap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lap.log; [ $rc -eq 0 ] || exit $rc
V="TSA_PENCIL_MODE=helix"; for m in 1 2 4; do for nw in 4 8; do V="$V TSA_PENCIL_MODE=lap,TSA_LAP_M=$m,TSA_LAP_NW=$nw"; done; done
for L in 64 128 256 512; do
  timeout -k 10 200 python tools/bench_variants.py --n 1 --L $L --rounds 7 --check --variants $V \
    > gpurun_out/lap_$L.json 2> gpurun_out/lap_$L.err || { tail -5 gpurun_out/lap_$L.err; exit 1; }
  echo "L=$L"; cat gpurun_out/lap_$L.json
done
timeout -k 10 300 python tools/bench_variants.py --n 1 --L 1024 --rounds 3 --score-bits 16 \
  --variants TSA_PENCIL_MODE=lap,TSA_LAP_M=1,TSA_LAP_NW=8 TSA_PENCIL_MODE=lap,TSA_LAP_M=2,TSA_LAP_NW=4 TSA_PENCIL_MODE=lap,TSA_LAP_M=2,TSA_LAP_NW=8 TSA_PENCIL_MODE=lap,TSA_LAP_M=4,TSA_LAP_NW=8 \
  > gpurun_out/lap_1024.json 2> gpurun_out/lap_1024.err || { tail -5 gpurun_out/lap_1024.err; exit 1; }
echo "L=1024"; cat gpurun_out/lap_1024.json
for n in 4 16 32; do
  timeout -k 10 200 python tools/bench_variants.py --n $n --L 256 --rounds 5 --check \
    --variants TSA_PENCIL_MODE=helix TSA_PENCIL_MODE=lap \
    > gpurun_out/lapn_$n.json 2> gpurun_out/lapn_$n.err || { tail -5 gpurun_out/lapn_$n.err; exit 1; }
  echo "n=$n"; cat gpurun_out/lapn_$n.json
done
timeout -k 10 120 python tools/lap_trace.py 64 128 256 > gpurun_out/lap_trace.jsonl; echo "trace rc=$?"
