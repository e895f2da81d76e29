#!/bin/bash
# Single-cube (lap kernel) knob sweep: tile width and rows per lap, 256^3 and 1024^3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_variants.py --n 1 --L 256 --rounds 7 --check \
  --variants "TSA_LAP_ZT=128" "TSA_LAP_ZT=256" "TSA_LAP_ZT=128,TSA_LAP_NW=8" "TSA_LAP_ZT=256,TSA_LAP_NW=8" \
  > gpurun_out/single256.json 2> gpurun_out/single256.err || { tail -5 gpurun_out/single256.err; exit 1; }
cat gpurun_out/single256.json
timeout -k 10 300 python tools/bench_variants.py --n 1 --L 1024 --rounds 3 --score-bits 16 \
  --variants "TSA_LAP_ZT=128" "TSA_LAP_ZT=256" "TSA_LAP_ZT=512" \
  > gpurun_out/single1024.json 2> gpurun_out/single1024.err || { tail -5 gpurun_out/single1024.err; exit 1; }
cat gpurun_out/single1024.json
