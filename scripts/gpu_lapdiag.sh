#!/bin/bash
# Lap-kernel diagnostics: per-step time (us, shader cycles), lap-to-lap lag and
# stalls of single cubes over (M, NW), chained and unchained (LB = one lap).
# SPECS overrides the list (tools/lap_trace.py SPEC syntax).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TSA_PKG_DIR=${TSA_PKG_DIR:-$GRAFT_REPO_ROOT/variants/diag}  # TSA_LAP_SINGLE needs the -DTSA_DIAG build
S=${SPECS:-"64:TSA_LAP_M=1,TSA_LAP_NW=8 64:TSA_LAP_M=1,TSA_LAP_NW=4 64x16x64:TSA_LAP_M=1,TSA_LAP_NW=8,TSA_LAP_SINGLE=1 64x8x64:TSA_LAP_M=1,TSA_LAP_NW=4,TSA_LAP_SINGLE=1 128 256 256x16x256:TSA_LAP_M=2,TSA_LAP_NW=8,TSA_LAP_SINGLE=1"}
timeout -k 10 300 python tools/lap_trace.py $S > gpurun_out/lapdiag.jsonl 2> gpurun_out/lapdiag.err
rc=$?; cat gpurun_out/lapdiag.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/lapdiag.err; exit $rc; }
