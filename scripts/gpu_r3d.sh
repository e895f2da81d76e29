#!/bin/bash
# Round 3 GPU pass: every gpu test, same-box A/B of the helix against the
# previous build (variants/r3prev), literal helix vs PLANE, ring-lag census.
export TSA_EXPECT_GPU=1
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r3d.log; [ $rc -eq 0 ] || exit $rc
LIBS=r3prev bash scripts/gpu_libab.sh || exit 1
bash scripts/gpu_literal.sh r3c_lit || exit 1
bash scripts/gpu_r3e.sh
