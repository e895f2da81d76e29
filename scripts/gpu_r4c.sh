#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TSA_EXPECT_GPU=1
TAG=${TAG:-r4c}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for L in 64 128 256; do
  echo "== lap VS vs f16 $L" >> $O/lapvs.jsonl
  timeout -k 10 120 python tools/bench_variants.py --n 1 --L $L --rounds 15 --preload --check --variants "TSA_NONE=0" "TSA_PENCIL_ARITH=f16" >> $O/lapvs.jsonl 2>> $O/lapvs.err || exit 1
done
cat $O/lapvs.jsonl
for i in 1 2; do
  for pk in variants/prev hw-accelerator-three-sequence-alignment_amd; do
    echo "== helix $pk" >> $O/helix_ab.jsonl
    TSA_PKG_DIR=$GRAFT_REPO_ROOT/$pk timeout -k 10 120 python tools/bench_variants.py --n 512 --L 256 --rounds 5 --variants "TSA_NONE=0" >> $O/helix_ab.jsonl 2>> $O/helix_ab.err || exit 1
  done
done
cat $O/helix_ab.jsonl
TAG=$TAG bash scripts/gpu_lapab.sh; rc=$?; echo "lapab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --profile-dir "$GRAFT_REPO_ROOT/$O/bench_profile" > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
