#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TSA_EXPECT_GPU=1
TAG=${TAG:-r4d}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
# single cubes: the r4b build (before the round loop) vs this tree, same box, spin preload
for i in 1 2; do
  for pk in variants/r4b hw-accelerator-three-sequence-alignment_amd; do
    for L in 64 256 512; do
      echo "== $pk $L" >> $O/single_ab.jsonl
      TSA_PKG_DIR=$GRAFT_REPO_ROOT/$pk timeout -k 10 120 python tools/bench_variants.py --n 1 --L $L --rounds 9 --preload --variants "TSA_NONE=0" >> $O/single_ab.jsonl 2>> $O/single_ab.err || exit 1
    done
  done
done
cat $O/single_ab.jsonl
run() { echo "== $*" >> $O/lapab.jsonl; timeout -k 10 300 python tools/bench_variants.py "$@" >> $O/lapab.jsonl 2>> $O/lapab.err; }
run --n 8 --L 512 --rounds 5 --check --variants "TSA_LAP_M=1" "TSA_LAP_M=2" "TSA_LAP_M=2,TSA_LAP_CHUNK=4" || exit 1
run --n 16 --L 256 --rounds 5 --check --variants "TSA_LAP_M=1" "TSA_LAP_M=2" || exit 1
cat $O/lapab.jsonl
timeout -k 10 600 python bench.py --profile-dir "$GRAFT_REPO_ROOT/$O/bench_profile" > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
TAG=$TAG KERNELS=pencil bash scripts/gpu_profile.sh
