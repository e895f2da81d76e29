set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TSA_EXPECT_GPU=1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
cat gpurun_out/bench.json
