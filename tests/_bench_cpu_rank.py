"""Helper (not a test module): runs bench.py's own rank code -- spawn_ranks,
run_rank, the contiguous shard, the score all-gather and the max-over-ranks
time -- on CPU over gloo, with the CPU oracle standing in for the GPU scorer
(test infrastructure: the product path has no CPU scorer). Driven by
tests/test_dist.py::test_bench_spawn_world2_gloo.

    python tests/_bench_cpu_rank.py --gpus 2 --per-gpu 3 --length 12 ...
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402


class OracleBatch:
    """GpuBatch's interface on the CPU oracle (checker only)."""

    def __init__(self, tsa, dev, seqs, offs, n, L, params, kernel):
        import torch
        import oracle
        self.torch, self.oracle = torch, oracle
        self.seqs, self.offs, self.n = seqs, offs, n
        self.out = torch.zeros(max(n, 1), dtype=torch.int32)

    def step(self):
        if self.n:
            self.out[: self.n] = self.torch.from_numpy(
                self.oracle.score_batch(self.seqs, self.offs, nthreads=1))

    def sync(self):
        pass

    def mark(self):
        import time
        return time.perf_counter()

    @staticmethod
    def elapsed_ms(e0, e1):
        return (e1 - e0) * 1e3

    def scores(self):
        return self.out[: self.n]


def main():
    args = bench.parse_args()
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(bench.spawn_ranks(args.gpus, sys.argv[1:], script=os.path.abspath(__file__)))
    import torch
    import oracle

    def check(rec, scores):
        synth = sys.modules["tsa_amd.synth"]
        seqs, offs = synth.batch(0, len(scores), args.length)
        rec["gathered"] = [int(v) for v in scores]
        rec["oracle"] = [int(v) for v in oracle.score_batch(seqs, offs, nthreads=1)]

    rec = bench.run_rank(args, int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                         int(os.environ.get("LOCAL_RANK", "0")), "gloo", OracleBatch,
                         device=torch.device("cpu"), extras=False, on_scores=check)
    if rec is not None:
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
