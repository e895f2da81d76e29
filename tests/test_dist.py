"""The N>1 path on CPU: world-size-2 gloo processes shard a batch of triples
contiguously, score their block (the CPU oracle stands in for the GPU here),
all-gather the int32 scores and take the max-over-ranks time -- exactly the
collective pattern bench.py uses over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, L, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import load_pkg  # noqa: E402
    load_pkg()
    import importlib
    shard = importlib.import_module("tsa_amd.shard")
    synth = importlib.import_module("tsa_amd.synth")
    import oracle
    i0, i1 = shard.shard_range(n_total, rank, world)
    seqs, offs = synth.batch(i0, i1 - i0, L)
    local = torch.from_numpy(oracle.score_batch(seqs, offs - offs[0], nthreads=1))
    allsc = shard.gather_scores(local, n_total, world)
    tmax = shard.max_over_ranks(float(rank + 1), torch.device("cpu"))
    if rank == 0:
        q.put((allsc.numpy().tolist(), tmax))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [7, 8])
def test_gloo_world2_shard_and_gather(tsa, orc, n_total):
    L = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, L, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import importlib
    synth = importlib.import_module("tsa_amd.synth")
    seqs, offs = synth.batch(0, n_total, L)
    assert got == orc.score_batch(seqs, offs).tolist()
    assert tmax == 2.0


def test_shard_ranges_cover_exactly(tsa):
    import importlib
    shard = importlib.import_module("tsa_amd.shard")
    for n in (1, 5, 512, 4096, 4097):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


@pytest.mark.parametrize("per_gpu", [3, 4])
def test_bench_spawn_world2_gloo(tsa, orc, per_gpu):
    """bench.py's own N>1 path: spawn_ranks starts 2 rank processes with the
    torch.distributed env set, run_rank shards contiguously, times between
    barriers, takes the max over ranks and all-gathers the scores; rank 0
    prints one JSON line with n_gpus 2. The oracle scores each rank's block
    (CPU stand-in for the GPU, tests/_bench_cpu_rank.py)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "_bench_cpu_rank.py"),
                        "--gpus", "2", "--per-gpu", str(per_gpu), "--length", "12",
                        "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["world_size"] == 2
    assert rec["config"]["triples_total"] == 2 * per_gpu and rec["scaling"] == "weak"
    assert rec["steps"] == 2 and rec["value"] > 0
    assert rec["gathered"] == rec["oracle"] and len(rec["gathered"]) == 2 * per_gpu


def test_bench_spawn_world8_record_fields(tsa, orc):
    """The driver's N = 8 line: bench.py's spawn path with 8 gloo ranks (CPU
    stand-in, tests/_bench_cpu_rank.py) prints one record whose
    config.devices.dist_world_size is 8, whose split-over-devices leg is laid
    over devices 0..7, and whose gathered scores equal the oracle's."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "_bench_cpu_rank.py"),
                        "--gpus", "8", "--per-gpu", "1", "--length", "8",
                        "--steps", "1", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["config"]["world_size"] == 8
    assert rec["config"]["devices"]["dist_world_size"] == 8
    assert rec["config"]["devices"]["backend"] == "gloo"
    assert rec["config"]["split_devices"] == "0,1,2,3,4,5,6,7"
    assert rec["gathered"] == rec["oracle"] and len(rec["gathered"]) == 8
    assert rec["fallbacks"]["all_zero"] is True


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
