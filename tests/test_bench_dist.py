"""Multi-rank path of bench.py on CPU (gloo, world_size 2): utterances shard across ranks
with no data-path collective; the timed region is barrier-bracketed, elapsed is the MAX over
ranks and audio is the SUM over ranks (weak scaling)."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import time

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seeds = []

    def utterance(seed, record):
        # rank 1 is deliberately slower: the reported elapsed must be the slower rank's
        time.sleep(0.05 * (rank + 1))
        if record:
            seeds.append(seed)
        return 1000 + rank

    elapsed, samples = bench.timed_region(1, 3, 2, rank, utterance, lambda: None, dist.barrier, dist)
    q.put((rank, elapsed, samples, seeds))
    dist.destroy_process_group()


def test_timed_region_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (r0, e0, s0, seeds0), (r1, e1, s1, seeds1) = res
    # max over ranks: both ranks report the same elapsed, at least the slow rank's 6 x 0.1 s
    assert e0 == pytest.approx(e1) and e0 >= 0.6
    # sum over ranks: 6 timed utterances per rank
    assert s0 == s1 == 6 * 1000 + 6 * 1001
    # every rank runs its own distinct utterances (no shared or replayed work)
    assert len(seeds0) == len(seeds1) == 6
    assert not set(seeds0) & set(seeds1) and len(set(seeds0)) == 6


def test_timed_region_single_rank():
    import bench

    n = []
    elapsed, samples = bench.timed_region(2, 4, 1, 0, lambda seed, rec: n.append(rec) or 7,
                                          lambda: None, lambda: None, None)
    assert samples == 28 and n.count(False) == 2 and n.count(True) == 4 and elapsed >= 0


def test_bench_launcher_spawns_ranks():
    """`bench.py --gpus 2` without torchrun: the parent starts 2 fresh child ranks (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set, gloo rendezvous on 127.0.0.1) before any GPU use
    and exits with their status; rank 0 prints one line with n_gpus = 2 and the SUM of both
    ranks' audio over the MAX elapsed."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--launcher-selftest"], capture_output=True, text=True, timeout=180,
                       env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["samples"] == 2 * 3 * 1000
    assert r["elapsed"] >= 3 * 0.04  # the slower rank (rank 1) sets the time
