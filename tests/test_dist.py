"""CPU, world_size 2 over gloo: the multi-GPU data path of bench.py.  Tiles shard with
the greedy byte-balanced split and no data-path collective; the only collectives are the timing
barrier and the max/sum reductions of the per-rank numbers."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    lib = bench.tile_library()
    allp = bench.sample_batch(lib, 600, bench.SEED)
    shards = bench.lpt_shards([len(t) for _, t in allp], world)
    mine = shards[rank]
    covt = bench.load_covt()
    plan = covt.Plan.from_tiles([allp[i][1] for i in mine])
    assert (plan.tile_status == 0).all()
    # gather shard membership and per-rank stream bytes
    got = [None] * world
    dist.all_gather_object(got, (mine, plan.in_bytes, plan.num_streams))
    stats = torch.tensor([float(rank + 1), float(plan.in_bytes)], dtype=torch.float64)
    mx, sm = stats.clone(), stats.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    weak = [k for k, _ in bench.sample_batch(lib, 50, bench.SEED + rank)]
    wk = [None] * world
    dist.all_gather_object(wk, weak)
    if rank == 0:
        q.put((got, float(mx[0]), float(sm[1]), wk))
    dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got, mx, total_in, weak = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    idx = sorted(i for g in got for i in g[0])
    assert idx == list(range(600))  # every tile exactly once, no data exchange needed
    loads = [g[1] for g in got]
    assert max(loads) / min(loads) < 1.1  # byte-balanced (greedy LPT)
    assert mx == 2.0 and total_in == sum(loads)
    assert weak[0] != weak[1]  # weak scaling: each rank samples its own batch


def test_lpt_shards_balance():
    import bench

    rng = np.random.default_rng(3)
    w = rng.integers(1, 1000, size=1000)
    for n in (1, 2, 4, 8):
        sh = bench.lpt_shards(list(w), n)
        assert sorted(i for s in sh for i in s) == list(range(1000))
        loads = [w[s].sum() for s in sh]
        assert max(loads) - min(loads) <= w.max()


@pytest.mark.parametrize("zooms", [None])
def test_batch_sampling_is_deterministic_and_covers_zooms(zooms):
    import bench

    lib = bench.tile_library()
    assert sorted(lib) == [2, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14]
    a = [k for k, _ in bench.sample_batch(lib, 1000, bench.SEED)]
    b = [k for k, _ in bench.sample_batch(lib, 1000, bench.SEED)]
    assert a == b
    assert len(set(a)) > 100
