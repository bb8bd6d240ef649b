#!/usr/bin/env python3
"""Stream launch vs captured-graph replay of the bench's decode step: per-step HIP events and wall
time over 20 steps each, alternating, outputs compared.  usage: graph_ab.py [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    import torch

    import bench

    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks])
    batch = covt.DeviceBatch(plan, "cuda")
    stream = torch.cuda.current_stream()
    for _ in range(3):
        batch.decode(stream)
    torch.cuda.synchronize()
    ref = batch.d_out.clone()
    batch.d_out.zero_()
    batch.decode_graph()
    torch.cuda.synchronize()
    assert torch.equal(ref, batch.d_out), "graph replay output differs"
    _, res = batch.results()
    assert (res[:, 0] == 0).all()

    def run(fn, steps=20):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s, e in ev:
            s.record(stream)
            fn()
            e.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / steps
        return float(np.mean([s.elapsed_time(e) for s, e in ev])), wall

    for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        a = run(lambda: batch.decode(stream))
        b = run(batch.decode_graph)
        print("round %d: streams %.3f ms (wall %.3f)  graph %.3f ms (wall %.3f)" % (r, a[0], a[1], b[0], b[1]), flush=True)


if __name__ == "__main__":
    main()
