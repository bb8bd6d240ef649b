#!/usr/bin/env python3
"""BASELINE configs 2-4: one decode launch per step submitted as stream operations (memset, fork
events, the family / chunk kernels on four queues, join) vs replayed from a captured HIP graph; HIP
events on the launch stream, mean of 200 after 20 warm-ups, outputs and statuses compared."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    lib = bench.tile_library()
    s = torch.cuda.current_stream()
    for name in bench.CONFIG_LEGS:
        picks = bench.config_tiles(lib, name)
        plan = covt.Plan.from_tiles([t for _, t in picks])
        batch = covt.DeviceBatch(plan, "cuda")
        sub = batch.subset(bench.config_mask(plan, name))
        res = {}
        for mode in ("stream", "graph", "stream", "graph"):
            fn = sub.decode if mode == "stream" else sub.decode_graph
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
            for a, b in ev:
                a.record(s)
                fn()
                b.record(s)
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(float(np.mean([a.elapsed_time(b) for a, b in ev])))
            out, r, _ = sub.results()
            res.setdefault(mode + "_out", []).append((out.copy(), r.copy()))
        same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
                   for a, b in zip(res["stream_out"], res["graph_out"]))
        print("%s: stream ops %.4f / %.4f ms, graph replay %.4f / %.4f ms, identical results: %s, statuses ok: %s"
              % (name, *res["stream"], *res["graph"], same, bool((res["graph_out"][0][1][:, 0] == 0).all())),
              flush=True)


if __name__ == "__main__":
    main()
