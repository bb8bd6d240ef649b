#!/usr/bin/env python3
"""covt_plan_decode_host[_shards] with PINNED caller buffers (tile bytes and outputs in page-locked host
memory) on the config-5 batch: 1 shard vs K shards on the same GPU, each shard its own stream and host
thread, so one shard's H2D, another's decode and a third's D2H overlap on the full-duplex link."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    blob, offs, sizes = covt.pack_tiles([t for _, t in picks])
    pin_in = torch.from_numpy(blob).pin_memory().numpy()
    plan = covt.Plan(pin_in, offs, sizes)
    assert plan.blob.ctypes.data == pin_in.ctypes.data  # the plan reads the pinned bytes in place
    out = torch.empty(max(plan.output_bytes, 1), dtype=torch.uint8).pin_memory().numpy()
    res = np.zeros((max(plan.num_streams, 1), 2), dtype=np.int32)
    ref = None
    for k in [int(a) for a in (sys.argv[1:] or ["1", "2", "4", "8"])]:
        devs = [torch.cuda.current_device()] * k
        plan.decode_host(out=out, res=res, shard_devices=devs)  # warm: device buffers per shard
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            plan.decode_host(out=out, res=res, shard_devices=devs)
            ts.append((time.perf_counter() - t) * 1e3)
        if ref is None:
            ref = (out[:plan.output_bytes].copy(), res.copy())
        ok = np.array_equal(res, ref[1]) and np.array_equal(out[:plan.output_bytes], ref[0])
        gbs = plan.in_bytes / (np.median(ts) * 1e-3) / 1e9
        print("pinned, %d shard(s) on one GPU: %.1f ms median (%.1f GB/s raw), identical to 1 shard: %s"
              % (k, np.median(ts), gbs, ok), flush=True)
        plan.release_device()


if __name__ == "__main__":
    main()
