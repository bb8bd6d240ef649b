"""Device-side plan timing on the bench batch (BASELINE config 5), in one process: wall-clock of
covt_device_plan_create per walk layout (covt_plan_options.device_walk: 0 = wave per tile with slots,
1 = walk twice, k >= 2 = k lanes per workgroup), interleaved rounds so box drift hits every setting
alike, plus the host plan for comparison.  Each setting's plan is checked equal to the host plan's
descriptors.  Usage: python tools/device_plan_ab.py [device_walk ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch

    lanes = [int(x) for x in sys.argv[1:]] or [0, 1]
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), 10000, bench.SEED)
    blob, offs, sizes = covt.pack_tiles([t for _, t in picks])
    t0 = time.perf_counter()
    hp = covt.Plan(blob, offs, sizes)
    t_host = time.perf_counter() - t0
    d_blob = torch.from_numpy(blob).cuda()
    d_off = torch.from_numpy(offs.astype(np.int64)).cuda()
    d_size = torch.from_numpy(sizes.astype(np.int64)).cuda()
    times = {k: [] for k in lanes}
    for rnd in range(6):
        for k in lanes:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dp = covt.DevicePlan(d_blob, d_off, d_size, options=covt.PlanOptions(device_walk=k))
            dt = time.perf_counter() - t0
            if rnd == 0:
                _, descs, _ = dp.host_copy()
                assert descs.tobytes() == hp.descs.tobytes(), k
            else:
                times[k].append(dt)
            dp.close()
    print("host plan (covt_plan_create): %.1f ms" % (t_host * 1e3))
    for k in lanes:
        print("device_walk=%-3d device plan median %.3f ms  min %.3f ms" %
              (k, np.median(times[k]) * 1e3, min(times[k]) * 1e3))


if __name__ == "__main__" and not os.environ.get("COVT_DPLAN_PROBE"):
    main()


def probe():
    """Where the walk's time goes: one tile alone vs 10k copies, for the smallest and the largest tile."""
    import torch

    covt = bench.load_covt()
    lib = [t for z in bench.tile_library().values() for _, t in z]
    lib.sort(key=len)
    one = os.environ.get("COVT_DPLAN_PROBE") == "2"  # counter runs: the smallest tile alone
    for name, tile in (("smallest", lib[0]),) + ((("largest", lib[-1]),) if not one else ()):
        for n in ((1,) if one else (1, 100, 10000)):
            blob, offs, sizes = covt.pack_tiles([tile] * n)
            d_blob = torch.from_numpy(blob).cuda()
            d_off = torch.from_numpy(offs.astype(np.int64)).cuda()
            d_size = torch.from_numpy(sizes.astype(np.int64)).cuda()
            ts = []
            for r in range(6):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dp = covt.DevicePlan(d_blob, d_off, d_size)
                ts.append(time.perf_counter() - t0)
                dp.close()
            print("%-8s tile (%d bytes) x %-5d device plan median %.3f ms" % (name, len(tile), n, np.median(ts[1:]) * 1e3))
            del d_blob


if __name__ == "__main__" and os.environ.get("COVT_DPLAN_PROBE"):
    probe()
