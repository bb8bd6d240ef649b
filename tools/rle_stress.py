#!/usr/bin/env python3
"""RLE-family stress sweep (GPU): many seeds of the adversarial Gen D topology streams of
tests/test_gpu_rle_adversarial.py plus random property columns, checked stream by stream against
the oracle in both Id modes.  usage: rle_stress.py [seeds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402


def main():
    import torch  # noqa: F401  (HIP runtime first, then libcovt)

    import bench
    import oracle
    import test_gpu_rle_adversarial as A
    from test_gpu_gend import _check_streams, _check_props, _synthetic_layer
    from oracle import gend as W

    covt = bench.load_covt()
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    tot = 0
    for seed in range(seeds):
        rng = np.random.default_rng(1000 + seed)
        tiles = [A._tile(rng, bad_types=(i % 4 == 3)) for i in range(12)]
        tiles += [W.tile([_synthetic_layer(rng, L) for L in range(int(rng.integers(1, 4)))]) for _ in range(8)]
        for mode in (0, 1):
            plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GEND, mode, covt.PLAN_PROPERTIES)
            assert (plan.tile_status == 0).all()
            out, res = plan.decode_host()
            tot += _check_streams(covt, oracle, plan, out, res, tiles, mode)
            buf, pres = plan.properties_host()
            _check_props(covt, oracle, plan, buf, pres, tiles, mode)
        print("seed %d ok (%d streams checked so far)" % (seed, tot), flush=True)


if __name__ == "__main__":
    main()
