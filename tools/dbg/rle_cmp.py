#!/usr/bin/env python3
"""Debug helper: decode one fixture tile's property plan with two libcovt builds (separate processes) and
print the first mismatching streams (op, index, values).  usage: rle_cmp.py TILE_KEY LIB_A LIB_B"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(key, out):
    sys.path.insert(0, ROOT)
    import torch

    import bench

    covt = bench.load_covt()
    lib = dict(kv for z in bench.tile_library().values() for kv in z)
    plan = covt.Plan.from_tiles([lib[key]], flags=covt.PLAN_PROPERTIES)
    batch = covt.DeviceBatch(plan, "cuda")
    batch.decode(torch.cuda.current_stream())
    torch.cuda.synchronize()
    o, r = batch.results()
    s = plan.streams
    np.savez(out, out=np.asarray(o), res=np.asarray(r), desc=s["desc_index"], off=s["out_off"], n=s["out_elems"],
             el=s["elem_bytes"], op=s["op"], nb=plan.descs.reshape(-1, 32)[:, 28:32].copy().view(np.int32).ravel())


def main():
    if sys.argv[1] == "--one":
        os.environ["COVT_LIB_VARIANT"] = sys.argv[4]
        one(sys.argv[2], sys.argv[3])
        return
    key, a, b = sys.argv[1:4]
    for lib, f in ((a, "/tmp/cmp_a.npz"), (b, "/tmp/cmp_b.npz")):
        subprocess.run([sys.executable, __file__, "--one", key, f, lib], check=True)
    A, B = np.load("/tmp/cmp_a.npz"), np.load("/tmp/cmp_b.npz")
    bad = 0
    for i in range(len(A["op"])):
        lo, n = int(A["off"][i]), int(A["n"][i]) * int(A["el"][i])
        x, y = A["out"][lo:lo + n], B["out"][lo:lo + n]
        ra, rb = A["res"][i], B["res"][i]
        if not np.array_equal(x, y) or tuple(ra) != tuple(rb):
            d = np.nonzero(x != y)[0]
            el = int(A["el"][i])
            j = int(d[0]) // el if len(d) else -1
            xa = x.view(np.int32) if el == 4 else x
            ya = y.view(np.int32) if el == 4 else y
            print("stream %d op %d bytes %d elems %d res %s vs %s first diff elem %d  a %s  b %s" % (
                i, A["op"][i], A["nb"][A["desc"][i]], A["n"][i], tuple(ra), tuple(rb), j,
                xa[max(j - 3, 0):j + 8].tolist(), ya[max(j - 3, 0):j + 8].tolist()))
            bad += 1
            if bad > 12:
                break
    print("mismatching streams:", bad)
    if os.environ.get("RLE_SHOW"):  # RLE_SHOW=stream:lo:hi -> B's int32 outputs, decoded as debug words
        i, lo_, hi_ = (int(v) for v in os.environ["RLE_SHOW"].split(":"))
        lo = int(A["off"][i])
        y = B["out"][lo:lo + int(A["n"][i]) * 4].view(np.int32)
        for r in range(lo_, hi_):
            w = int(y[r])
            # (a debug build writing (group << 20 | run << 19 | group start << 4 | lane % 16) per output)
            print(r, "g", w >> 20, "run", (w >> 19) & 1, "gs", (w >> 4) & 0x7fff, "lane%16", w & 15)


def dump(key, i, f):
    """write stream i's input bytes of tile `key` (property plan) to f"""
    sys.path.insert(0, ROOT)
    import bench

    covt = bench.load_covt()
    lib = dict(kv for z in bench.tile_library().values() for kv in z)
    plan = covt.Plan.from_tiles([lib[key]], flags=covt.PLAN_PROPERTIES)
    s = plan.streams[i]
    open(f, "wb").write(np.asarray(plan.blob).view(np.uint8)[int(s["in_off"]):int(s["in_off"]) + int(s["byte_length"])].tobytes())


if __name__ == "__main__":
    main()
