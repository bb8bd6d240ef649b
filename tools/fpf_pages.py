#!/usr/bin/env python3
"""FastPFOR page statistics of the bench batch on the CPU (no GPU): how many blocks carry exceptions and how many
sit on pages whose metadata (byte container, directory, exception arrays) exceeds the decode's 1 KiB meta window
(`xin` false in run_fastpfor_stream), plus the metadata sizes of those pages.
usage: fpf_pages.py [tiles]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    covt = bench.load_covt()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    plan = covt.Plan.from_tiles([t for _, t in bench.sample_batch(bench.tile_library(), n, bench.SEED)])
    blob, s = plan.blob, plan.streams
    rows = []
    for i in np.nonzero(np.isin(s["op"], [10, 11, 12]))[0]:
        off, nw = int(s["in_off"][i]), int(s["byte_length"][i]) // 4

        def W(k):
            return int.from_bytes(blob[off + 4 * k: off + 4 * k + 4], "big") if k < nw else 0
        if nw == 0:
            continue
        L = W(0) - W(0) % 256
        p, done = 1, 0
        while done < L:
            size = min(L - done, 65536)
            ie = p + W(p)
            mw0 = ie - (((off + 4 * ie) & 15) >> 2)  # the meta window's first word (16-byte grid)
            bytesize = W(ie)
            ie += 1
            bc = ie
            ie += (bytesize + 3) // 4
            arr0 = ie
            bm = W(ie) & ~1
            ie += 1
            for k in range(2, 33):
                if bm & (1 << (k - 1)):
                    sz = W(ie)
                    ie += 1
                    g = (sz + 31) // 32
                    ie += g * k - ((g * 32 - sz) * k) // 32
            cont = bytes(blob[off + 4 * bc: off + 4 * bc + 4 * ((bytesize + 3) // 4)])
            cb = b"".join(cont[q:q + 4][::-1] for q in range(0, len(cont), 4))  # LE bytes of the BE words
            cur, exc = 0, 0
            for _ in range(size // 256):
                ce = cb[cur + 1]
                exc += ce > 0
                cur += 3 + ce if ce else 2
            rows.append((size // 256, exc, ie - mw0 <= 255, bytesize, 4 * (ie - arr0)))
            done += size
            p = ie
    r = np.array(rows, dtype=np.int64)
    xin = r[:, 2] == 1
    print("pages %d (%d in the meta window), blocks %d, blocks with exceptions %.3f, blocks on pages past the "
          "meta window %.3f" % (len(r), xin.sum(), r[:, 0].sum(), r[:, 1].sum() / r[:, 0].sum(),
                                r[~xin, 0].sum() / r[:, 0].sum()))
    for q in (50, 75, 90):
        print("  pages past the window, p%d: container %d B, exception arrays %d B" % (
            q, np.percentile(r[~xin, 3], q), np.percentile(r[~xin, 4], q)))


if __name__ == "__main__":
    main()
