#!/usr/bin/env python3
"""How much of the property plan's int RLE work sits in windows of one-byte literal groups only?

ORC RLE v1 (RunLengthIntegerReader): a header byte c < 0x80 starts a run of c + 3 values (a delta byte,
a base varint); c >= 0x80 starts 256 - c literal varints.  run_rle_int (covt_decode.hip) decodes a stream
1 KiB window at a time, the groups complete inside the window.  This walks the RLE-family RLE_I32 /
RLE_U64 / RLE_S64 streams of the config-5 property plan on the host, cuts them into windows the way the
kernel does (window start = the first unfinished group's header, 16-byte aligned in the blob), and counts
the windows and values whose groups are all literal groups of one-byte varints.
usage: rle_windows.py [n_tiles]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

KWIN = 1024


def groups(b, n):
    """(start, end, values, kind) of the stream's groups; kind 0 run, 1 literal one-byte, 2 literal wider"""
    out, p, v = [], 0, 0
    while v < n and p < len(b):
        c = b[p]
        if c < 0x80:
            q = p + 2
            while q < len(b) and b[q] & 0x80:
                q += 1
            out.append((p, q + 1, c + 3, 0))
            v += c + 3
            p = q + 1
        else:
            cnt = 256 - c
            q, wide = p + 1, False
            for _ in range(cnt):
                s = q
                while q < len(b) and b[q] & 0x80:
                    q += 1
                wide |= q != s
                q += 1
            out.append((p, q, cnt, 2 if wide else 1))
            v += cnt
            p = q
    return out


def main():
    n_tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    covt = bench.load_covt()
    picks = bench.sample_batch(bench.tile_library(), n_tiles, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks], flags=covt.PLAN_PROPERTIES)
    d = plan.descs.reshape(-1, 32)
    in_off = d[:, 0:8].copy().view(np.uint64).ravel()
    nv = d[:, 20:24].copy().view(np.int32).ravel()
    op = d[:, 24]
    flags = d[:, 26:28].copy().view(np.uint16).ravel()
    blen = d[:, 28:32].copy().view(np.int32).ravel()
    sel = np.nonzero(np.isin(op, [2, 3, 4]) & ((flags & 0x1f) == 0))[0]
    blob = plan.blob
    tot_w = tot_v = one_w = one_v = 0
    kinds_v = np.zeros(3, np.int64)
    for i in sel:
        a = int(in_off[i])
        b = blob[a:a + int(blen[i])].tolist()
        gs = groups(b, int(nv[i]))
        for g in gs:
            kinds_v[g[3]] += g[2]
        k = 0
        while k < len(gs):
            woff = ((a + gs[k][0]) & ~15) - a
            j = k
            while j < len(gs) and gs[j][1] <= woff + KWIN:
                j += 1
            if j == k:  # a group longer than a window: the multi-window literal path
                j = k + 1
            vals = sum(g[2] for g in gs[k:j])
            tot_w += 1
            tot_v += vals
            if all(g[3] == 1 for g in gs[k:j]):
                one_w += 1
                one_v += vals
            k = j
    print("RLE-family int RLE streams: %d, windows %d, values %d" % (len(sel), tot_w, tot_v))
    print("values by group kind: runs %d, one-byte literals %d, wider literals %d" % tuple(kinds_v))
    print("windows of one-byte literal groups only: %d (%.1f %%), their values %d (%.1f %%)" %
          (one_w, 100.0 * one_w / max(tot_w, 1), one_v, 100.0 * one_v / max(tot_v, 1)))


if __name__ == "__main__":
    main()
