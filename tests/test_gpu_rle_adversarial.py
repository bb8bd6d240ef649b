"""RLE family on adversarial count streams, bit-exact against the oracle (statuses included).

Geometry topology streams (GeometryOffsets / PartOffsets / RingOffsets: ORC RLE v1 decoded to int32,
COVT_OP_RLE_I32; DecodingUtils.decodeRle then the (int) cast of CovtParser.java:135-274) are written
by the restated Gen D writer (oracle/gend.py) from synthetic int64 sequences chosen to stress the wave
decoder rather than to be valid geometry: runs of 3-130 with every delta, literal groups of 1-128
values from 1-byte to 10-byte varints (values past 2^31 truncate in the int cast), long arithmetic
sequences split into chains of runs with one delta across 2^32, group boundaries
at every window offset, and long alternations of short runs and short literals (~200 groups/KiB,
the walk-bound shape of dictionary-index streams).  GeometryType bytes include out-of-range values,
which the reference rejects (GeometryType.values()[b]).  Streams are decoded in both Id modes."""
import numpy as np
import pytest

from oracle import gend as W
from test_gpu_gend import _check_streams

pytestmark = pytest.mark.gpu


def _counts(rng, n):
    out = []
    while len(out) < n:
        k = int(rng.integers(0, 7))
        if k == 0:  # arithmetic run, any delta the header can carry
            base = int(rng.integers(0, 1 << int(rng.integers(1, 62))))
            d = int(rng.integers(-128, 128))
            m = int(rng.integers(3, 131))
            if base + d * m < 0:
                d = abs(d)
            out += [base + d * i for i in range(m)]
        elif k == 1:  # literals of mixed magnitude (1..10-byte varints)
            m = int(rng.integers(1, 129))
            bits = rng.integers(1, 63, size=m)
            out += [int(rng.integers(0, 1 << int(b))) for b in bits]
        elif k == 2:  # short runs and short literals alternating
            for _ in range(int(rng.integers(1, 40))):
                v = int(rng.integers(0, 300))
                out += [v] * int(rng.integers(3, 6)) + [int(x) for x in rng.integers(0, 1 << 20, size=int(rng.integers(1, 4)))]
        elif k == 3:  # values just past the int32 range
            out += [int(x) for x in rng.integers((1 << 31) - 3, (1 << 33), size=int(rng.integers(1, 40)))]
        elif k == 4:  # a long literal stretch (crosses 1 KiB windows)
            out += [int(x) for x in rng.integers(1 << 40, 1 << 56, size=int(rng.integers(100, 600)))]
        elif k == 5:  # constant run
            out += [int(rng.integers(0, 1 << 16))] * int(rng.integers(3, 300))
        else:  # a long arithmetic sequence (chains of runs with one delta, merged by the decoder) across 2^32
            d = int(rng.integers(-128, 128))
            m = int(rng.integers(131, 3000))
            base = (1 << 32) - int(rng.integers(0, 200)) * max(abs(d), 1)
            if base + d * m < 0:
                d = abs(d)
            out += [base + d * i for i in range(m)]
    return np.array(out[:n], dtype=np.int64)


def _tile(rng, bad_types):
    layers = []
    for L in range(int(rng.integers(1, 4))):
        n = int(rng.choice([1, 3, 64, 257, 1000, 5000]))
        types = rng.integers(0, 6, size=n).astype(np.uint8)
        if n > 8:
            types[: n // 3] = types[0]  # byte runs
        if bad_types and n > 1:
            types[int(rng.integers(0, n))] = 6 + int(rng.integers(0, 200))
        go = _counts(rng, int(rng.integers(1, 20000)))
        po = _counts(rng, int(rng.integers(1, 6000)))
        ro = _counts(rng, int(rng.integers(1, 3000)))
        xy = rng.integers(0, 4096, size=(64, 2))
        g = W.geometry_column(types, geometry_offsets=go, part_offsets=po, ring_offsets=ro, vertices=xy,
                              column_type=W.CT_PLAIN, allow_fpf_topology=False, allow_fpf_vertex=False)
        layers.append(W.layer("L%d" % L, 4096, n, [W.id_column(np.arange(n, dtype=np.uint64)), g], layer_id=L))
    return W.tile(layers)


@pytest.mark.parametrize("mode", [0, 1], ids=["format", "java"])
def test_adversarial_rle_streams_bitexact(covt, oracle, gpu_available, mode):
    rng = np.random.default_rng(7 + mode)
    tiles = [_tile(rng, bad_types=(i % 5 == 4)) for i in range(24)]
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GEND, mode)
    assert (plan.tile_status == 0).all()
    ops = set(plan.streams["op"].tolist())
    assert {covt.OP_RLE_I32, covt.OP_BYTE_RLE_U8} <= ops
    out, res = plan.decode_host()
    assert _check_streams(covt, oracle, plan, out, res, tiles, mode) >= 100
    # some GeometryType streams must have been rejected, the rest decoded
    gt = plan.streams["op"] == covt.OP_BYTE_RLE_U8
    assert (res[gt, 0] != 0).any() and (res[gt, 0] == 0).any()
    # both launch shapes of the device path (pin the fused and the forked kernels)
    import torch

    db = covt.DeviceBatch(plan, "cuda")
    for launch in (covt.LAUNCH_FUSED, covt.LAUNCH_FORKED):
        db.d_out.fill_(0x5A)
        db.decode(launch=launch)
        torch.cuda.synchronize()
        dout, dres = db.results()
        assert np.array_equal(dres, res), launch
        assert _check_streams(covt, oracle, plan, dout, dres, tiles, mode) >= 100
