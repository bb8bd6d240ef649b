"""Split-stream plan layout (CPU): long Java-capped varint streams become chunks of COVT_SPLIT_SLOTS
descriptors (include/covt.h), contiguous byte ranges covering the stream, family counts and the
descriptor -> stream map consistent; the env knobs COVT_SPLIT_MIN / COVT_SPLIT_CHUNK are read at plan
creation."""
import os

import numpy as np
import pytest

from conftest import ROOT

DESC = np.dtype([("in_off", np.uint64), ("out_off", np.uint64), ("avail", np.int32), ("num_values", np.int32),
                 ("op", np.uint8), ("num_bits", np.uint8), ("flags", np.uint16), ("byte_length", np.int32)])


def _tile(name="5_16_20"):
    return open(os.path.join(ROOT, "tests", "golden", "tiles", "omt", name + ".covt"), "rb").read()


@pytest.mark.parametrize("chunk", [64, 1000, 4096])
def test_split_layout(covt, monkeypatch, chunk):
    monkeypatch.setenv("COVT_SPLIT_MIN", "256")
    monkeypatch.setenv("COVT_SPLIT_RATIO", "0")
    monkeypatch.setenv("COVT_SPLIT_CHUNK", str(chunk))
    monkeypatch.setenv("COVT_SPLIT_VALUES", "512")
    plan = covt.Plan.from_tiles([_tile(), _tile("14_8298_10748")])
    d = plan.descs.view(DESC)
    assert d.size == plan.num_descs == plan.family_counts.sum()
    fam0 = int(plan.family_counts[:covt.FAMILY_SPLIT].sum())
    sp = d[fam0:]
    assert plan.family_counts[covt.FAMILY_SPLIT_FPF] > 0
    assert sp.size % covt.SPLIT_SLOTS == 0 and sp.size > 0
    st = plan.streams
    split_streams = set()
    rle_ranges = {}
    for k in range(0, sp.size, covt.SPLIT_SLOTS):
        cd, rg = sp[k], sp[k + 1]
        fpf = bool(cd["flags"] & covt.DESC_SPLIT_FPF)
        rle = bool(cd["flags"] & covt.DESC_SPLIT_RLE)
        kind = cd["flags"] & (covt.DESC_SPLIT_FPF | covt.DESC_SPLIT_RLE)
        assert cd["flags"] == covt.DESC_SPLIT | kind and not (fpf and rle)
        c4, c5 = int(plan.family_counts[covt.FAMILY_SPLIT]), int(plan.family_counts[covt.FAMILY_SPLIT_FPF])
        assert (fpf, rle) == (c4 <= k < c4 + c5, k >= c4 + c5)  # varint, FastPFOR, then RLE chunks
        assert all(sp[k + q]["flags"] == covt.DESC_SPLIT_PAD | kind for q in range(1, covt.SPLIT_SLOTS))
        i = int(plan.desc_streams[fam0 + k])
        assert all(plan.desc_streams[fam0 + k + q] == i for q in range(covt.SPLIT_SLOTS))
        c = int(cd["avail"])
        if fpf:  # FastPFOR: value ranges of COVT_SPLIT_VALUES
            assert (int(rg["in_off"]), int(rg["out_off"])) == (c * 512, min((c + 1) * 512, int(st["num_values"][i])))
        elif rle:  # RLE: whole groups from the host walk (checked below)
            rle_ranges.setdefault(i, []).append((c, int(rg["in_off"]), int(rg["out_off"]), int(sp[k + 2]["in_off"]),
                                                 int(sp[k + 2]["out_off"]), int(sp[k + 3]["in_off"])))
        else:
            assert (int(rg["in_off"]), int(rg["out_off"])) == (c * chunk, min((c + 1) * chunk,
                                                                               int(st["byte_length"][i])))
        if c == 0:
            assert st["desc_index"][i] == fam0 + k  # the stream's result entry = its chunk 0
            split_streams.add(i)
        else:
            assert int(sp[k - covt.SPLIT_SLOTS]["avail"]) == c - 1 and plan.desc_streams[fam0 + k - 1] == i
    for i in split_streams:
        cost = int(st["byte_length"][i]) + int(st["out_elems"][i]) * int(st["elem_bytes"][i]) // 4
        assert cost > 256 and st["op"][i] in (
            covt.OP_VARINT_ZZ_DELTA_I32, covt.OP_VARINT_ZZ_DELTA_XY, covt.OP_VARINT_DELTA_MORTON, covt.OP_VARINT_I32,
            covt.OP_VARINT_U64, covt.OP_FPF_ZZ_DELTA_I32, covt.OP_FPF_ZZ_DELTA_XY, covt.OP_FPF_DELTA_MORTON,
            covt.OP_RLE_U64, covt.OP_RLE_I32, covt.OP_RLE_S64, covt.OP_BYTE_RLE_U8, covt.OP_BYTE_RLE_RAW)
    # RLE chunks tile the stream's bytes and values; the last one ends at the stream's consumed bytes
    assert rle_ranges
    for i, rows in rle_ranges.items():
        rows.sort()
        assert [r[0] for r in rows] == list(range(len(rows))) and len(rows) >= 2
        assert rows[0][1] == 0 and rows[0][3] == 0
        for a, b in zip(rows, rows[1:]):
            assert a[2] == b[1] and a[3] + a[4] == b[3]  # contiguous bytes, contiguous values
        assert rows[-1][3] + rows[-1][4] == int(st["num_values"][i]) and rows[-1][2] == rows[0][5]
        assert rows[0][5] <= int(st["byte_length"][i])
    # every stream has exactly one result entry, and non-split descriptors map 1:1
    assert len(set(st["desc_index"].tolist())) == plan.num_streams
    assert np.array_equal(plan.desc_streams[st["desc_index"]], np.arange(plan.num_streams))


def test_split_disabled_and_subset(covt, monkeypatch):
    monkeypatch.setenv("COVT_SPLIT_MIN", "-1")
    plan = covt.Plan.from_tiles([_tile()])
    assert plan.family_counts[covt.FAMILY_SPLIT] == 0 and plan.num_descs == plan.num_streams
    monkeypatch.setenv("COVT_SPLIT_MIN", "256")
    monkeypatch.setenv("COVT_SPLIT_RATIO", "0")
    monkeypatch.setenv("COVT_SPLIT_CHUNK", "512")
    plan = covt.Plan.from_tiles([_tile()])
    assert plan.family_counts[covt.FAMILY_SPLIT] > 0
    mask = plan.streams["stream_type"] == covt.VERTEX_BUFFER
    descs, counts, prim = plan.subset_descs(mask)
    assert counts.sum() == descs.size // 32 == prim.size
    assert (prim >= 0).sum() == mask.sum() and set(prim[prim >= 0].tolist()) == set(np.nonzero(mask)[0].tolist())
    assert counts[covt.FAMILY_SPLIT] % covt.SPLIT_SLOTS == 0


def test_split_threshold_relative_to_batch(covt, monkeypatch):
    """Default policy: a stream is split only above COVT_SPLIT_MIN and above the batch's stream bytes /
    COVT_SPLIT_RATIO -- one tile splits its long streams, a big batch of the same tiles splits none."""
    monkeypatch.delenv("COVT_SPLIT_MIN", raising=False)
    monkeypatch.delenv("COVT_SPLIT_RATIO", raising=False)
    one = covt.Plan.from_tiles([_tile()])
    assert one.family_counts[covt.FAMILY_SPLIT] > 0
    many = covt.Plan.from_tiles([_tile()] * 1000)
    assert many.family_counts[covt.FAMILY_SPLIT] == 0


@pytest.mark.parametrize("props", [False, True])
def test_plan_independent_of_host_threads(covt, monkeypatch, props):
    """The plan's host phases (walk, records, launch keys, descriptors, geometry columns) run on ranges
    of tiles / streams per thread with local offsets rebased afterwards: the plan must be byte-identical
    for any thread count (COVT_PLAN_THREADS), splits and properties included."""
    import glob

    names = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "*.covt")))[:40]
    tiles = [open(n, "rb").read() for n in names] * 25  # 1000 tiles: up to 16 walk ranges (>= 64 tiles each)
    flags = covt.PLAN_PROPERTIES if props else 0
    monkeypatch.setenv("COVT_SPLIT_MIN", "4096")
    plans = []
    for thr in ("1", "3", "16"):
        monkeypatch.setenv("COVT_PLAN_THREADS", thr)
        p = covt.Plan.from_tiles(tiles, flags=flags)
        plans.append(p)
    a = plans[0]
    assert a.family_counts[covt.FAMILY_SPLIT:].sum() > 0  # split descriptors exercised
    for b in plans[1:]:
        for f in ("descs", "desc_streams", "family_counts", "streams", "tile_status", "geom", "gdescs", "props",
                  "pdescs"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
        assert (a.in_bytes, a.out_bytes, a.vertices, a.output_bytes, a.assembly_bytes, a.property_bytes) == \
               (b.in_bytes, b.out_bytes, b.vertices, b.output_bytes, b.assembly_bytes, b.property_bytes)
