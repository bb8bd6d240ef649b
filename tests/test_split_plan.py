"""Split-stream plan layout (CPU): long Java-capped varint streams become chunks of COVT_SPLIT_SLOTS
descriptors (include/covt.h), contiguous byte ranges covering the stream, family counts and the
descriptor -> stream map consistent; the split rule follows the plan's covt_plan_options, and the
library ignores the environment (no COVT_* variable changes a plan)."""
import os

import numpy as np
import pytest

from conftest import ROOT

DESC = np.dtype([("in_off", np.uint64), ("out_off", np.uint64), ("avail", np.int32), ("num_values", np.int32),
                 ("op", np.uint8), ("num_bits", np.uint8), ("flags", np.uint16), ("byte_length", np.int32)])


def _tile(name="5_16_20"):
    return open(os.path.join(ROOT, "tests", "golden", "tiles", "omt", name + ".covt"), "rb").read()


@pytest.mark.parametrize("chunk", [64, 1000, 4096])
def test_split_layout(covt, chunk):
    opts = covt.PlanOptions(split_min=256, split_ratio=0, split_chunk=chunk, split_values=512)
    plan = covt.Plan.from_tiles([_tile(), _tile("14_8298_10748")], options=opts)
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


def test_split_disabled_and_subset(covt):
    plan = covt.Plan.from_tiles([_tile()], options=covt.PlanOptions(split_min=-1))
    assert plan.family_counts[covt.FAMILY_SPLIT] == 0 and plan.num_descs == plan.num_streams
    plan = covt.Plan.from_tiles([_tile()], options=covt.PlanOptions(split_min=256, split_ratio=0, split_chunk=512))
    assert plan.family_counts[covt.FAMILY_SPLIT] > 0
    mask = plan.streams["stream_type"] == covt.VERTEX_BUFFER
    descs, counts, prim = plan.subset_descs(mask)
    assert counts.sum() == descs.size // 32 == prim.size
    assert (prim >= 0).sum() == mask.sum() and set(prim[prim >= 0].tolist()) == set(np.nonzero(mask)[0].tolist())
    assert counts[covt.FAMILY_SPLIT] % covt.SPLIT_SLOTS == 0


def test_split_threshold_relative_to_batch(covt):
    """Default policy: a stream is split only above COVT_SPLIT_MIN and above the batch's stream bytes /
    COVT_SPLIT_RATIO -- one tile splits its long streams, a big batch of the same tiles splits none."""
    one = covt.Plan.from_tiles([_tile()])
    assert one.family_counts[covt.FAMILY_SPLIT] > 0
    many = covt.Plan.from_tiles([_tile()] * 1000)
    assert many.family_counts[covt.FAMILY_SPLIT] == 0


@pytest.mark.parametrize("props", [False, True])
def test_plan_independent_of_host_threads(covt, props):
    """The plan's host phases (walk, records, launch keys, descriptors, geometry columns) run on ranges
    of tiles / streams per thread with local offsets rebased afterwards: the plan must be byte-identical
    for any thread count (covt_plan_options.plan_threads), splits and properties included."""
    import glob

    names = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "*.covt")))[:40]
    tiles = [open(n, "rb").read() for n in names] * 25  # 1000 tiles: up to 16 walk ranges (>= 64 tiles each)
    flags = covt.PLAN_PROPERTIES if props else 0
    plans = []
    for thr in (1, 3, 16):
        p = covt.Plan.from_tiles(tiles, flags=flags, options=covt.PlanOptions(split_min=4096, split_max_streams=0,
                                                                                           plan_threads=thr))
        plans.append(p)
    a = plans[0]
    assert a.family_counts[covt.FAMILY_SPLIT:].sum() > 0  # split descriptors exercised
    for b in plans[1:]:
        for f in ("descs", "desc_streams", "family_counts", "streams", "tile_status", "geom", "gdescs", "props",
                  "pdescs"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f
        assert (a.in_bytes, a.out_bytes, a.vertices, a.output_bytes, a.assembly_bytes, a.property_bytes) == \
               (b.in_bytes, b.out_bytes, b.vertices, b.output_bytes, b.assembly_bytes, b.property_bytes)


def _fpf_states_py(b, n, unit, nch):
    """Independent restatement of the chunk start states (JavaFastPFOR FastPFOR.decodePage framing):
    per chunk starting inside a page at block j > 0, (page's first value, header offset, packed word,
    exception cursor per array 0..32); None where the chunk starts a page or lies past the blocks."""
    W = np.frombuffer(b[: len(b) // 4 * 4], dtype=">u4").astype(np.int64)
    L = int(W[0]) if W[0] < 2 ** 31 else -1
    out = [None] * nch
    if L < 0:
        return out
    L -= L % 256
    p, done = 1, 0
    while done < L:
        size = min(L - done, 65536)
        ie = p + int(W[p])
        bcw = (int(W[ie]) + 3) // 4
        bc = ie + 1
        ie = bc + bcw
        bm = int(W[ie]) & ~1
        ie += 1
        for k in range(2, 33):
            if bm >> (k - 1) & 1:
                sz = int(W[ie])
                ie += 1
                g = (sz + 31) // 32
                ie += g * k - ((g * 32 - sz) * k) // 32
        cont = b"".join(int(x).to_bytes(4, "little") for x in W[bc: bc + bcw])  # container byte order
        cur, pk, xc = 0, p + 1, [0] * 33
        for j in range(size // 256):
            v = done + 256 * j
            if j > 0 and v % unit == 0 and v // unit < nch:
                out[v // unit] = (done, cur, pk, tuple(xc))
            bb = int(np.int8(cont[cur])) if cur < len(cont) else 0
            ce = cont[cur + 1]
            if ce:
                idx = int(np.int8(cont[cur + 2])) - bb
                if 2 <= idx <= 32:
                    xc[idx] += ce
                cur += 3 + ce
            else:
                cur += 2
            pk += 8 * bb
        done += size
        p = ie
    return out


def test_fastpfor_chunk_states(covt):
    """The plan's host walk of the FastPFOR block headers before each split chunk (pads [2..7] of the
    chunk, int32 slots in every field but op / num_bits / flags) equals an independent Python walk."""
    plan = covt.Plan.from_tiles([_tile("14_8298_10748"), _tile()],
                                options=covt.PlanOptions(split_min=256, split_ratio=0, split_values=512))
    raw = plan.descs.reshape(-1, 32)
    d = plan.descs.view(DESC)
    f0 = int(plan.family_counts[:covt.FAMILY_SPLIT_FPF].sum())
    nf = int(plan.family_counts[covt.FAMILY_SPLIT_FPF])
    offs = [0, 4, 8, 12, 16, 20, 28]

    def slots(k):
        return [int(np.frombuffer(raw[k + 2 + i // 7][offs[i % 7]:offs[i % 7] + 4].tobytes(), dtype="<i4")[0])
                for i in range(37)]

    st = plan.streams
    checked = 0
    cache = {}
    for k in range(f0, f0 + nf, covt.SPLIT_SLOTS):
        i = int(plan.desc_streams[k])
        s = st[i]
        if i not in cache:
            b = plan.blob[int(s["in_off"]): int(s["in_off"]) + int(s["byte_length"])].tobytes()
            nch = -(-int(s["num_values"]) // 512)
            cache[i] = _fpf_states_py(b, int(s["num_values"]), 512, nch)
        c = int(d[k]["avail"])
        got = slots(k)
        want = cache[i][c]
        if want is None:
            assert got[0] == 0
            continue
        assert got[0] == 1
        assert (got[1], got[2], got[3], tuple(got[4:37])) == want
        checked += 1
    assert checked > 10


def _states_hook(covt, body, n, unit):
    import ctypes as C

    nch = -(-n // unit)
    out = np.zeros(max(nch, 1) * 42, dtype=np.int32)
    buf = np.frombuffer(body, dtype=np.uint8) if body else np.zeros(1, dtype=np.uint8)
    st = covt.lib().covt_debug_fpf_chunk_states(buf.ctypes.data_as(C.POINTER(C.c_uint8)), len(body), n,
                                                C.c_int64(unit), C.c_int64(nch),
                                                out.ctypes.data_as(C.POINTER(C.c_int32)))
    assert st == 0
    return out[: nch * 42].reshape(nch, 42)


def test_fastpfor_chunk_states_synthetic(covt, oracle):
    """The plan's FastPFOR chunk-state walk (covt_debug_fpf_chunk_states) on synthetic streams: equal to
    the Python restatement on well-formed single- and multi-page streams at several chunk sizes; on
    bit-flipped streams it never reads outside the stream and marks states present or absent (0 / 1)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_synthetic import _fpf_values

    rng = np.random.default_rng(7)
    checked = 0
    for n in (1000, 4096 + 77, 65536 + 256 + 13, 140000):
        enc = oracle.encode_fastpfor(_fpf_values(rng, n))
        for unit in (256, 1024, 2048):
            got = _states_hook(covt, enc, n, unit)
            want = _fpf_states_py(enc, n, unit, got.shape[0])
            for c, w in enumerate(want):
                if w is None:
                    assert got[c, 0] == 0, (n, unit, c)
                    continue
                assert got[c, 0] == 1 and (got[c, 1], got[c, 2], got[c, 3], tuple(got[c, 4:37])) == w, (n, unit, c)
                checked += 1
    assert checked > 100
    enc = oracle.encode_fastpfor(_fpf_values(rng, 70000))
    for _ in range(40):
        e = bytearray(enc)
        for _ in range(int(rng.integers(1, 4))):
            e[int(rng.integers(0, len(e)))] ^= 1 << int(rng.integers(0, 8))
        got = _states_hook(covt, bytes(e), 70000, 512)
        assert set(np.unique(got[:, 0]).tolist()) <= {0, 1}


def test_environment_ignored(covt, monkeypatch):
    """The library reads no COVT_* environment variable: a process that inherits the round-1/2 A/B knobs
    plans exactly as one that does not (covt_plan_options replaced them)."""
    base = covt.Plan.from_tiles([_tile()])
    for k, v in (("COVT_SPLIT_MIN", "-1"), ("COVT_SPLIT_RATIO", "1"), ("COVT_SPLIT_CHUNK", "64"),
                 ("COVT_SPLIT_VALUES", "256"), ("COVT_LANE_MAX_BYTES", "1000"), ("COVT_LANE_MIN_STREAMS", "0"),
                 ("COVT_PLAN_THREADS", "3"), ("COVT_FPF_SPLIT_WEIGHT", "8"), ("COVT_QUEUE_ORDER", "3012"),
                 ("COVT_SPLIT_QUEUES", "1"), ("COVT_HOST_PREFAULT", "0")):
        monkeypatch.setenv(k, v)
    p = covt.Plan.from_tiles([_tile()])
    for f in ("descs", "desc_streams", "family_counts", "streams"):
        assert np.array_equal(getattr(base, f), getattr(p, f)), f


def test_options_validated(covt):
    """Out-of-range options are COVT_ERR_INVALID_ARG (IllegalArgumentException), not silently clamped."""
    for kw in ({"split_chunk": 63}, {"split_values": 300}, {"split_values": 0}, {"fpf_split_weight": 0},
               {"split_ratio": -1}, {"plan_threads": -2}, {"prefault_threads": 0}, {"host_prefault": 2},
               {"device_walk": 257}, {"flags": 0x80}, {"split_max_streams": -1}, {"split_grow": 2}):
        with pytest.raises(covt.IllegalArgumentException):
            covt.Plan.from_tiles([_tile()], options=covt.PlanOptions(**kw))
    o = covt.PlanOptions()
    assert (o.split_min, o.split_ratio, o.split_chunk, o.split_values, o.lane_max_bytes, o.lane_min_streams,
            o.lane_max_values, o.split_max_streams, o.split_grow) == (8192, 3000, 2048, 2048, 0, 65536, 0, 65536, 1)
    for kw in ({"lane_max_bytes": 65536}, {"lane_max_values": 32768}, {"lane_max_values": -1}):
        with pytest.raises(covt.IllegalArgumentException):
            covt.Plan.from_tiles([_tile()], options=covt.PlanOptions(**kw))


def test_lane_limits_auto_by_plan_flags(covt):
    """covt_plan_options.lane_max_bytes / lane_max_values 0 = auto: RLE streams of <= 128 bytes and <= 256
    values join the lane family of an Id/Geometry plan, <= 512 / 512 in a plan with property columns
    (DESIGN.md §6.0); explicit limits override the auto ones."""
    tiles = [_tile(n) for n in ("5_16_20", "10_530_682", "14_8298_10748")]
    opts = covt.PlanOptions(lane_min_streams=0)  # no batch-size gate: every eligible stream is a lane stream

    def lane_streams(plan):  # the lane family's descriptors (num_values: the values the kernel decodes)
        d = plan.descs.view(DESC)
        return d[(d["flags"] & covt.DESC_LANE) != 0]

    for flags, max_b, max_v in ((0, 128, 256), (covt.PLAN_PROPERTIES, 512, 512)):
        ls = lane_streams(covt.Plan.from_tiles(tiles, flags=flags, options=opts))
        assert len(ls) > 0
        assert ls["avail"].max() <= max_b and ls["num_values"].max() <= max_v
        if flags:  # the property plan's longer lanes are used
            assert ls["avail"].max() > 128
    ls = lane_streams(covt.Plan.from_tiles(tiles, flags=covt.PLAN_PROPERTIES,
                                           options=covt.PlanOptions(lane_min_streams=0, lane_max_bytes=64,
                                                                    lane_max_values=100)))
    assert ls["avail"].max() <= 64 and ls["num_values"].max() <= 100


def _chunk_units(covt, plan):
    """(varint chunk bytes, FastPFOR chunk values) seen in a plan's split descriptors (None: no such chunk)"""
    d = plan.descs.view(DESC)
    fam0 = int(plan.family_counts[:covt.FAMILY_SPLIT].sum())
    sp = d[fam0:]
    units = {"varint": set(), "fpf": set()}
    for k in range(0, sp.size, covt.SPLIT_SLOTS):
        cd, rg = sp[k], sp[k + 1]
        if cd["flags"] & covt.DESC_SPLIT_RLE or int(cd["avail"]) != 0:
            continue
        kind = "fpf" if cd["flags"] & covt.DESC_SPLIT_FPF else "varint"
        nxt = k + covt.SPLIT_SLOTS
        if nxt < sp.size and int(sp[nxt]["avail"]) == 1:  # a first chunk with a successor: a full chunk
            units[kind].add(int(rg["out_off"]) - int(rg["in_off"]))
    return units


def test_split_grow_and_max_streams(covt):
    """covt_plan_options.split_grow: chunks double for plans of >= 4 MiB of cost and quadruple from 48 MiB
    (covt_internal.h split_grow_factor, the same in the device plan); split_max_streams: a plan of more streams
    splits nothing."""
    import glob

    names = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "*.covt")))
    tiles = [open(n, "rb").read() for n in names]
    base = dict(split_min=256, split_ratio=0, split_chunk=1000, split_values=512, split_max_streams=0)
    fixed = covt.Plan.from_tiles(tiles, options=covt.PlanOptions(split_grow=0, **base))
    st = fixed.streams
    cost = int((st["byte_length"].astype(np.int64) + st["out_elems"].astype(np.int64) * st["elem_bytes"] // 4).sum())
    grow = 4 if cost >= 48 << 20 else 2 if cost >= 4 << 20 else 1
    assert grow > 1, cost  # (the fixture library is a plan of several MiB of cost)
    grown = covt.Plan.from_tiles(tiles, options=covt.PlanOptions(split_grow=1, **base))
    uf, ug = _chunk_units(covt, fixed), _chunk_units(covt, grown)
    assert uf["varint"] == {1000} and ug["varint"] == {1000 * grow}
    assert uf["fpf"] == {512} and ug["fpf"] == {512 * grow}
    assert grown.num_descs < fixed.num_descs
    # split_max_streams: the bound is inclusive
    n = fixed.num_streams
    at = covt.Plan.from_tiles(tiles, options=covt.PlanOptions(**dict(base, split_max_streams=n)))
    over = covt.Plan.from_tiles(tiles, options=covt.PlanOptions(**dict(base, split_max_streams=n - 1)))
    assert at.family_counts[covt.FAMILY_SPLIT:].sum() > 0
    assert over.family_counts[covt.FAMILY_SPLIT:].sum() == 0 and over.num_descs == n
