"""GPU parity of the property-column path (decode of present / data / length streams + covt_props.hip
materialization) against the CPU oracle (oracle/covt_oracle_props.c, restating
CovtParser.decodePropertyColumn CovtParser.java:276-354), bit-exact through the C-ABI.  The oracle itself
is pinned by the reference's MVT originals (tests/test_props_oracle.py)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, tile_key, tile_paths

pytestmark = pytest.mark.gpu


def _tile(name):
    return open(os.path.join(GOLDEN, "tiles", "omt", name + ".covt"), "rb").read()


def _oracle_props(oracle, tile, mode):
    st, props = oracle.walk_properties(tile)
    assert st == 0
    return props, [oracle.decode_property(tile, p, mode) for p in props]


def _check_column(covt, plan, buf, pres, c, o, where):
    ost, oval, ovals, odoff, odby, onv = o
    st = int(pres["status"][c])
    assert st == ost, (where, st, ost)
    if st:
        return
    col = plan.property_column(buf, pres, c)
    assert col.n_valid == onv, where
    assert np.array_equal(col.validity, oval), where
    assert np.array_equal(col.values.view(np.uint8), np.asarray(ovals).view(np.uint8)), where
    if col.type == covt.PROP_STRING:
        assert np.array_equal(col.dict_offsets, odoff), where
        assert np.array_equal(col.dict_bytes, odby), where


@pytest.mark.parametrize("id_mode", [0, 1], ids=["format", "java"])
def test_fixture_property_columns_bitexact(covt, oracle, gpu_available, id_mode):
    paths = tile_paths()
    tiles = [open(p, "rb").read() for p in paths]
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GENC, id_mode, covt.PLAN_PROPERTIES)
    buf, pres = plan.properties_host()
    P = plan.props
    n_ok = 0
    cache = {}
    for c in range(plan.num_property_columns):
        t = int(P["tile"][c])
        if t not in cache:
            cache[t] = _oracle_props(oracle, tiles[t], id_mode)
        props, outs = cache[t]
        k = int(np.sum(P["tile"][:c] == t))  # tile-order index within the tile
        assert (props[k].layer, props[k].column, props[k].lang) == (P["layer"][c], P["column"][c], P["lang"][c])
        assert plan.property_name(c) == oracle.prop_name(tiles[t], props[k])
        _check_column(covt, plan, buf, pres, c, outs[k], (tile_key(paths[t]), c))
        n_ok += int(pres["status"][c]) == 0
    assert plan.num_property_columns == sum(len(cache[t][0]) for t in cache) >= 13000
    assert n_ok == plan.num_property_columns


def test_device_batch_properties_match_host(covt, gpu_available):
    import torch

    tiles = [open(p, "rb").read() for p in tile_paths(("omt", "bing"))[:40]]
    plan = covt.Plan.from_tiles(tiles, flags=covt.PLAN_PROPERTIES)
    hb, hr = plan.properties_host()
    b = covt.DeviceBatch(plan, "cuda:0")
    b.decode()
    b.materialize_properties()
    torch.cuda.synchronize()
    db, dr = b.property_results()
    assert np.array_equal(hr, dr)
    for c in range(plan.num_property_columns):
        x, y = plan.property_column(hb, hr, c), plan.property_column(db, dr, c)
        assert np.array_equal(x.validity, y.validity) and np.array_equal(x.values, y.values), c


def test_decode_covt_properties_equal_java_view(covt, oracle, gpu_available):
    """CovtParser mirror: List<Optional> per property column equals the oracle's Java-level view."""
    t = _tile("5_16_20")
    layers = covt.CovtParser.decode_covt(t, properties=True)
    st, props = oracle.walk_properties(t)
    seen = 0
    for p in props:
        lc = [x for x in layers if x.layer == p.layer][0]
        col = lc.properties[oracle.prop_name(t, p)]
        assert col.to_list() == oracle.property_values(t, p)[1]
        seen += 1
    assert seen == len(props) > 100


def test_batch_properties_digests(covt, oracle, gpu_available):
    """A 2,000-tile config-5 style batch: every property column equals the oracle's column of its source
    tile (goldens reused per source tile)."""
    import bench
    import torch

    picks = bench.sample_batch(bench.tile_library(), 2000, bench.SEED)
    plan = covt.Plan.from_tiles([t for _, t in picks], flags=covt.PLAN_PROPERTIES)
    b = covt.DeviceBatch(plan, "cuda:0")
    b.decode()
    b.materialize_properties()
    torch.cuda.synchronize()
    buf, pres = b.property_results()
    assert (pres["status"] == 0).all()
    ref = {}
    P = plan.props
    first = {}
    for c in range(plan.num_property_columns):
        first.setdefault(int(P["tile"][c]), c)
    for c in range(plan.num_property_columns):
        key, tile = picks[int(P["tile"][c])]
        if key not in ref:
            props, outs = _oracle_props(oracle, tile, 0)
            ref[key] = [hashlib.sha256(np.asarray(o[1]).tobytes() + np.asarray(o[2]).view(np.uint8).tobytes())
                        .hexdigest() for o in outs]
        col = plan.property_column(buf, pres, c)
        d = hashlib.sha256(col.validity.tobytes() + col.values.view(np.uint8).tobytes()).hexdigest()
        assert d == ref[key][c - first[int(P["tile"][c])]], (key, c)


@pytest.mark.parametrize("n_tiles", [60, 20], ids=["wave_per_column", "cooperative"])
def test_corrupted_property_streams_status_parity(covt, oracle, gpu_available, n_tiles):
    """Bit flips / truncations inside property streams: the GPU reports exactly the oracle's status and,
    when that is OK, exactly its column.  20 tiles (2,900 columns) take the small-batch path, where the
    tile's 35k-feature columns are materialized by whole workgroups (props_coop_kernel)."""
    rng = np.random.default_rng(11 if n_tiles == 60 else 12)
    base = _tile("5_16_20")
    st, props = oracle.walk_properties(base)
    tiles = []
    for i in range(n_tiles):
        p = props[int(rng.integers(0, len(props)))]
        role = int(rng.choice([r for r in range(4) if p.s_off[r] >= 0 and p.s_bl[r] > 0]))
        t = bytearray(base)
        o = p.s_off[role] + int(rng.integers(0, p.s_bl[role]))
        t[o] = int(rng.integers(0, 256))
        tiles.append(bytes(t))
    plan = covt.Plan.from_tiles(tiles, flags=covt.PLAN_PROPERTIES)
    buf, pres = plan.properties_host()
    P = plan.props
    n_err = 0
    for t in range(len(tiles)):
        props_t, outs = _oracle_props(oracle, tiles[t], 0)
        idx = np.nonzero(P["tile"] == t)[0]
        assert len(idx) == len(props_t)
        for c, o in zip(idx, outs):
            _check_column(covt, plan, buf, pres, int(c), o, (t, int(c)))
            n_err += o[0] != 0
    assert n_err >= (5 if n_tiles == 60 else 1)
    assert (plan.num_property_columns <= 4096) == (n_tiles == 20)
