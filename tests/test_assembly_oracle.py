"""CPU: the geometry-assembly oracle (oracle_assemble_geometry, the restatement of
CovtParser.convertGeometryColumn, CovtParser.java:135-274) pinned against the reference's own data,
and the plan's geometry-column table (C-ABI, no GPU).

1. known answers on hand-built columns (every geometry type, empty parts/rings, closing vertices,
   the error statuses);
2. the oracle's nested offsets agree with the independent Python walk ``covt_geom.assemble`` on every
   geometry column of the 126 decodable fixtures;
3. MVT pin: assembled layers reproduce the digests of the reference's MVT originals
   (test/fixtures/omt/mvt via tests/golden/mvt_digests.json) for the same 780 layers as the stream
   cross-check in test_oracle.py;
4. the plan's geometry-column records and descriptors (covt_plan_geometry_columns / _descs).
"""
import json
import os

import numpy as np

import covt_asm as A
import covt_geom as G
from conftest import GOLDEN


def test_assembly_kats(oracle):
    # POLYGON (2 rings of 3, PLAIN: closed by the assembly), POINT, MULTILINESTRING (2 lines: 2, 3)
    vb = np.arange(2 * 12, dtype=np.int32)
    st, geo, part, ring, xy = oracle.assemble_geometry([2, 0, 4], [2], [2, 2, 3], [3, 3], None, vb, False)
    assert st == 0
    assert geo.tolist() == [0, 1, 2, 4] and part.tolist() == [0, 2, 3, 4, 5]
    assert ring.tolist() == [0, 4, 8, 9, 11, 14]
    assert xy[:, 0].tolist() == [0, 2, 4, 0, 6, 8, 10, 6, 12, 14, 16, 18, 20, 22]
    # ICE: vertexBuffer[2 * vertexOffsets[i]]; Gen C ICE rings carry their closing vertex
    vb = np.array([10, 11, 20, 21, 30, 31], dtype=np.int32)
    st, geo, part, ring, xy = oracle.assemble_geometry([2, 1], None, [1, 2], [4], [0, 1, 2, 0, 2, 2], vb, True)
    assert st == 0 and ring.tolist() == [0, 4, 6]
    assert xy.tolist() == [[10, 11], [20, 21], [30, 31], [10, 11], [30, 31], [30, 31]]
    # MULTIPOINT (Java rejects it; format truth: a geometryOffsets count of points), empty parts
    vb = np.arange(8, dtype=np.int32)
    st, geo, part, ring, xy = oracle.assemble_geometry([3, 4, 5, 3], [2, 0, 0, 1], [], [], None, vb, False)
    assert st == 0 and geo.tolist() == [0, 2, 2, 2, 3] and part.tolist() == [0, 1, 2, 3]
    assert xy.tolist() == [[0, 1], [2, 3], [4, 5]]
    # a polygon part with no rings, a ring with no vertices (no closing vertex to add)
    st, geo, part, ring, xy = oracle.assemble_geometry([2, 2], None, [0, 1], [0], None, vb, False)
    assert st == 0 and part.tolist() == [0, 0, 1] and ring.tolist() == [0, 0] and xy.size == 0
    # errors
    assert oracle.assemble_geometry([6], None, None, None, None, vb, False)[0] == oracle.ERR_HEADER
    assert oracle.assemble_geometry([4], [], [], [], None, vb, False)[0] == oracle.ERR_COUNT  # go over-read
    assert oracle.assemble_geometry([1], None, [9], None, None, vb, False)[0] == oracle.ERR_COUNT  # > vb
    assert oracle.assemble_geometry([1], None, [-1], None, None, vb, False)[0] == oracle.ERR_COUNT
    assert oracle.assemble_geometry([1], None, [2], None, [0, 4], vb, False)[0] == oracle.ERR_TRUNCATED


def _features_py(c):
    a = c["arr"].get
    return G.assemble(c["types"], a(5), a(6), a(7), a(8), a(9), c["closed"])


def test_oracle_assembly_matches_python_walk(oracle, decodable_tiles):
    n_cols = 0
    for key, t in decodable_tiles:
        for L, c in A.oracle_tile_columns(oracle, t).items():
            assert c["status"] == 0, (key, L)
            st, geo, part, ring, xy = c["asm"]
            assert st == 0, (key, L, st)
            assert geo[0] == 0 and np.all(np.diff(geo) >= 0) and np.all(np.diff(part) >= 0)
            assert np.all(np.diff(ring) >= 0) and ring[-1] == xy.shape[0]
            assert A.to_features(c["types"], geo, part, ring, xy) == _features_py(c), (key, L)
            n_cols += 1
    assert n_cols >= 700


def test_oracle_assembly_mvt_pin(oracle):
    dig = json.load(open(os.path.join(GOLDEN, "mvt_digests.json")))
    match = total = 0
    for name, layers in dig.items():
        t = open(os.path.join(GOLDEN, "tiles", "omt", name + ".covt"), "rb").read()
        cols = A.oracle_tile_columns(oracle, t)
        tile_ok = all(c["status"] == 0 for c in cols.values()) and bool(cols)
        for L, rec in layers.items():
            total += 1
            c = cols.get(int(L))
            g = None
            if tile_ok and c is not None and c["asm"] is not None and c["asm"][0] == 0 and 9 in c["arr"]:
                st, geo, part, ring, xy = c["asm"]
                g = G.layer_digest(A.to_features(c["types"], geo, part, ring, xy))
            m = g == rec["geom"]
            assert m == rec["oracle_geom_match"], (name, L, rec["name"])
            match += m
    assert total == 860 and match == 780


def test_plan_geometry_columns(covt, oracle, decodable_tiles):
    tiles = [t for _, t in decodable_tiles[:40]]
    plan = covt.Plan.from_tiles(tiles)
    g, st = plan.geom, plan.streams
    assert plan.num_geometry_columns == g.size > 0
    descs = np.frombuffer(plan.gdescs.tobytes(), dtype=np.uint8)
    assert sorted(g["desc_index"].tolist()) == list(range(g.size))
    ends = []
    for c in range(g.size):
        rec = g[c]
        cols = A.oracle_tile_columns(oracle, tiles[rec["tile"]])
        oc = cols[int(rec["layer"])]
        for k in range(6):
            si = int(rec["stream"][k])
            assert (si >= 0) == ((4 + k) in oc["arr"]), (c, k)
            if si >= 0:
                assert st["tile"][si] == rec["tile"] and st["layer"][si] == rec["layer"]
                assert st["stream_type"][si] == 4 + k
        n_src = oc["arr"][8].size if 8 in oc["arr"] else oc["arr"].get(9, np.zeros(0)).size // 2
        npo = oc["arr"][6].size if 6 in oc["arr"] else 0
        nro = oc["arr"][7].size if 7 in oc["arr"] else 0
        closed = bool(rec["flags"] & covt.GEOM_CLOSED_IN_STREAM)
        assert closed == oc["closed"]
        assert (rec["part_cap"], rec["ring_cap"], rec["coord_cap"]) == \
               (n_src + npo, n_src + npo + nro, n_src + (0 if closed else nro))
        assert rec["n_features"] == oc["arr"][4].size
        offs = rec["out_off"].tolist()
        assert all(o % 16 == 0 for o in offs) and offs == sorted(offs)
        ends.append((offs[0], offs[5] + 4 * int(rec["ring_cap"])))
        d = covt.GeomDesc.from_buffer_copy(descs[rec["desc_index"] * 160:(rec["desc_index"] + 1) * 160].tobytes())
        assert list(d.out_off) == offs and d.coord_cap == rec["coord_cap"]
        for k in range(6):
            si = int(rec["stream"][k])
            assert d.in_off[k] == (st["out_off"][si] if si >= 0 else -1)
            assert d.in_res[k] == (st["desc_index"][si] if si >= 0 else -1)
    ends.sort()
    assert all(a[1] <= b[0] for a, b in zip(ends, ends[1:])) and ends[-1][1] <= plan.assembly_bytes
