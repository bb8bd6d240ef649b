"""The C MVT decoder behind the MVT-vs-COVT benchmark (oracle/mvt_decode.c) agrees
with the independent Python MVT reader of the parity tests (tests/covt_geom.mvt_layers) on every OMT
MVT fixture: feature and vertex totals per tile, and feature counts with tests/golden/mvt_digests.json.
The MVT originals live only in the reference checkout, so this runs where that is present (CPU)."""
import glob
import json
import os

import pytest

import covt_geom as G

MVT_DIR = "/root/reference/test/fixtures/omt/mvt"
HERE = os.path.dirname(os.path.abspath(__file__))


def _mvt_files():
    return sorted(glob.glob(os.path.join(MVT_DIR, "*.mvt")))


@pytest.mark.skipif(not _mvt_files(), reason="reference MVT fixtures not present")
def test_mvt_decoder_matches_python_reader(oracle):
    digests = json.load(open(os.path.join(HERE, "golden", "mvt_digests.json")))
    files = _mvt_files()
    assert len(files) >= 90
    for i, f in enumerate(files):
        data = open(f, "rb").read()
        st, nf, nv, _, _, _ = oracle.mvt_decode(data)
        assert st == 0, f
        key = os.path.basename(f)[:-4]
        if key in digests:
            assert nf == sum(int(v["n_features"]) for v in digests[key].values()), f
        if i % 9 == 0:  # the pure-Python reader is slow: every ninth tile
            layers = G.mvt_layers(data)
            assert nf == sum(len(L["features"]) for L in layers.values())
            assert nv == sum(len(p) for L in layers.values() for _, _, parts in L["features"] for p in parts)
        st2, nf2, nv2, _, nval, _ = oracle.mvt_decode(data, with_props=True)
        assert (st2, nf2, nv2) == (0, nf, nv) and nval > 0


def test_mvt_decoder_rejects_truncation(oracle):
    files = _mvt_files()
    data = open(files[0], "rb").read() if files else bytes([0x1a, 0x05, 0x12, 0x03, 0x22, 0x01, 0x09])
    assert oracle.mvt_decode(data[: len(data) // 2])[0] == 1 or len(data) < 8
    assert oracle.mvt_decode(b"\x1a\x7f")[0] == 1  # a layer longer than the tile
