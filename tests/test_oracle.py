"""CPU: the oracle pinned against the reference's own data.

1. known-answer vectors of the reference's TS unit tests (tests/golden/kats.json);
2. fixture self-consistency: every Id/Geometry stream of the 126 decodable fixtures consumes exactly
   its byteLength and each tile walk ends at EOF (SURVEY.md §8(c) pin 1); the excluded tiles fail;
3. MVT cross-check: geometry and ids decoded by the oracle equal the reference's MVT originals for the
   committed pass list (the analogue of CovtParserTest.compareTiles, SURVEY.md §8(c) pin 2);
4. regression pin: oracle outputs hash to the committed digests (tests/golden/oracle_streams.json);
5. a second, pure-Python restatement (oracle/pyref.py) agrees with the C oracle;
6. encoder round trips (ORC writers, FastPFOR, varints) and Java's RLE re-encode advance.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import covt_geom as G
from conftest import GOLDEN, tile_key, tile_paths


def test_kats(oracle):
    k = json.load(open(os.path.join(GOLDEN, "kats.json")))
    for v in k["varint"]:
        st, vals, pos = oracle.decode_varint(bytes(v["bytes"]), v["pos"], 1)
        assert st == 0 and list(vals) == [v["value"]] and pos == v["end"]
    for v in k["varint_java_divergence"]:
        st, vals, pos = oracle.decode_varint(bytes(v["bytes"]), v["pos"], 1)
        assert st == 0 and list(vals) == [v["java_value"]] and pos == v["java_end"]
        st, vals, pos = oracle.decode_varint_u64(bytes(v["bytes"]), v["pos"], 1)
        assert st == 0 and list(vals) == [v["u64_value"]] and pos == v["u64_end"]
    for v in k["zigzag_varint"]:
        st, vals, pos = oracle.decode_zigzag_varint(bytes(v["bytes"]), v["pos"], 1)
        assert st == 0 and list(vals) == [v["value"]] and pos == v["end"]
    for v in k["rle"]:
        st, vals, pos, cons = oracle.decode_rle(bytes(v["bytes"]), v["n"], 0, v["signed"])
        assert st == 0 and list(vals) == v["values"] and cons == v["end"]


def test_fixture_self_consistency(oracle, golden_streams):
    n_dec = 0
    for p in tile_paths():
        key = tile_key(p)
        t = open(p, "rb").read()
        st, ss = oracle.walk_tile(t)
        rec = golden_streams["tiles"][key]
        assert st == rec["walk_status"], key
        ok = st == 0
        for s in ss:
            st2, arr, cons = oracle.decode_stream(t, s)
            ok &= st2 == 0 and cons == s.byte_length
        assert ok == rec["decodable"], key
        n_dec += ok
    assert n_dec == 126  # 90 OMT + 27 Bing + 9 Amazon
    undec = sorted(k for k, r in golden_streams["tiles"].items() if not r["decodable"])
    assert undec == ["amazon/6_33_21", "amazon/8_136_89", "omt/4_8_10"]  # SURVEY Q4 (varint labelled FastPFOR)


def test_vertex_offsets_in_range(oracle, decodable_tiles):
    for key, t in decodable_tiles:
        st, ss = oracle.walk_tile(t)
        by_layer = {}
        for s in ss:
            by_layer.setdefault(s.layer, {})[s.stream_type] = (s, oracle.decode_stream(t, s)[1])
        for L, d in by_layer.items():
            if 8 in d:
                nverts = d[9][1].size // 2
                assert d[8][1].min() >= 0 and d[8][1].max() < nverts, (key, L)


def test_mvt_cross_check(oracle):
    """Per-layer digests of the reference's MVT fixtures (computed by tests/golden/make_golden.py from
    test/fixtures/omt/mvt) against the oracle's decoded GeometryColumn / id column."""
    dig = json.load(open(os.path.join(GOLDEN, "mvt_digests.json")))
    geo = ids = total = 0
    for name, layers in dig.items():
        t = open(os.path.join(GOLDEN, "tiles", "omt", name + ".covt"), "rb").read()
        st, ss = oracle.walk_tile(t)
        dec = {}
        tile_ok = st == 0
        for s in ss:
            st2, arr, _ = oracle.decode_stream(t, s)
            tile_ok &= st2 == 0
            dec.setdefault(s.layer, {})[(s.column_kind, s.stream_type)] = (st2, arr, s)
        for L, rec in layers.items():
            total += 1
            d = dec.get(int(L), {})
            ok_all = tile_ok  # the generator scores a tile with any failing stream as unmatched
            g = None
            if ok_all and (1, 9) in d:
                def arr(k):
                    return d[(1, k)][1] if (1, k) in d else None
                try:
                    g = G.layer_digest(G.assemble(arr(4), arr(5), arr(6), arr(7), arr(8), arr(9),
                                                  d[(1, 9)][2].column_type in (3, 4)))
                except (StopIteration, IndexError):
                    g = None
            gm = g == rec["geom"]
            assert gm == rec["oracle_geom_match"], (name, L, rec["name"])
            geo += gm
            im = (0, 1) in d and ok_all and G.ids_digest(d[(0, 1)][1]) == rec["ids"]
            assert im == rec["oracle_ids_match"], (name, L)
            ids += im
    assert total == 860 and geo == 780 and ids == 852


def test_oracle_regression_digests(oracle, golden_streams):
    cols = golden_streams["columns"]
    i_f, i_j = cols.index("fmt_sha256"), cols.index("java_sha256")
    for p in tile_paths():
        key = tile_key(p)
        t = open(p, "rb").read()
        st, ss = oracle.walk_tile(t)
        rows = golden_streams["tiles"][key]["streams"]
        assert len(rows) == len(ss)
        for s, row in zip(ss, rows):
            for mode, col in ((0, i_f), (1, i_j)):
                st2, arr, cons = oracle.decode_stream(t, s, mode)
                d = hashlib.sha256(arr.tobytes()).hexdigest() if st2 == 0 else None
                assert d == row[col], (key, s.layer, s.stream_type, mode)


def test_5_16_20_full_arrays(oracle):
    t = open(os.path.join(GOLDEN, "tiles", "omt", "5_16_20.covt"), "rb").read()
    z = np.load(os.path.join(GOLDEN, "5_16_20.npz"))
    st, ss = oracle.walk_tile(t)
    assert st == 0 and len(ss) == len(z.files) == 41
    for i, s in enumerate(ss):
        k = "s%03d_L%d_k%d_t%d" % (i, s.layer, s.column_kind, s.stream_type)
        assert np.array_equal(oracle.decode_stream(t, s)[1], z[k])


# ---- second restatement ----------------------------------------------------------------------
PYREF_TILES = ("omt/5_16_20", "omt/2_2_2", "omt/12_2131_2733", "bing/4-9-5", "amazon/5_5_11")


@pytest.mark.parametrize("key", PYREF_TILES)
def test_pyref_agrees_on_fixtures(oracle, key):
    from oracle import pyref as R

    t = open(os.path.join(GOLDEN, "tiles", key + ".covt"), "rb").read()
    st, ss = oracle.walk_tile(t)
    for s in ss:
        o = s.offset
        end = o + s.byte_length
        if s.column_kind == 1 and s.stream_type == 4:
            ref, _ = R.decode_byte_rle(t[:end], s.num_values, o)
        elif s.encoding == 5 or (s.column_kind == 0 and s.encoding == 4):
            ref, _ = R.decode_rle(t[:end], s.num_values, o, False)
            if s.column_kind == 1:
                ref = [R.i32(x) for x in ref]
        elif s.encoding == 9:
            if s.stream_type == 9 and s.column_type == 4:
                ref, _ = R.decode_fastpfor_delta_morton_codes(t, s.num_values, s.byte_length, o, s.num_bits)
            elif s.stream_type == 9:
                n = s.num_values * (2 if s.column_type == 3 else 1)  # ICE VB holds 2n ints
                ref, _ = R.decode_fastpfor_delta_coordinates(t, n, s.byte_length, o)
            else:
                ref, _ = R.decode_fastpfor_zigzag_delta(t, s.num_values, s.byte_length, o)
        elif s.encoding == 4:
            if s.stream_type == 9 and s.column_type == 4:
                ref, _ = R.decode_delta_varint_morton_codes(t[:end], o, s.num_values, s.num_bits)
            elif s.stream_type == 9:
                n = s.num_values * (2 if s.column_type == 3 else 1)
                ref, _ = R.decode_zigzag_delta_varint_coordinates(t[:end], o, n)
            else:
                ref, _ = R.decode_zigzag_delta_varint(t[:end], o, s.num_values)
        elif s.encoding == 1:  # format-truth id varints: full LEB128
            pos, ref = o, []
            for _ in range(s.num_values):
                v, pos = R._vulong(t, pos)
                ref.append(R.i64(v))
        else:
            continue
        st2, arr, _ = oracle.decode_stream(t, s)
        assert st2 == 0
        assert [int(x) for x in arr] == [int(x) for x in ref], (key, s.layer, s.stream_type)


@pytest.mark.parametrize("seed", range(5))
def test_pyref_agrees_on_random_streams(oracle, seed):
    from oracle import pyref as R

    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, size=600).astype(np.uint8)
    b[rng.random(600) < 0.6] |= 0x80
    buf = bytes(b)
    for n in (1, 50, 150):
        st, vals, pos = oracle.decode_varint(buf, 3, n)
        try:
            ref, rpos = R.decode_varint(buf, 3, n)
            assert st == 0 and list(vals) == ref and pos == rpos
        except R.Truncated:
            assert st == oracle.ERR_TRUNCATED
    raw = rng.integers(0, 1 << int(rng.integers(1, 33)), size=int(rng.integers(0, 1500)), dtype=np.uint64)
    raw = raw.astype(np.uint32)
    enc = oracle.encode_fastpfor(raw)
    ref, cnt = R.fastpfor_uncompress(enc, 0, len(enc), raw.size)
    assert cnt == raw.size and ref == [int(x) for x in raw]
    for nb in (13, 14, 17):
        st, vals, _ = oracle.decode_fastpfor_delta_morton_codes(enc, raw.size, len(enc), 0, nb)
        ref, _ = R.decode_fastpfor_delta_morton_codes(enc, raw.size, len(enc), 0, nb)
        assert st == 0 and [int(x) for x in vals] == ref


def test_morton_java_semantics(oracle):
    from oracle import pyref as R

    rng = np.random.default_rng(7)
    for code in [0, 1, -1, 2**31 - 1, -2**31] + [int(x) for x in rng.integers(-2**31, 2**31, size=200)]:
        for nb in (0, 1, 2, 13, 14, 16, 17, 24, 31, 32, 33, 40):
            assert oracle.decode_morton(code, nb) == R.morton(code, nb), (code, nb)


# ---- encoders ---------------------------------------------------------------------------------
def test_rle_writer_round_trip_and_advance(oracle):
    rng = np.random.default_rng(11)
    for _ in range(30):
        n = int(rng.integers(0, 3000))
        vals = np.cumsum(rng.integers(-3, 4, size=n)).astype(np.int64)
        mask = rng.random(n) < 0.1
        vals[mask] = rng.integers(0, 1 << 40, size=int(mask.sum()))
        for signed in (False, True):
            enc = oracle.encode_rle(vals, signed)
            st, dec, pos, cons = oracle.decode_rle(enc + b"\x00\x00", n, 0, signed)
            assert st == 0 and np.array_equal(dec, vals) and pos == cons == len(enc)


def test_byte_rle_writer_round_trip(oracle):
    rng = np.random.default_rng(12)
    for _ in range(30):
        n = int(rng.integers(0, 2000))
        vals = np.repeat(rng.integers(0, 4, size=n), rng.integers(1, 6, size=n))[:n].astype(np.uint8)
        enc = oracle.encode_byte_rle(vals)
        st, dec, pos, cons = oracle.decode_byte_rle(enc, n, 0, len(enc))
        assert st == 0 and np.array_equal(dec, vals) and cons == len(enc)


def test_fixture_rle_streams_are_writer_canonical(oracle, decodable_tiles):
    """Java advances RLE streams by the length of their re-encoding (DecodingUtils.java:268-270,
    :308-310); on every fixture RLE stream that equals the bytes consumed."""
    for key, t in decodable_tiles[::4]:
        st, ss = oracle.walk_tile(t)
        for s in ss:
            if s.encoding == 5 and not (s.column_kind == 1 and s.stream_type == 4):
                st2, vals, pos, cons = oracle.decode_rle(t, s.num_values, s.offset, False)
                assert st2 == 0 and pos - s.offset == cons == s.byte_length, key


def test_fastpfor_encoder_page_and_tail(oracle):
    for n in (0, 1, 255, 256, 300, 65536, 65536 + 300):
        raw = (np.arange(n, dtype=np.uint64) * 2654435761 % (1 << 20)).astype(np.uint32)
        enc = oracle.encode_fastpfor(raw)
        st, dec, cnt = oracle.fastpfor_uncompress(enc, 0, len(enc), n)
        assert st == 0 and cnt == n and np.array_equal(dec, raw)
        if n:
            assert int.from_bytes(enc[:4], "big") == n - n % 256  # FastPFOR header = coded count


def test_oracle_asan_build_runs_fixtures(tmp_path):
    """Host sanitizer build (ASan+UBSan) of the oracle decodes the fixtures without reports."""
    import subprocess
    import sys

    from conftest import ROOT

    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle_covt_asan.so"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("no sanitizer toolchain: " + r.stderr[-200:])
    code = (
        "import ctypes, glob, sys\n"
        "sys.path.insert(0, %r)\n"
        "import oracle as O\n"
        "O._LIB_PATH = %r\n"
        "for p in sorted(glob.glob(%r))[:40]:\n"
        "    t = open(p, 'rb').read()\n"
        "    st, ss = O.walk_tile(t)\n"
        "    for s in ss: O.decode_stream(t, s)\n"
        "print('ok')\n" % (ROOT, os.path.join(ROOT, "oracle", "liboracle_covt_asan.so"),
                           os.path.join(GOLDEN, "tiles", "*", "*.covt")))
    env = dict(os.environ)
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    env["LD_PRELOAD"] = " ".join(x for x in (asan, ubsan) if os.path.isabs(x))
    env["ASAN_OPTIONS"] = "detect_leaks=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
