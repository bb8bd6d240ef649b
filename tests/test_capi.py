"""CPU: the C-ABI library loads, exports every entry point include/covt.h declares, and its host-side
container walk (the plan) agrees with the oracle's walk on every fixture.  No compute calls: the
decode entry points need a GPU and must fail loudly (never fall back to the CPU) without one."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, tile_key, tile_paths


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "covt.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(covt_[a-z0-9_]+)\s*\(", hdr)))


def test_header_symbols_exported(covt):
    so = os.path.join(ROOT, "cov-tiles_amd", "libcovt.so")
    assert os.path.exists(so), "run __graft_entry__.build()"
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (covt_\w+)", out))
    decl = declared_symbols()
    assert len(decl) >= 23
    missing = [s for s in decl if s not in exported]
    assert not missing, missing
    assert set(decl) == set(covt.EXPORTED_SYMBOLS)
    L = covt.lib()
    for s in decl:
        assert hasattr(L, s)


def test_kernel_compiled_for_gfx950():
    """The fat binary embedded in libcovt.so carries a gfx950 code object (and nothing else)."""
    blob = open(os.path.join(ROOT, "cov-tiles_amd", "libcovt.so"), "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}  # (hipcub's host-side arch tables name other targets as strings)


def test_library_built_from_these_sources(covt):
    """libcovt.so carries the sha256 of the sources it was compiled from (Makefile BUILD_ID): a library
    that travels with the tree to the GPU box is the one these sources build (bench.py records both ids)."""
    assert covt.library_build_id() == covt.source_build_id(), "stale libcovt.so: run __graft_entry__.build()"


def test_struct_layouts(covt):
    import ctypes as C

    assert C.sizeof(covt.StreamDesc) == 32
    assert C.sizeof(covt.StreamResult) == 8
    assert C.sizeof(covt.StreamInfo) == 72


@pytest.mark.parametrize("fmt_mode", [(0, 0), (0, 1)])
def test_plan_matches_oracle_walk(covt, oracle, fmt_mode):
    fmt, id_mode = fmt_mode
    paths = tile_paths()
    tiles = [open(p, "rb").read() for p in paths]
    plan = covt.Plan.from_tiles(tiles, fmt, id_mode)
    st = plan.streams
    assert plan.num_streams == len(st)
    # every stream owns one descriptor (its result entry); split streams add chunks + pads
    di = np.sort(st["desc_index"])
    assert np.unique(di).size == plan.num_streams and di.max() < plan.num_descs
    assert np.array_equal(plan.desc_streams[st["desc_index"]], np.arange(plan.num_streams))
    descs = plan.descs.view(np.uint8).reshape(-1, 32)
    for t, p in enumerate(paths):
        ost, oss = oracle.walk_tile(tiles[t])
        assert (plan.tile_status[t] == 0) == (ost == 0), tile_key(p)
        idx = np.nonzero(st["tile"] == t)[0]
        assert len(idx) == len(oss)
        for i, s in zip(idx, oss):
            row = st[i]
            assert (row["layer"], row["column_kind"], row["stream_type"], row["encoding"], row["column_type"],
                    row["num_values"], row["byte_length"], row["num_bits"]) == \
                   (s.layer, s.column_kind, s.stream_type, s.encoding, s.column_type, s.num_values,
                    s.byte_length, s.num_bits)
            assert row["in_off"] == int(plan.offsets[t]) + s.offset
            eb, ne = oracle.stream_output(s, id_mode)
            if row["op"] != covt.OP_NONE:
                assert (row["elem_bytes"], row["out_elems"]) == (eb, ne)
            assert row["out_off"] % 128 == 0  # every stream slice starts on a 128-byte line (kOutAlign)
            d = descs[row["desc_index"]]
            assert int.from_bytes(d[0:8].tobytes(), "little") == row["in_off"]
            assert int.from_bytes(d[8:16].tobytes(), "little") == row["out_off"]
            assert d[24] == row["op"]
    # output slices are disjoint and in bounds
    ends = st["out_off"] + st["out_elems"] * st["elem_bytes"]
    order = np.argsort(st["out_off"], kind="stable")
    assert (st["out_off"][order][1:] >= ends[order][:-1]).all()
    assert ends.max() <= plan.output_bytes


@pytest.mark.parametrize("id_mode", [0, 1])
def test_plan_properties_match_oracle_walk(covt, oracle, id_mode):
    """COVT_PLAN_PROPERTIES: one record per property (sub)column in the oracle's walk order, its decode
    streams (column_kind 2) on the right payload bytes with CovtParser.decodePropertyColumn's ops, and
    disjoint 16-byte aligned output slices; Id/Geometry streams unchanged."""
    paths = tile_paths()
    tiles = [open(p, "rb").read() for p in paths]
    plan = covt.Plan.from_tiles(tiles, 0, id_mode, covt.PLAN_PROPERTIES)
    plain = covt.Plan.from_tiles(tiles, 0, id_mode)
    st = plan.streams
    assert np.array_equal(st[st["column_kind"] != 2][["tile", "layer", "stream_type", "op", "in_off"]],
                          plain.streams[["tile", "layer", "stream_type", "op", "in_off"]])
    P = plan.props
    k = 0
    for t, p in enumerate(paths):
        ost, props = oracle.walk_properties(tiles[t])
        assert ost == 0
        for q in props:
            r = P[k]
            assert (r["tile"], r["layer"], r["column"], r["lang"], r["n_features"]) == \
                   (t, q.layer, q.column, q.lang, q.n_features)
            assert plan.property_name(k) == oracle.prop_name(tiles[t], q)
            for role in range(3):
                si = int(r["stream"][role])
                if si < 0:
                    continue
                s = st[si]
                assert s["column_kind"] == 2 and s["stream_type"] == role
                assert s["in_off"] == int(plan.offsets[t]) + q.s_off[role]
                if role == 0:
                    assert s["op"] == covt.OP_BYTE_RLE_RAW and s["out_elems"] == (q.n_features + 7) // 8
                elif q.type == covt.PROP_INT64:
                    assert s["op"] == {5: covt.OP_RLE_S64,
                                       2: (covt.OP_VARINT_ZZ_S64, covt.OP_VARINT_ZZ_I32_AS_I64)[id_mode],
                                       4: (covt.OP_VARINT_ZZ_DELTA_S64, covt.OP_VARINT_ZZ_DELTA_I64)[id_mode]}[q.s_enc[1]]
                elif q.type == covt.PROP_STRING:
                    assert s["op"] == covt.OP_RLE_I32
            k += 1
    assert k == plan.num_property_columns
    owners = plan.pdescs["flags"] & covt.PROP_DICT_OWNER != 0
    assert owners.sum() >= 2500
    ends = []
    for r, d in zip(P, plan.pdescs[P["desc_index"]]):
        assert (d["out_off"] == r["out_off"]).all()
        for m in range(4):
            if r["out_off"][m] >= 0:
                assert r["out_off"][m] % 16 == 0 and r["out_off"][m] <= plan.property_bytes
    assert plan.property_bytes > 0


def test_plan_op_selection_follows_covtparser_dispatch(covt):
    """CovtParser.decodeGeometryColumn (:392-511) / decodedIds (:552-572) dispatch table."""
    t = open(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "5_16_20.covt"), "rb").read()
    for id_mode, id_ops in ((0, {5: covt.OP_RLE_U64, 1: covt.OP_VARINT_U64, 4: covt.OP_RLE_U64}),
                            (1, {5: covt.OP_RLE_U64, 1: covt.OP_VARINT_I32_AS_I64, 4: covt.OP_VARINT_ZZ_DELTA_I64})):
        plan = covt.Plan.from_tiles([t], 0, id_mode)
        for s in plan.streams:
            if s["column_kind"] == 0:
                assert s["op"] == id_ops[int(s["encoding"])]
            elif s["stream_type"] == 4:
                assert s["op"] == covt.OP_BYTE_RLE_U8
            elif s["stream_type"] in (5, 6, 7):
                assert s["op"] == {5: covt.OP_RLE_I32, 9: covt.OP_FPF_ZZ_DELTA_I32}[int(s["encoding"])]
            elif s["stream_type"] == 8:
                assert s["op"] == {4: covt.OP_VARINT_ZZ_DELTA_I32, 9: covt.OP_FPF_ZZ_DELTA_I32}[int(s["encoding"])]
            elif s["column_type"] == 4:
                assert s["op"] == {4: covt.OP_VARINT_DELTA_MORTON, 9: covt.OP_FPF_DELTA_MORTON}[int(s["encoding"])]
            else:
                assert s["op"] == {4: covt.OP_VARINT_ZZ_DELTA_XY, 9: covt.OP_FPF_ZZ_DELTA_XY}[int(s["encoding"])]


def test_plan_rejects_truncated_and_garbage(covt):
    t = open(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "5_16_20.covt"), "rb").read()
    rng = np.random.default_rng(5)
    tiles = [t[:len(t) // 2], t[:100], b"", bytes(rng.integers(0, 256, size=3000).astype(np.uint8)), t]
    plan = covt.Plan.from_tiles(tiles)
    assert (plan.tile_status[:4] != 0).all() and plan.tile_status[4] == 0
    assert set(np.unique(plan.streams["tile"])) == {4}


def test_no_cpu_fallback_without_gpu(covt):
    """The product path raises when no device is usable; it never decodes on the CPU."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(covt.CovtError):
        covt.DecodingUtils.decodeVarint(b"\x01\x02", covt.IntWrapper(0), 2)
    plan = covt.Plan.from_tiles([open(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "2_2_2.covt"),
                                      "rb").read()])
    with pytest.raises(covt.CovtError):
        plan.decode_host()


def test_host_entry_rejects_short_buffer(covt):
    """covt_plan_decode_host[_multi|_shards] check n_bytes against the plan's tiles before any device
    call (a short caller buffer would otherwise be read past its end)."""
    import ctypes as C

    t = open(os.path.join(ROOT, "tests", "golden", "tiles", "omt", "5_16_20.covt"), "rb").read()
    plan = covt.Plan.from_tiles([t, t])
    L = covt.lib()
    out = np.zeros(plan.output_bytes, dtype=np.uint8)
    res = np.zeros((plan.num_streams, 2), dtype=np.int32)
    blob = plan.blob
    short = int(plan.offsets[1] + plan.sizes[1]) - 1
    u8 = blob.ctypes.data_as(C.POINTER(C.c_uint8))
    assert L.covt_plan_decode_host(plan._h, u8, short, out.ctypes.data, res.ctypes.data) == covt.ERR_INVALID_ARG
    assert L.covt_plan_decode_host_multi(plan._h, u8, short, 2, out.ctypes.data, res.ctypes.data) == \
        covt.ERR_INVALID_ARG
    devs = np.zeros(2, dtype=np.int32)
    assert L.covt_plan_decode_host_shards(plan._h, u8, short, 2, devs.ctypes.data_as(C.POINTER(C.c_int32)),
                                          out.ctypes.data, res.ctypes.data) == covt.ERR_INVALID_ARG
    assert L.covt_plan_decode_host(plan._h, None, 0, out.ctypes.data, res.ctypes.data) == covt.ERR_INVALID_ARG
    assert L.covt_plan_release_device(plan._h) == covt.OK


def test_floats_le_and_string_entries(covt):
    """decodeFloatsLE (DecodingUtils.java:446) and decodeString (:21, :28): host-side views, Java bounds."""
    D = covt.DecodingUtils
    vals = np.array([1.5, -2.25, 3e38, np.inf], dtype="<f4")
    buf = b"\x07" + vals.tobytes() + b"\x00"
    p = covt.IntWrapper(1)
    assert np.array_equal(D.decodeFloatsLE(buf, p, 4), vals) and p.get() == 17
    with pytest.raises(covt.ArrayIndexOutOfBoundsException):
        D.decodeFloatsLE(buf, covt.IntWrapper(3), 4)
    s = "Zürich 東京".encode("utf-8")
    buf = b"\xff" + bytes([len(s)]) + s + b"tail"
    p = covt.IntWrapper(1)
    assert D.decodeString(buf, p) == "Zürich 東京" and p.get() == 2 + len(s)
    assert D.decodeString(buf, p, 4) == "tail" and p.get() == len(buf)
    long = b"x" * 300
    buf = bytes([0x80 | (300 & 0x7f), 300 >> 7]) + long
    p = covt.IntWrapper(0)
    assert D.decodeString(buf, p) == long.decode() and p.get() == len(buf)
    with pytest.raises(covt.ArrayIndexOutOfBoundsException):
        D.decodeString(buf[:-1], covt.IntWrapper(0))


def test_device_batch_api_surface(covt):
    """The device-resident batch classes keep their whole method set (checked on CPU)."""
    for m in ("decode", "decode_graph", "subset", "assemble", "materialize_properties", "results",
              "assembly_results", "property_results"):
        assert callable(getattr(covt.DeviceBatch, m, None)), m
    for m in ("decode", "results"):
        assert callable(getattr(covt.DeviceSubset, m, None)), m


def test_python_constants_mirror_header(covt):
    """Every #define of include/covt.h that the Python module mirrors (same name without COVT_) has the same
    value: launch modes and FastPFOR kernel flags, families, descriptor flags, scratch release flags, ..."""
    hdr = open(os.path.join(ROOT, "include", "covt.h")).read()
    defs = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define COVT_([A-Z0-9_]+)\s+(0x[0-9a-fA-F]+|\d+)u?\b", hdr)}
    checked = [k for k in defs if isinstance(getattr(covt, k, None), int)]
    for k in checked:
        assert getattr(covt, k) == defs[k], k
    for k in ("LAUNCH_AUTO", "LAUNCH_FUSED", "LAUNCH_FORKED", "LAUNCH_FPF_STREAM", "LAUNCH_FPF_CLASSIC",
              "FAMILY_FASTPFOR", "FAMILY_SPLIT_FPF", "DESC_SPLIT", "RELEASE_PINNED", "INPUT_PADDING"):
        assert k in checked, k
