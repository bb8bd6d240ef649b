"""GPU parity of the split-stream path (COVT_FAMILY_SPLIT, include/covt.h): long Java-capped varint
streams decoded by one wave per chunk with a decoupled look-back must equal the one-wave decode and
the oracle (DecodingUtils.java:35-112, :394-409) bit for bit -- values, running sums across chunk
edges, x/y parity, the consumed position, and the errors of short streams.

* every stream of every fixture tile with splitting forced at small chunk sizes, both Id modes;
* adversarial byte strings (long runs of continuation bytes, so values capped at 4 bytes end on a
  byte with bit 7 set, also right at chunk edges), exact / short (trailing bytes) / over-long
  (truncated) value counts, every split op, chunk sizes from 16 bytes to 4 KiB;
* 64-bit LEB128 id streams (VARINT_U64, ZZ_S64): values up to 10 bytes, over-long (11 byte to 2 KiB)
  values before, at and after num_values -- an error only when one of the first num_values is.
"""
import hashlib

import numpy as np
import pytest

from conftest import tile_key, tile_paths

pytestmark = pytest.mark.gpu

DESC = np.dtype([("in_off", np.uint64), ("out_off", np.uint64), ("avail", np.int32), ("num_values", np.int32),
                 ("op", np.uint8), ("num_bits", np.uint8), ("flags", np.uint16), ("byte_length", np.int32)])


@pytest.mark.parametrize("chunk,values,launch", [(100, 256, 0), (1024, 2048, 0), (100, 256, 1), (1024, 2048, 2)],
                         ids=["c100_auto", "c1024_auto", "c100_fused", "c1024_forked"])
@pytest.mark.parametrize("id_mode", [0, 1], ids=["id_format", "id_java"])
def test_fixtures_forced_split(covt, gpu_available, golden_streams, chunk, values, id_mode, launch):
    import torch

    paths = tile_paths()
    keys = [tile_key(p) for p in paths]
    tiles = [open(p, "rb").read() for p in paths]
    opts = covt.PlanOptions(split_min=200, split_ratio=0, split_chunk=chunk, split_values=values)
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GENC, id_mode, options=opts)
    assert plan.family_counts[covt.FAMILY_SPLIT] > 1000 and plan.family_counts[covt.FAMILY_SPLIT_FPF] > 100
    assert plan.family_counts[covt.FAMILY_SPLIT_RLE] > 100
    db = covt.DeviceBatch(plan, "cuda")
    for _ in range(2):  # the look-back records are reset per launch
        db.decode(launch=launch)
    torch.cuda.synchronize()
    out, res = db.results()
    col = golden_streams["columns"]
    pre = "fmt_" if id_mode == 0 else "java_"
    ish, ist, ico = col.index(pre + "sha256"), col.index(pre + "status"), col.index(pre + "consumed")
    st = plan.streams
    fam0 = int(plan.family_counts[:covt.FAMILY_SPLIT].sum())
    n_split = 0
    for t, key in enumerate(keys):
        rec = golden_streams["tiles"][key]
        if rec["walk_status"] != 0:
            continue
        idx = np.nonzero(st["tile"] == t)[0]
        for i, row in zip(idx, rec["streams"]):
            n_split += int(st["desc_index"][i] >= fam0)
            assert (int(res[i][0]) == 0) == (row[ist] == 0), (key, int(i))
            if row[ist] != 0:
                continue
            assert int(res[i][1]) == row[ico], (key, int(i))
            assert hashlib.sha256(plan.stream_array(out, int(i)).tobytes()).hexdigest() == row[ish], (key, int(i))
    assert n_split > 300


def _j4_count(b: bytes) -> int:
    """Values Java's 4-byte-capped decodeVarint reads from the whole buffer (DecodingUtils.java:157-186)."""
    p = n = 0
    while p < len(b):
        k = 0
        while k < 3 and p + k < len(b) and b[p + k] & 0x80:
            k += 1
        if p + k >= len(b):
            break  # a value cut off by the end
        p += k + 1
        n += 1
    return n


LAUNCHES = pytest.mark.parametrize("launch", [1, 2], ids=["fused", "forked"])  # COVT_LAUNCH_FUSED / _FORKED


def _split_launch(covt, buf: bytes, op: int, n: int, nb: int, chunk: int, out_bytes: int, fpf=False, states=None,
                  launch=0):
    """One split stream through the grouped launch: byte chunks (varint) or value chunks (FastPFOR).
    states: FastPFOR chunk start states (nch x 42 int32, the plan's host walk) for pads [2..7]."""
    import ctypes as C

    import torch

    bl = len(buf)
    total = n if fpf else bl
    nch = (total + chunk - 1) // chunk
    fl = covt.DESC_SPLIT_FPF if fpf else 0
    d = np.zeros(nch * covt.SPLIT_SLOTS, dtype=DESC)
    for c in range(nch):
        k = c * covt.SPLIT_SLOTS
        d[k] = (0, 0, c, n, op, nb, covt.DESC_SPLIT | fl, bl)
        d[k + 1 : k + covt.SPLIT_SLOTS]["flags"] = covt.DESC_SPLIT_PAD | fl
        d[k + 1]["in_off"], d[k + 1]["out_off"] = c * chunk, min((c + 1) * chunk, total)
        if states is not None:  # seven int32 slots per pad, every field but op / num_bits / flags
            raw = d.view(np.uint8).reshape(-1, 32)
            for i in range(42):
                o = (0, 4, 8, 12, 16, 20, 28)[i % 7]
                raw[k + 2 + i // 7, o:o + 4] = np.frombuffer(np.int32(states[c, i]).tobytes(), dtype=np.uint8)
    counts = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
    counts[covt.FAMILY_SPLIT_FPF if fpf else covt.FAMILY_SPLIT] = d.size
    dev = torch.device("cuda")
    d_in = torch.zeros(bl + covt.INPUT_PADDING + 16, dtype=torch.uint8, device=dev)
    d_in[:bl] = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev) if bl else d_in[:0]
    d_desc = torch.from_numpy(d.view(np.uint8)).to(dev)
    d_out = torch.full((out_bytes + 16,), 0x5A, dtype=torch.uint8, device=dev)
    d_res = torch.full((d.size * 2,), 0x33, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    st = covt.lib().covt_decode_streams_device_grouped_mode(d_in.data_ptr(), d_desc.data_ptr(),
                                                            counts.ctypes.data_as(C.POINTER(C.c_int64)),
                                                            d_out.data_ptr(), d_res.data_ptr(), s.cuda_stream, launch)
    assert st == 0
    torch.cuda.synchronize()
    return d_out.cpu().numpy()[:out_bytes], d_res.cpu().numpy().reshape(-1, 2)[0]


def _oracle(oracle, covt, op, buf, n, nb):
    O = oracle
    if op in (covt.OP_VARINT_I32, covt.OP_VARINT_I32_AS_I64):
        st, arr, pos = O.decode_varint(buf, 0, n)[:3]
    elif op in (covt.OP_VARINT_ZZ_I32, covt.OP_VARINT_ZZ_I32_AS_I64):
        st, arr, pos = O.decode_zigzag_varint(buf, 0, n)[:3]
    elif op in (covt.OP_VARINT_ZZ_DELTA_I32, covt.OP_VARINT_ZZ_DELTA_I64):
        st, arr, pos = O.decode_zigzag_delta_varint(buf, 0, n)[:3]
    elif op == covt.OP_VARINT_ZZ_DELTA_XY:
        st, arr, pos = O.decode_zigzag_delta_varint_coordinates(buf, 0, n)[:3]
    else:
        st, arr, pos = O.decode_delta_varint_morton_codes(buf, 0, n, nb)[:3]
    if op in (covt.OP_VARINT_I32_AS_I64, covt.OP_VARINT_ZZ_I32_AS_I64, covt.OP_VARINT_ZZ_DELTA_I64):
        arr = np.asarray(arr, dtype=np.int32).astype(np.int64)
    return st, np.asarray(arr), pos


def _streams(rng, oracle):
    """(name, bytes) adversarial and plain varint byte strings."""
    out = []
    vals = rng.integers(0, 1 << 28, size=9000, dtype=np.uint64) >> rng.integers(0, 28, size=9000).astype(np.uint64)
    out.append(("plain", oracle.encode_varints(vals)))
    for p_cont in (0.5, 0.8, 0.97):  # runs of continuation bytes: values capped at 4 bytes
        b = rng.random(20000) < p_cont
        raw = rng.integers(0, 128, size=b.size).astype(np.uint8) | (b.astype(np.uint8) << 7)
        out.append(("rand%.2f" % p_cont, raw.tobytes()))
    out.append(("all_cont", b"\x80" * 9001))  # every value is four continuation bytes
    z = bytearray(oracle.encode_varints(rng.integers(0, 200, size=3000, dtype=np.uint64)))
    for k in range(0, len(z) - 8, 97):  # capped values sprinkled in
        z[k:k + 4] = b"\xff\x81\x80\x80"
    out.append(("sprinkled", bytes(z)))
    return out


@LAUNCHES
@pytest.mark.parametrize("chunk", [16, 64, 100, 1000, 4096])
def test_adversarial_streams_split(covt, oracle, gpu_available, chunk, launch):
    rng = np.random.default_rng(chunk)
    ops = [covt.OP_VARINT_I32, covt.OP_VARINT_ZZ_I32, covt.OP_VARINT_ZZ_DELTA_I32, covt.OP_VARINT_ZZ_DELTA_XY,
           covt.OP_VARINT_DELTA_MORTON, covt.OP_VARINT_I32_AS_I64, covt.OP_VARINT_ZZ_I32_AS_I64,
           covt.OP_VARINT_ZZ_DELTA_I64]
    n_checked = 0
    for name, buf in _streams(rng, oracle):
        total = _j4_count(buf)
        for op in ops:
            nb = 14 if op == covt.OP_VARINT_DELTA_MORTON else 0
            for n in (total, total - 37, total + 1, 1):
                if op == covt.OP_VARINT_ZZ_DELTA_XY and n & 1:
                    n -= 1  # the plan never splits odd x,y streams
                if n <= 0:
                    continue  # nor empty ones
                nvals = n  # varints to read (Morton: one per vertex)
                ebytes = (8 if op in (covt.OP_VARINT_I32_AS_I64, covt.OP_VARINT_ZZ_I32_AS_I64,
                                      covt.OP_VARINT_ZZ_DELTA_I64) else 4) * (2 * nvals if nb else nvals)
                o_st, o_arr, o_pos = _oracle(oracle, covt, op, buf, nvals, nb)
                out, r = _split_launch(covt, buf, op, nvals, nb, chunk, ebytes, launch=launch)
                assert (int(r[0]) == 0) == (o_st == 0), (name, op, n, int(r[0]), o_st)
                if o_st == 0:
                    assert int(r[1]) == o_pos, (name, op, n)
                    got = out.view(np.int64 if ebytes == 8 * (2 * nvals if nb else nvals) else np.int32)
                    assert np.array_equal(got, o_arr.astype(got.dtype)), (name, op, n)
                n_checked += 1
    assert n_checked > 150


@LAUNCHES
@pytest.mark.parametrize("values", [256, 512, 4096])
def test_fastpfor_streams_split(covt, oracle, gpu_available, values, launch):
    """FastPFOR streams split into chunks of whole blocks: every chunk walks the page directories and the
    block headers before its range, sums its values in a first pass and stores them with its
    predecessors' carry in a second (exceptions of index 1 and > 1, all bit widths, multi-page, VByte
    tails, zero-filled and over-long value counts, corrupted payloads)."""
    from test_gpu_synthetic import _fpf_values

    rng = np.random.default_rng(values)
    n_checked = 0
    for n in (300, 1000, 4096 + 77, 65536, 65536 + 256 + 13, 140000):
        raw = _fpf_values(rng, n)
        enc = oracle.encode_fastpfor(raw)
        buf = b"\x01\x02\x03" + enc + b"\x09" * 5
        bl = len(enc)
        body = buf[3:]
        for op, nb in ((covt.OP_FPF_ZZ_DELTA_I32, 0), (covt.OP_FPF_ZZ_DELTA_XY, 0), (covt.OP_FPF_DELTA_MORTON, 14)):
            for nv in (n, n + 10):  # numValues past the coded values: Java's zero-filled tail
                if op == covt.OP_FPF_ZZ_DELTA_XY and nv & 1:
                    continue
                if op == covt.OP_FPF_ZZ_DELTA_I32:
                    o = oracle.decode_fastpfor_zigzag_delta(body, nv, bl, 0)
                elif op == covt.OP_FPF_ZZ_DELTA_XY:
                    o = oracle.decode_fastpfor_delta_coordinates(body, nv, bl, 0)
                else:
                    o = oracle.decode_fastpfor_delta_morton_codes(body, nv, bl, 0, nb)
                ne = 2 * nv if nb else nv
                out, r = _split_launch(covt, body[:bl], op, nv, nb, values, 4 * ne, fpf=True, launch=launch)
                assert (int(r[0]) == 0) == (o[0] == 0), (n, op, nv, int(r[0]), o[0])
                if o[0] == 0:
                    assert int(r[1]) == bl
                    assert np.array_equal(out.view(np.int32), np.asarray(o[1], dtype=np.int32)), (n, op, nv)
                n_checked += 1
    # corrupted payloads: a status (never a fault), equal arrays whenever the oracle decodes
    raw = _fpf_values(rng, 5000)
    enc = oracle.encode_fastpfor(raw)
    for _ in range(12):
        e = bytearray(enc)
        for _ in range(int(rng.integers(1, 4))):
            e[int(rng.integers(0, len(e)))] ^= 1 << int(rng.integers(0, 8))
        e = bytes(e)
        o = oracle.decode_fastpfor_zigzag_delta(e, 5000, len(e), 0)
        out, r = _split_launch(covt, e, covt.OP_FPF_ZZ_DELTA_I32, 5000, 0, values, 4 * 5000, fpf=True,
                               launch=launch)
        if o[0] == 0:
            assert int(r[0]) == 0 and np.array_equal(out.view(np.int32), np.asarray(o[1], dtype=np.int32))
        n_checked += 1
    assert n_checked > 40


@pytest.mark.parametrize("values", [256, 2048])
def test_fastpfor_split_host_states(covt, oracle, gpu_available, values):
    """FastPFOR chunks given the plan's host walk of the headers before them (pads [2..7], as
    covt_plan_create leaves them; covt_debug_fpf_chunk_states): bit-exact with the oracle on well-formed
    single- and multi-page streams; on bit-flipped ones a status, and the oracle's arrays whenever it
    decodes (states present before the damage, absent after it)."""
    from test_gpu_synthetic import _fpf_values
    from test_split_plan import _states_hook

    rng = np.random.default_rng(100 + values)
    n_checked = 0
    for n in (1000, 4096 + 77, 65536 + 256 + 13, 140000):
        enc = oracle.encode_fastpfor(_fpf_values(rng, n))
        st = _states_hook(covt, enc, n, values)
        assert st[:, 0].sum() > 0 or n <= values  # (one chunk: nothing before it to walk)
        for op, nb in ((covt.OP_FPF_ZZ_DELTA_I32, 0), (covt.OP_FPF_ZZ_DELTA_XY, 0), (covt.OP_FPF_DELTA_MORTON, 14)):
            if op == covt.OP_FPF_ZZ_DELTA_XY and n & 1:
                continue
            if op == covt.OP_FPF_ZZ_DELTA_I32:
                o = oracle.decode_fastpfor_zigzag_delta(enc, n, len(enc), 0)
            elif op == covt.OP_FPF_ZZ_DELTA_XY:
                o = oracle.decode_fastpfor_delta_coordinates(enc, n, len(enc), 0)
            else:
                o = oracle.decode_fastpfor_delta_morton_codes(enc, n, len(enc), 0, nb)
            ne = 2 * n if nb else n
            out, r = _split_launch(covt, enc, op, n, nb, values, 4 * ne, fpf=True, states=st)
            assert o[0] == 0 and int(r[0]) == 0 and int(r[1]) == len(enc), (n, op)
            assert np.array_equal(out.view(np.int32), np.asarray(o[1], dtype=np.int32)), (n, op)
            n_checked += 1
    enc = oracle.encode_fastpfor(_fpf_values(rng, 70000))
    for _ in range(16):
        e = bytearray(enc)
        for _ in range(int(rng.integers(1, 4))):
            e[int(rng.integers(0, len(e)))] ^= 1 << int(rng.integers(0, 8))
        e = bytes(e)
        st = _states_hook(covt, e, 70000, values)
        o = oracle.decode_fastpfor_zigzag_delta(e, 70000, len(e), 0)
        out, r = _split_launch(covt, e, covt.OP_FPF_ZZ_DELTA_I32, 70000, 0, values, 4 * 70000, fpf=True, states=st)
        if o[0] == 0:  # (as the one-wave test: a status always, the oracle's arrays whenever it decodes)
            assert int(r[0]) == 0 and np.array_equal(out.view(np.int32), np.asarray(o[1], dtype=np.int32))
        n_checked += 1
    assert n_checked > 20


def _u64_count(b: bytes) -> int:
    """Terminators (bytes with bit 7 clear) = 64-bit LEB128 values in the buffer."""
    return int(np.count_nonzero(np.frombuffer(b, dtype=np.uint8) < 0x80))


def _u64_streams(rng, oracle):
    big = rng.integers(0, 1 << 63, size=6000, dtype=np.uint64) >> rng.integers(0, 63, size=6000).astype(np.uint64)
    plain = oracle.encode_varints(big)
    out = [("plain", plain)]
    for bad_len in (11, 40, 1500, 2100):  # one over-long value, at three places
        for frac in (0.02, 0.5, 0.97):
            k = _u64_count(plain[: int(len(plain) * frac)])
            cut = [i for i, x in enumerate(plain) if x < 0x80][k] + 1  # after value k
            out.append(("bad%d@%.2f" % (bad_len, frac), plain[:cut] + b"\x81" * (bad_len - 1) + b"\x01" + plain[cut:]))
    out.append(("tail_cont", plain + b"\x80" * 3000))  # trailing bytes without a terminator
    return out


@pytest.mark.parametrize("chunk", [16, 100, 1024, 2048])
def test_u64_streams_split(covt, oracle, gpu_available, chunk):
    rng = np.random.default_rng(1000 + chunk)
    n_checked = n_err = 0
    for name, buf in _u64_streams(rng, oracle):
        total = _u64_count(buf)
        for op in (covt.OP_VARINT_U64, covt.OP_VARINT_ZZ_S64):
            for n in (total, total - 37, total // 2, total + 1, 1):
                o_st, o_arr, o_pos = oracle.decode_varint_u64(buf, 0, n)
                if op == covt.OP_VARINT_ZZ_S64:
                    u = o_arr.astype(np.uint64)
                    o_arr = ((u >> np.uint64(1)) ^ (np.uint64(0) - (u & np.uint64(1)))).view(np.int64)
                out, r = _split_launch(covt, buf, op, n, 0, chunk, 8 * n)
                assert (int(r[0]) == 0) == (o_st == 0), (name, op, n, int(r[0]), o_st)
                if o_st == 0:
                    assert int(r[1]) == o_pos, (name, op, n)
                    assert np.array_equal(out.view(np.int64), o_arr.view(np.int64)), (name, op, n)
                else:
                    n_err += 1
                n_checked += 1
    assert n_checked > 100 and n_err > 10


def _rle_chunks(buf: bytes, n: int, byte_rle: bool, elem: int, unit: int):
    """Mirror of the plan's host walk (covt_host.cpp rle_chunks): chunks of whole ORC RLE groups,
    cut every `unit` of bytes + output bytes / 4; (chunks, consumed) or None if n values do not fit."""
    pos = v = cs = cv = 0
    ch = []

    def varint():
        nonlocal pos
        while True:
            if pos >= len(buf):
                return False
            b = buf[pos]
            pos += 1
            if not b & 0x80:
                return True

    while v < n:
        if pos >= len(buf):
            return None
        if (pos - cs) + (v - cv) * elem // 4 >= unit:
            ch.append((cs, pos, cv, v - cv))
            cs, cv = pos, v
        h = buf[pos]
        if h < 0x80:
            if byte_rle:
                if pos + 2 > len(buf):
                    return None
                pos += 2
            else:
                pos += 2
                if pos > len(buf) or not varint():
                    return None
            v += h + 3
        else:
            cnt = 256 - h
            pos += 1
            if byte_rle:
                if pos + cnt > len(buf):
                    return None
                pos += cnt
            else:
                for _ in range(cnt):
                    if not varint():
                        return None
            v += cnt
    ch.append((cs, pos, cv, n - cv))
    return ch, pos


def _rle_values(rng, n, big=False):
    """Runs (constant and stepped, negative deltas), literal stretches, optionally 64-bit magnitudes."""
    out = []
    while len(out) < n:
        k = int(rng.integers(1, 300))
        kind = int(rng.integers(0, 3))
        base = int(rng.integers(0, 1 << 62)) if big else int(rng.integers(0, 1 << 20))
        if kind == 0:
            out += [base] * k
        elif kind == 1:
            d = int(rng.integers(-128, 128))
            out += [max(base + d * i, 0) for i in range(k)]
        else:
            hi = (1 << 62) if big else (1 << 20)
            out += [int(x) for x in rng.integers(0, hi, size=k)]
    return np.array(out[:n], dtype=np.uint64)


@LAUNCHES
@pytest.mark.parametrize("unit", [64, 700, 4096])
def test_rle_streams_split(covt, oracle, gpu_available, unit, launch):
    """Long ORC RLE streams split at group starts by the plan's host walk: each chunk decodes its groups
    into its slice of the stream's output (byte RLE: shared edge packets written byte-exact), the
    stream's result = the lowest chunk status + the walked consumed bytes."""
    import ctypes as C

    import torch

    rng = np.random.default_rng(unit)
    cases = []
    for n in (3000, 20000):
        v = _rle_values(rng, n)
        cases.append((covt.OP_RLE_U64, oracle.encode_rle(v, False), n, 8))
        cases.append((covt.OP_RLE_I32, oracle.encode_rle(v, False), n, 4))
        vb = _rle_values(rng, n, big=True)
        cases.append((covt.OP_RLE_U64, oracle.encode_rle(vb, False), n, 8))
        s = vb.view(np.int64) >> np.int64(1)
        s[::3] = -s[::3]
        cases.append((covt.OP_RLE_S64, oracle.encode_rle(s, True), n, 8))
        bts = np.minimum(_rle_values(rng, n) % 7, 5).astype(np.uint8)
        cases.append((covt.OP_BYTE_RLE_U8, oracle.encode_byte_rle(bts), n, 1))
        raw = (_rle_values(rng, n) % 256).astype(np.uint8)
        cases.append((covt.OP_BYTE_RLE_RAW, oracle.encode_byte_rle(raw), n, 1))
        bad = bts.copy()
        bad[int(n * 0.9)] = 9  # GeometryType out of range in a late chunk
        cases.append((covt.OP_BYTE_RLE_U8, oracle.encode_byte_rle(bad), n, 1))
    dev = torch.device("cuda")
    n_checked = n_bad = 0
    for op, buf, total, elem in cases:
        byte_rle = op in (covt.OP_BYTE_RLE_U8, covt.OP_BYTE_RLE_RAW)
        for n in (total, total - 1, total // 3 + 1):
            walked = _rle_chunks(buf, n, byte_rle, elem, unit)
            if walked is None or len(walked[0]) < 2:
                continue
            ch, consumed = walked
            d = np.zeros(len(ch) * covt.SPLIT_SLOTS, dtype=DESC)
            for c, (s0, e0, v0, nv) in enumerate(ch):
                k = c * covt.SPLIT_SLOTS
                d[k] = (0, 0, c, n, op, 0, covt.DESC_SPLIT | covt.DESC_SPLIT_RLE, len(buf))
                d[k + 1 : k + covt.SPLIT_SLOTS]["flags"] = covt.DESC_SPLIT_PAD | covt.DESC_SPLIT_RLE
                d[k + 1]["in_off"], d[k + 1]["out_off"] = s0, e0
                d[k + 2]["in_off"], d[k + 2]["out_off"] = v0, nv
                d[k + 3]["in_off"] = consumed
            counts = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
            counts[covt.FAMILY_SPLIT_RLE] = d.size
            d_in = torch.zeros(len(buf) + covt.INPUT_PADDING + 16, dtype=torch.uint8, device=dev)
            d_in[:len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
            d_desc = torch.from_numpy(d.view(np.uint8)).to(dev)
            nbytes = n * elem
            d_out = torch.full((nbytes + 32,), 0x5A, dtype=torch.uint8, device=dev)
            d_res = torch.full((d.size * 2,), 0x33, dtype=torch.int32, device=dev)
            st = covt.lib().covt_decode_streams_device_grouped_mode(d_in.data_ptr(), d_desc.data_ptr(),
                                                                    counts.ctypes.data_as(C.POINTER(C.c_int64)),
                                                                    d_out.data_ptr(), d_res.data_ptr(),
                                                                    torch.cuda.current_stream().cuda_stream, launch)
            assert st == 0
            torch.cuda.synchronize()
            out = d_out.cpu().numpy()
            r = d_res.cpu().numpy().reshape(-1, 2)[0]
            if byte_rle:
                o_st, o_arr, _, o_cons = oracle.decode_byte_rle(buf, n, 0, len(buf))
                if op == covt.OP_BYTE_RLE_U8 and o_st == 0 and (np.asarray(o_arr) > 5).any():
                    o_st = covt.ERR_BAD_HEADER
            else:
                o_st, o_arr, _, o_cons = oracle.decode_rle(buf, n, 0, op == covt.OP_RLE_S64)
            assert (int(r[0]) == 0) == (o_st == 0), (op, n, unit, int(r[0]), o_st)
            n_bad += o_st != 0
            if o_st == 0:
                assert int(r[1]) == o_cons, (op, n, unit)
                dt = {1: np.uint8, 4: np.int32, 8: np.int64}[elem]
                got = out[:nbytes].view(dt)
                assert np.array_equal(got, np.asarray(o_arr).astype(np.int64).astype(dt)), (op, n, unit)
                assert (out[nbytes:] == 0x5A).all(), (op, n, unit)  # chunks write nothing past the stream
            n_checked += 1
    assert n_checked > 20 and n_bad > 0
