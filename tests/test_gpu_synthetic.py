"""GPU vs oracle on seeded synthetic streams built with the oracle's encoders (restated
EncodingUtils / ORC writers / JavaFastPFOR compress): varint widths 1-4 B and the Java 4-byte cap,
RLE run/literal mixes incl. 64-bit values, FastPFOR with b in 0..32, exception index 1 and >1,
multi-page (>65536 values) and VariableByte tails of 0-255 values, empty and truncated streams."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def zz32(v):
    v = np.asarray(v, dtype=np.int64)
    return ((v << 1) ^ (v >> 63)) & 0xFFFFFFFF


def _check(got_fn, ora):
    """got_fn: () -> (values, pos); ora: (status, values, pos[, ...])"""
    if ora[0] != 0:
        with pytest.raises(Exception):
            got_fn()
        return
    vals, pos = got_fn()
    assert np.array_equal(vals, ora[1])
    assert pos == ora[2]


def _call(D, covt, name, *args, pos_index):
    def f():
        a = list(args)
        p = covt.IntWrapper(a[pos_index])
        a[pos_index] = p
        v = getattr(D, name)(*a)
        return v, p.get()
    return f


@pytest.mark.parametrize("seed", range(6))
def test_varint_family(covt, oracle, gpu_available, seed):
    rng = np.random.default_rng(seed)
    D = covt.DecodingUtils
    n = int(rng.integers(0, 5000))
    width = rng.integers(1, 5, size=n)
    vals = (rng.integers(0, 1 << 28, size=n) >> (7 * (4 - width))).astype(np.uint64)
    prefix = bytes(rng.integers(0, 256, size=int(rng.integers(0, 40))).astype(np.uint8))
    buf = prefix + oracle.encode_varints(vals) + bytes(rng.integers(0, 256, size=7).astype(np.uint8))
    p0 = len(prefix)
    _check(_call(D, covt, "decodeVarint", buf, p0, n, pos_index=1), oracle.decode_varint(buf, p0, n))
    _check(_call(D, covt, "decodeZigZagVarint", buf, p0, n, pos_index=1), oracle.decode_zigzag_varint(buf, p0, n))
    _check(_call(D, covt, "decodeZigZagDeltaVarint", buf, p0, n, pos_index=1),
           oracle.decode_zigzag_delta_varint(buf, p0, n))
    n2 = n - (n & 1)
    _check(_call(D, covt, "decodeZigZagDeltaVarintCoordinates", buf, p0, n2, pos_index=1),
           oracle.decode_zigzag_delta_varint_coordinates(buf, p0, n2))
    for nb in (13, 14, 1, 16, 17, 31, 32, 0):
        _check(_call(D, covt, "decodeDeltaVarintMortonCodes", buf, p0, n, nb, pos_index=1),
               oracle.decode_delta_varint_morton_codes(buf, p0, n, nb))


@pytest.mark.parametrize("seed", range(8))
def test_varint_java_cap_adversarial(covt, oracle, gpu_available, seed):
    """Random bytes biased to continuation bytes: exercises the 4-byte cap (DecodingUtils.java:157-186)
    and truncation at the end of the buffer."""
    rng = np.random.default_rng(100 + seed)
    D = covt.DecodingUtils
    m = int(rng.integers(1, 3000))
    b = rng.integers(0, 256, size=m).astype(np.uint8)
    b[rng.random(m) < 0.7] |= 0x80
    buf = bytes(b)
    for n in (1, m // 8, m // 4, m // 2, m):
        _check(_call(D, covt, "decodeVarint", buf, 0, n, pos_index=1), oracle.decode_varint(buf, 0, n))
        _check(_call(D, covt, "decodeZigZagDeltaVarint", buf, 0, n, pos_index=1),
               oracle.decode_zigzag_delta_varint(buf, 0, n))


def _rle_values(rng, n, signed):
    out = []
    while len(out) < n:
        kind = rng.integers(0, 5)
        if kind == 4:  # a long arithmetic sequence across a 2^32 multiple: a chain of runs with one delta
            d = int(rng.integers(1, 128)) * (1 if rng.integers(0, 2) else -1)
            m = int(rng.integers(131, 2000))
            edge = int(rng.integers(1, 4)) << 32
            base = (-edge if signed and rng.integers(0, 2) else edge) - d * int(rng.integers(0, m))
            if not signed and base + d * m < 0:
                base, d = edge, abs(d)
            out += [base + i * d for i in range(m)]
        elif kind == 0:  # run with small delta
            base = int(rng.integers(-(1 << 40), 1 << 40)) if signed else int(rng.integers(0, 1 << 40))
            d = int(rng.integers(-128, 128))
            out += [base + i * d for i in range(int(rng.integers(3, 300)))]
        elif kind == 1:  # constant run
            out += [int(rng.integers(0, 100))] * int(rng.integers(1, 200))
        elif kind == 2:  # literals incl. full 64-bit unsigned patterns
            k = int(rng.integers(1, 300))
            if signed:
                out += [int(x) for x in rng.integers(-(1 << 62), 1 << 62, size=k)]
            else:
                out += [int(x) for x in rng.integers(-(1 << 63), (1 << 63) - 1, size=k, dtype=np.int64)]
        else:
            out += [int(x) for x in rng.integers(0, 10, size=int(rng.integers(1, 20)))]
    return np.array(out[:n], dtype=np.int64)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("signed", [False, True])
def test_rle(covt, oracle, gpu_available, seed, signed):
    rng = np.random.default_rng(200 + seed)
    D = covt.DecodingUtils
    n = int(rng.integers(0, 20000))
    vals = _rle_values(rng, n, signed)
    enc = oracle.encode_rle(vals, signed)
    buf = b"\x07\x01" + enc + b"\x00" * 3
    ora = oracle.decode_rle(buf, n, 2, signed)
    assert ora[0] == 0 and np.array_equal(ora[1], vals) and ora[2] == 2 + len(enc) == 2 + ora[3]
    _check(_call(D, covt, "decodeRle", buf, n, 2, signed, pos_index=2), ora)
    # truncated stream: both must fail (EOF) -- the buffer ends inside the stream
    if len(enc) > 4:
        cut = buf[:2 + len(enc) // 2]
        ora = oracle.decode_rle(cut, n, 2, signed)
        _check(_call(D, covt, "decodeRle", cut, n, 2, signed, pos_index=2), ora)


@pytest.mark.parametrize("seed", range(6))
def test_byte_rle(covt, oracle, gpu_available, seed):
    rng = np.random.default_rng(300 + seed)
    D = covt.DecodingUtils
    parts = []
    while sum(len(p) for p in parts) < 5000:
        if rng.random() < 0.5:
            parts.append(np.full(int(rng.integers(1, 400)), rng.integers(0, 256), dtype=np.uint8))
        else:
            parts.append(rng.integers(0, 256, size=int(rng.integers(1, 300))).astype(np.uint8))
    vals = np.concatenate(parts)
    n = int(rng.integers(0, vals.size + 1))
    vals = vals[:n]
    enc = oracle.encode_byte_rle(vals)
    buf = b"\xaa" + enc + b"\x00"
    ora = oracle.decode_byte_rle(buf, n, 1, len(enc))
    assert ora[0] == 0 and np.array_equal(ora[1], vals)
    _check(_call(D, covt, "decodeByteRle", buf, n, 1, len(enc), pos_index=2), ora)


def _fpf_values(rng, n):
    """Blocks with various bit widths and outliers (exception index 1 and >1)."""
    v = np.zeros(n, dtype=np.uint64)
    i = 0
    while i < n:
        k = min(n - i, int(rng.integers(1, 700)))
        b = int(rng.integers(0, 33))
        hi = (1 << b) if b < 32 else (1 << 32)
        blk = rng.integers(0, max(hi, 1), size=k, dtype=np.uint64)
        if rng.random() < 0.5:  # outliers -> exceptions
            m = rng.random(k) < rng.random() * 0.2
            blk[m] = rng.integers(0, 1 << 32, size=int(m.sum()), dtype=np.uint64)
        if rng.random() < 0.3:  # exactly one extra bit -> exception index 1
            m = rng.random(k) < 0.05
            blk[m] |= np.uint64(1 << min(b, 31))
        v[i:i + k] = blk
        i += k
    return (v & np.uint64(0xFFFFFFFF)).astype(np.uint32)


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 1000, 4096 + 77, 65536, 65536 + 256 + 13, 140000])
def test_fastpfor(covt, oracle, gpu_available, n):
    rng = np.random.default_rng(n)
    D = covt.DecodingUtils
    raw = _fpf_values(rng, n)
    enc = oracle.encode_fastpfor(raw)
    st, dec, cnt = oracle.fastpfor_uncompress(enc, 0, len(enc), n)
    assert st == 0 and cnt == n and np.array_equal(dec, raw)
    buf = b"\x01\x02\x03" + enc + b"\x09" * 5  # unaligned start
    bl = len(enc)
    for name, ora in (
        ("decodeFastPfor128ZigZagDelta", oracle.decode_fastpfor_zigzag_delta(buf, n, bl, 3)),
        ("decodeFastPfor128DeltaCoordinates", oracle.decode_fastpfor_delta_coordinates(buf, n, bl, 3)),
    ):
        _check(_call(D, covt, name, buf, n, bl, 3, pos_index=3), ora)
    for nb in (13, 14, 20):
        _check(_call(D, covt, "decodeFastPfor128DeltaMortonCodes", buf, n, bl, 3, nb, pos_index=3),
               oracle.decode_fastpfor_delta_morton_codes(buf, n, bl, 3, nb))


def test_fastpfor_degenerate(covt, oracle, gpu_available):
    D = covt.DecodingUtils
    # byteLength 0 with numValues > 0: Java leaves decompressedValues zero-filled
    for name, ora in (("decodeFastPfor128ZigZagDelta", oracle.decode_fastpfor_zigzag_delta(b"", 5, 0, 0)),):
        _check(_call(D, covt, name, b"", 5, 0, 0, pos_index=3), ora)
    _check(_call(D, covt, "decodeFastPfor128DeltaMortonCodes", b"", 3, 0, 0, 14, pos_index=3),
           oracle.decode_fastpfor_delta_morton_codes(b"", 3, 0, 0, 14))
    # fewer values coded than numValues (VByte tail short) -> zero tail
    enc = oracle.encode_fastpfor(np.arange(300, dtype=np.uint32))
    _check(_call(D, covt, "decodeFastPfor128ZigZagDelta", enc, 310, len(enc), 0, pos_index=3),
           oracle.decode_fastpfor_zigzag_delta(enc, 310, len(enc), 0))
    # more values coded than numValues -> ArrayIndexOutOfBounds in Java
    _check(_call(D, covt, "decodeFastPfor128ZigZagDelta", enc, 290, len(enc), 0, pos_index=3),
           oracle.decode_fastpfor_zigzag_delta(enc, 290, len(enc), 0))
    # byteLength past the end of the buffer: Arrays.copyOfRange zero-pads
    _check(_call(D, covt, "decodeFastPfor128ZigZagDelta", enc[:-8], 300, len(enc), 0, pos_index=3),
           oracle.decode_fastpfor_zigzag_delta(enc[:-8], 300, len(enc), 0))


@pytest.mark.parametrize("seed", range(4))
def test_fastpfor_corrupt_headers_fail_cleanly(covt, oracle, gpu_available, seed):
    """Bit-flipped FastPFOR payloads: the GPU must return a status (never fault), and agree with the
    oracle whenever the oracle decodes successfully."""
    rng = np.random.default_rng(900 + seed)
    D = covt.DecodingUtils
    raw = _fpf_values(rng, 3000)
    enc = bytearray(oracle.encode_fastpfor(raw))
    for _ in range(20):
        e = bytearray(enc)
        for _ in range(int(rng.integers(1, 4))):
            e[int(rng.integers(0, len(e)))] ^= 1 << int(rng.integers(0, 8))
        e = bytes(e)
        ora = oracle.decode_fastpfor_zigzag_delta(e, 3000, len(e), 0)
        try:
            vals, pos = _call(D, covt, "decodeFastPfor128ZigZagDelta", e, 3000, len(e), 0, pos_index=3)()
            ok = True
        except Exception:  # noqa: BLE001
            ok = False
        if ora[0] == 0:
            assert ok and np.array_equal(vals, ora[1])
