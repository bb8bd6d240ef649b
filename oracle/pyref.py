"""TEST INFRASTRUCTURE ONLY -- a second, pure-Python restatement of the reference path, written
independently of covt_oracle.c and used to cross-check it on small inputs (pure-Python loops:
small cases only).  Java semantics throughout (int32 wrap, >>> logical shift).

Sources followed (reference paths relative to /root/reference):
  evaluation/java/src/main/java/com/covt/decoder/DecodingUtils.java:35-444
  evaluation/java/src/main/java/com/covt/converter/GeometryUtils.java:34-47
  orc-core 1.8.1 RunLengthIntegerReader / RunLengthByteReader
  JavaFastPFOR 0.1.12 FastPFOR + VariableByte
"""
from __future__ import annotations

M32 = 0xFFFFFFFF


def i32(x: int) -> int:
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


def i64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


class Truncated(Exception):
    pass


def _b(src, o):
    if o < 0 or o >= len(src):
        raise Truncated(o)
    return src[o]


def varint_java(src, pos):
    """DecodingUtils.java:157-186 -> (value, new_pos)"""
    v = 0
    for i in range(4):
        b = _b(src, pos)
        pos += 1
        v |= (b & 0x7F) << (7 * i)
        if i < 3 and not (b & 0x80):
            break
    return i32(v), pos


def zigzag(e: int) -> int:
    e &= M32
    return i32((e >> 1) ^ (-(e & 1) & M32))


def decode_varint(src, pos, n):
    out = []
    for _ in range(n):
        v, pos = varint_java(src, pos)
        out.append(v)
    return out, pos


def decode_zigzag_delta_varint(src, pos, n):
    out, prev = [], 0
    for _ in range(n):
        v, pos = varint_java(src, pos)
        prev = i32(prev + zigzag(v))
        out.append(prev)
    return out, pos


def decode_zigzag_delta_varint_coordinates(src, pos, n):
    out, px, py = [0] * n, 0, 0
    for i in range(0, n, 2):
        dx, pos = varint_java(src, pos)
        dy, pos = varint_java(src, pos)
        px, py = i32(px + zigzag(dx)), i32(py + zigzag(dy))
        out[i] = px
        out[i + 1] = py
    return out, pos


def morton(code: int, nb: int):
    te = i32(2 << ((nb - 2) & 31))
    half = int(te / 2)  # Java int division truncates toward zero

    def axis(c):
        coord = 0
        for i in range(nb):
            bit = c & (1 << ((2 * i) & 63))  # Python ints are sign-extended like Java long
            coord = i32(coord | (bit >> (i & 63)))
        return coord

    return i32(axis(code) - half), i32(axis(code >> 1) - half)


def decode_delta_varint_morton_codes(src, pos, n, nb):
    out, prev = [], 0
    for _ in range(n):
        d, pos = varint_java(src, pos)
        prev = i32(prev + d)
        out += list(morton(prev, nb))
    return out, pos


def _vulong(src, o):
    r, sh = 0, 0
    while True:
        b = _b(src, o)
        o += 1
        r |= (b & 0x7F) << (sh & 63)
        sh += 7
        if b < 0x80:
            return r & ((1 << 64) - 1), o


def decode_rle(src, n, pos, signed):
    """ORC RLE v1 integer reader -> (values, consumed_end)"""
    out, o = [], pos
    while len(out) < n:
        c = _b(src, o)
        o += 1
        if c < 0x80:
            cnt = c + 3
            d = _b(src, o)
            o += 1
            d = d - 256 if d > 127 else d
            base, o = _vulong(src, o)
            base = i64((base >> 1) ^ -(base & 1)) if signed else i64(base)
            for i in range(cnt):
                if len(out) < n:
                    out.append(i64(base + i * d))
        else:
            for _ in range(256 - c):
                v, o = _vulong(src, o)
                v = i64((v >> 1) ^ -(v & 1)) if signed else i64(v)
                if len(out) < n:
                    out.append(v)
    return out, o


def decode_byte_rle(src, n, pos):
    out, o = [], pos
    while len(out) < n:
        c = _b(src, o)
        o += 1
        if c < 0x80:
            v = _b(src, o)
            o += 1
            out += [v] * min(c + 3, n - len(out))
        else:
            k = 256 - c
            if o + k > len(src):
                raise Truncated(o)
            out += list(src[o:o + min(k, n - len(out))])
            o += k
    return out, o


def fastpfor_uncompress(src, pos, byte_length, n):
    """Composition(FastPFOR, VariableByte) over big-endian words -> (raw uint32 list, decoded count)."""
    nw = byte_length // 4
    data = bytes(src[pos:pos + 4 * nw]).ljust(4 * nw, b"\x00")
    W = [int.from_bytes(data[4 * i:4 * i + 4], "big") for i in range(nw)]
    out = [0] * n
    if nw == 0:
        return out, 0

    def wget(i):
        return W[i] if 0 <= i < nw else 0

    def unpack(base, r, b):
        if b == 0:
            return 0
        bit = r * b
        wi, off = base + (bit >> 5), bit & 31
        cat = wget(wi) | (wget(wi + 1) << 32)
        return (cat >> off) & ((1 << b) - 1)

    L = i32(W[0])
    assert L >= 0
    L -= L % 256
    assert L <= n
    p, done = 1, 0
    while done < L:
        ts = min(65536, L - done)
        p0 = p
        ie = p0 + i32(W[p0])
        bytesize = W[ie]
        ie += 1
        bcw = (bytesize + 3) // 4
        container = b"".join(W[ie + k].to_bytes(4, "little") for k in range(bcw))
        ie += bcw
        bitmap = W[ie]
        ie += 1
        xs = {}
        for k in range(2, 33):
            if bitmap & (1 << (k - 1)):
                size = W[ie]
                ie += 1
                groups = (size + 31) // 32
                xs[k] = [unpack(ie + (i // 32) * k, i % 32, k) for i in range(size)]
                ie += groups * k - ((groups * 32 - size) * k) // 32
        ptr = {k: 0 for k in xs}
        bc, pk = 0, p0 + 1
        for run in range(ts // 256):
            b = container[bc]
            b = b - 256 if b > 127 else b
            ce = container[bc + 1]
            bc += 2
            base = done + run * 256
            for mb in range(8):
                for r in range(32):
                    out[base + mb * 32 + r] = unpack(pk, r, b)
                pk += b
            if ce:
                mbits = container[bc]
                bc += 1
                idx = mbits - b
                for _ in range(ce):
                    q = container[bc]
                    bc += 1
                    ex = 1 if idx == 1 else xs[idx][ptr[idx]]
                    if idx != 1:
                        ptr[idx] += 1
                    out[base + q] = (out[base + q] | (ex << (b & 31))) & M32
        done += ts
        p = ie
    # VariableByte tail: LE bytes of the remaining words, terminator bit set
    outpos, v, shift = L, 0, 0
    for q in range(p, nw):
        for k in range(4):
            c = (W[q] >> (8 * k)) & 0xFF
            v = (v + ((c & 127) << (shift & 31))) & M32
            if c & 128:
                out[outpos] = v
                outpos += 1
                v, shift = 0, 0
            else:
                shift += 7
    return out, outpos


def decode_fastpfor_zigzag_delta(src, n, byte_length, pos):
    raw, _ = fastpfor_uncompress(src, pos, byte_length, n)
    out, prev = [], 0
    for x in raw:
        prev = i32(prev + zigzag(x))
        out.append(prev)
    return out, pos + byte_length


def decode_fastpfor_delta_coordinates(src, n, byte_length, pos):
    raw, _ = fastpfor_uncompress(src, pos, byte_length, n)
    out, px, py = [0] * n, 0, 0
    for i in range(0, n, 2):
        px, py = i32(px + zigzag(raw[i])), i32(py + zigzag(raw[i + 1]))
        out[i], out[i + 1] = px, py
    return out, pos + byte_length


def decode_fastpfor_delta_morton_codes(src, n, byte_length, pos, nb):
    raw, _ = fastpfor_uncompress(src, pos, byte_length, n)
    out, prev = [], 0
    for x in raw:
        prev = i32(prev + x)
        out += list(morton(prev, nb))
    return out, pos + byte_length
