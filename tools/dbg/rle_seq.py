"""Debug: replay test_rle_streams_split[64]; on the first mismatch relaunch the case (multi-chunk and
one-chunk-per-stream) and print per-chunk statuses."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import load_covt  # noqa: E402
import oracle  # noqa: E402
from test_gpu_split import DESC, _rle_chunks, _rle_values  # noqa: E402

covt = load_covt()
unit = 64
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
    bad[int(n * 0.9)] = 9
    cases.append((covt.OP_BYTE_RLE_U8, oracle.encode_byte_rle(bad), n, 1))
dev = torch.device("cuda")


def launch(op, buf, n, elem, ch, consumed, multi):
    d = np.zeros(len(ch) * covt.SPLIT_SLOTS, dtype=DESC)
    for c, (s0, e0, v0, nv) in enumerate(ch):
        k = c * covt.SPLIT_SLOTS
        d[k] = (0, 0, c if multi else 0, n, op, 0, covt.DESC_SPLIT | covt.DESC_SPLIT_RLE, len(buf))
        d[k + 1: k + covt.SPLIT_SLOTS]["flags"] = covt.DESC_SPLIT_PAD | covt.DESC_SPLIT_RLE
        d[k + 1]["in_off"], d[k + 1]["out_off"] = s0, e0
        d[k + 2]["in_off"], d[k + 2]["out_off"] = v0, nv
        d[k + 3]["in_off"] = consumed
    counts = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
    counts[covt.FAMILY_SPLIT_RLE] = d.size
    d_in = torch.zeros(len(buf) + covt.INPUT_PADDING + 16, dtype=torch.uint8, device=dev)
    d_in[:len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    d_desc = torch.from_numpy(d.view(np.uint8)).to(dev)
    d_out = torch.full((n * elem + 32,), 0x5A, dtype=torch.uint8, device=dev)
    d_res = torch.full((d.size * 2,), 0x33, dtype=torch.int32, device=dev)
    st = covt.lib().covt_decode_streams_device_grouped(d_in.data_ptr(), d_desc.data_ptr(),
                                                       counts.ctypes.data_as(C.POINTER(C.c_int64)), d_out.data_ptr(),
                                                       d_res.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert st == 0
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), d_res.cpu().numpy().reshape(-1, 8, 2)


for ci, (op, buf, total, elem) in enumerate(cases):
    byte_rle = op in (covt.OP_BYTE_RLE_U8, covt.OP_BYTE_RLE_RAW)
    for n in (total, total - 1, total // 3 + 1):
        w = _rle_chunks(buf, n, byte_rle, elem, unit)
        if w is None or len(w[0]) < 2:
            continue
        ch, consumed = w
        out, r = launch(op, buf, n, elem, ch, consumed, True)
        if byte_rle:
            o = oracle.decode_byte_rle(buf, n, 0, len(buf))
        else:
            o = oracle.decode_rle(buf, n, 0, op == covt.OP_RLE_S64)
        ok = (int(r[0, 0, 0]) == 0) == (o[0] == 0) or (op == covt.OP_BYTE_RLE_U8)
        print(ci, op, n, "chunks", len(ch), "status", r[0, 0], "oracle", o[0], o[3], "OK" if ok else "MISMATCH", flush=True)
        if not ok:
            out2, r2 = launch(op, buf, n, elem, ch, consumed, True)
            print("  relaunch multi status", r2[0, 0])
            out3, r3 = launch(op, buf, n, elem, ch, consumed, False)
            badc = np.nonzero(r3[:, 0, 0] != 0)[0]
            print("  one-chunk streams failing:", badc[:10], r3[badc[:10], 0])
            for c in badc[:4]:
                print("   ", c, ch[c], buf[ch[c][0]:ch[c][1]][:48].hex())
            sys.exit(1)
