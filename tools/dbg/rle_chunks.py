"""Debug: every RLE chunk of a failing split case as its own one-chunk stream (own result entry)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import load_covt  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_split import DESC, _rle_chunks, _rle_values  # noqa: E402

covt = load_covt()
unit = 64
MULTI = len(sys.argv) > 1
rng = np.random.default_rng(unit)
for n in (3000, 20000):
    v = _rle_values(rng, n)
    buf = O.encode_rle(v, False)
    if n == 3000:  # advance the generator like the test
        _rle_values(rng, n, big=True)
        _rle_values(rng, n)
        _rle_values(rng, n)
        continue
    ch, consumed = _rle_chunks(buf, n, False, 8, unit)
    print("n", n, "bytes", len(buf), "chunks", len(ch))
    d = np.zeros(len(ch) * covt.SPLIT_SLOTS, dtype=DESC)
    for c, (s0, e0, v0, nv) in enumerate(ch):
        k = c * covt.SPLIT_SLOTS
        d[k] = (0, 0, c if MULTI else 0, n, covt.OP_RLE_U64, 0, covt.DESC_SPLIT | covt.DESC_SPLIT_RLE, len(buf))
        d[k + 1: k + covt.SPLIT_SLOTS]["flags"] = covt.DESC_SPLIT_PAD | covt.DESC_SPLIT_RLE
        d[k + 1]["in_off"], d[k + 1]["out_off"] = s0, e0
        d[k + 2]["in_off"], d[k + 2]["out_off"] = v0, nv
        d[k + 3]["in_off"] = consumed
    counts = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
    counts[covt.FAMILY_SPLIT_RLE] = d.size
    dev = torch.device("cuda")
    d_in = torch.zeros(len(buf) + covt.INPUT_PADDING + 16, dtype=torch.uint8, device=dev)
    d_in[:len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    d_desc = torch.from_numpy(d.view(np.uint8)).to(dev)
    d_out = torch.full((n * 8 + 32,), 0x5A, dtype=torch.uint8, device=dev)
    d_res = torch.full((d.size * 2,), 0x33, dtype=torch.int32, device=dev)
    st = covt.lib().covt_decode_streams_device_grouped(d_in.data_ptr(), d_desc.data_ptr(),
                                                       counts.ctypes.data_as(C.POINTER(C.c_int64)), d_out.data_ptr(),
                                                       d_res.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    r = d_res.cpu().numpy().reshape(-1, 8, 2)[:, 0, :]
    print("entry 0:", r[0], "MULTI", MULTI)
    bad = np.nonzero(r[:, 0] != 0)[0]
    print("failing chunks", len(bad), bad[:20])
    for c in bad[:6]:
        s0, e0, v0, nv = ch[c]
        print(c, (s0, e0, v0, nv), "sb mod 16", s0 % 16, "bytes", buf[s0:e0][:40].hex())
    o = O.decode_rle(buf, n, 0, False)
    got = d_out.cpu().numpy()[:n * 8].view(np.int64)
    print("values equal", np.array_equal(got, o[1]))
