"""The two FastPFOR family kernels (include/covt.h COVT_LAUNCH_FPF_STREAM / _CLASSIC) must agree bit for bit:
values, statuses and consumed positions, on every fixture tile in both Id modes and on a synthetic batch of
FastPFOR streams (exceptions of index 1 and > 1, all bit widths, multi-page, VByte tails, zero-filled and
over-long value counts, corrupted payloads); the synthetic streams that the oracle decodes are also checked
against it (DecodingUtils.java:316-409).  The automatic choice (covt_internal.h kFpfStreamMinStreams) only picks
between these two, so both must stay parity-green whatever the batch size."""
import ctypes as C

import numpy as np
import pytest

from conftest import tile_paths
from test_gpu_split import DESC
from test_gpu_synthetic import _fpf_values

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("id_mode", [0, 1], ids=["id_format", "id_java"])
def test_fixture_tiles_both_fpf_kernels(covt, gpu_available, id_mode):
    import torch

    tiles = [open(p, "rb").read() for p in tile_paths()]
    plan = covt.Plan.from_tiles(tiles, covt.FORMAT_GENC, id_mode)
    assert plan.family_counts[covt.FAMILY_FASTPFOR] > 100
    db = covt.DeviceBatch(plan, "cuda")
    got = []
    for v in (covt.LAUNCH_FPF_STREAM, covt.LAUNCH_FPF_CLASSIC):
        db.d_out.fill_(0x5A)
        db.d_res.fill_(0x33)
        db.decode(launch=covt.LAUNCH_FORKED | v)
        torch.cuda.synchronize()
        got.append(db.results())
    (o1, r1), (o2, r2) = got
    assert np.array_equal(r1, r2)
    assert np.array_equal(o1, o2)
    assert np.array_equal(r1, plan.decode_host()[1])


def test_launch_mode_validation(covt, gpu_available):
    tiles = [open(p, "rb").read() for p in tile_paths()[:2]]
    db = covt.DeviceBatch(covt.Plan.from_tiles(tiles, covt.FORMAT_GENC, 0), "cuda")
    with pytest.raises(Exception):
        db.decode(launch=covt.LAUNCH_FORKED | covt.LAUNCH_FPF_STREAM | covt.LAUNCH_FPF_CLASSIC)


def _synthetic_batch(covt, oracle, rng):
    """(input bytes, descs in launch order, output bytes, (oracle result, elements, corrupted) per desc)."""
    ops = (covt.OP_FPF_ZZ_DELTA_I32, covt.OP_FPF_ZZ_DELTA_XY, covt.OP_FPF_DELTA_MORTON)
    blob, descs, ora = bytearray(), [], []
    out_off = 0
    sizes = [0, 1, 255, 256, 257, 1000, 4096 + 77, 65536, 65536 + 256 + 13, 140000] + \
        [int(x) for x in rng.integers(1, 20000, size=40)]
    for i, n in enumerate(sizes):
        raw = _fpf_values(rng, n)
        enc = bytearray(oracle.encode_fastpfor(raw))
        if i % 7 == 6 and len(enc) > 8:  # corrupted payload
            for _ in range(int(rng.integers(1, 4))):
                enc[int(rng.integers(0, len(enc)))] ^= 1 << int(rng.integers(0, 8))
        enc = bytes(enc)
        op = ops[i % 3]
        nb = 14 if op == covt.OP_FPF_DELTA_MORTON else 0
        nv = n + (10 if i % 5 == 4 else 0) - (3 if i % 11 == 10 and n > 3 else 0)
        if op == covt.OP_FPF_ZZ_DELTA_XY:
            nv -= nv & 1
        ne = 2 * nv if nb else nv
        while len(blob) % 16:
            blob.append(0)
        descs.append((len(blob), out_off, len(enc), nv, op, nb, 0, len(enc)))
        blob += enc
        out_off += (4 * ne + 127) // 128 * 128
        if op == covt.OP_FPF_ZZ_DELTA_I32:
            o = oracle.decode_fastpfor_zigzag_delta(enc, nv, len(enc), 0)
        elif op == covt.OP_FPF_ZZ_DELTA_XY:
            o = oracle.decode_fastpfor_delta_coordinates(enc, nv, len(enc), 0)
        else:
            o = oracle.decode_fastpfor_delta_morton_codes(enc, nv, len(enc), 0, nb)
        ora.append((o, ne, i % 7 == 6))
    # largest stream first, as the plan orders a family
    order = sorted(range(len(descs)), key=lambda k: -descs[k][2])
    d = np.array([descs[k] for k in order], dtype=DESC)
    return bytes(blob), d, out_off, [ora[k] for k in order]


@pytest.mark.parametrize("seed", range(3))
def test_synthetic_batch_both_fpf_kernels(covt, oracle, gpu_available, seed):
    import torch

    rng = np.random.default_rng(4242 + seed)
    blob, d, out_bytes, ora = _synthetic_batch(covt, oracle, rng)
    counts = np.zeros(covt.NUM_FAMILIES, dtype=np.int64)
    counts[covt.FAMILY_FASTPFOR] = d.size
    dev = torch.device("cuda")
    d_in = torch.zeros(len(blob) + covt.INPUT_PADDING + 16, dtype=torch.uint8, device=dev)
    d_in[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    d_desc = torch.from_numpy(d.view(np.uint8)).to(dev)
    got = []
    for v in (covt.LAUNCH_FPF_STREAM, covt.LAUNCH_FPF_CLASSIC):
        d_out = torch.full((out_bytes + 16,), 0x5A, dtype=torch.uint8, device=dev)
        d_res = torch.full((d.size * 2,), 0x33, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream()
        st = covt.lib().covt_decode_streams_device_grouped_mode(
            d_in.data_ptr(), d_desc.data_ptr(), counts.ctypes.data_as(C.POINTER(C.c_int64)), d_out.data_ptr(),
            d_res.data_ptr(), s.cuda_stream, covt.LAUNCH_FORKED | v)
        assert st == 0
        torch.cuda.synchronize()
        got.append((d_out.cpu().numpy(), d_res.cpu().numpy().reshape(-1, 2)))
    (o1, r1), (o2, r2) = got
    assert np.array_equal(r1, r2)
    assert np.array_equal(o1, o2)
    n_ok = n_bad = 0
    for k, ((o, ne, corrupt), row) in enumerate(zip(ora, d)):
        if not corrupt:  # a corrupted payload: any status, equal values whenever the oracle decodes
            assert (int(r1[k, 0]) == 0) == (o[0] == 0), (k, int(r1[k, 0]), o[0])
        if o[0] != 0:
            n_bad += 1
            continue
        n_ok += 1
        assert int(r1[k, 0]) == 0, k
        assert int(r1[k, 1]) == int(row["byte_length"])
        off = int(row["out_off"])
        assert np.array_equal(o1[off:off + 4 * ne].view(np.int32), np.asarray(o[1], dtype=np.int32)), k
    assert n_ok > 30 and n_bad >= 1
