"""Parity of exactly the launches bench.py times for BASELINE configs 2-4 (bench.config_launch: the
config's fixture tiles planned with the default options -- so the long streams of these small batches
are split into chunks -- and one DeviceSubset launch over the config's streams).  Every selected
stream's output SHA-256, status and consumed bytes must equal the oracle digest of its source tile
(tests/golden/oracle_streams.json, pinned by the reference's fixtures and MVT originals); streams the
subset does not select must not be written.  The subset is launched twice (the split look-back records
are reset per launch).  Reference: CovtParser.java:392-511 (geometry), :552-572 (ids)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["config2", "config3", "config4"])
def test_config_launch_matches_oracle(covt, gpu_available, golden_streams, name):
    import torch

    import bench

    lib = bench.tile_library()
    picks, plan, mask, batch, sub = bench.config_launch(lib, name, covt, "cuda")
    assert sub.num_streams == int(mask.sum()) > 0
    if name != "config2":  # the small batches split their long poles (the path the legs time)
        assert plan.family_counts[covt.FAMILY_SPLIT:].sum() > 0
    batch.d_out.fill_(0xA5)  # sentinel: bytes no selected stream owns must stay untouched
    for _ in range(2):
        sub.decode()
    torch.cuda.synchronize()
    out, res, idx = sub.results()
    assert sorted(idx.tolist()) == sorted(np.nonzero(mask)[0].tolist())
    col = golden_streams["columns"]
    ish, ist, ico = col.index("fmt_sha256"), col.index("fmt_status"), col.index("fmt_consumed")
    st = plan.streams
    rows = {}
    for t, (key, _) in enumerate(picks):
        rec = golden_streams["tiles"][key]
        assert rec["walk_status"] == 0, key
        for i, row in zip(np.nonzero(st["tile"] == t)[0], rec["streams"]):
            rows[int(i)] = (key, row)
    checked = 0
    for r, i in zip(res, idx):
        key, row = rows[int(i)]
        assert int(r[0]) == row[ist] and row[ist] == 0, (name, key, int(i), int(r[0]))
        assert int(r[1]) == row[ico], (name, key, int(i))
        assert hashlib.sha256(plan.stream_array(out, int(i)).tobytes()).hexdigest() == row[ish], (name, key, int(i))
        checked += 1
    assert checked == int(mask.sum())
    # streams outside the subset: their output slices still hold the sentinel
    for i in np.nonzero(~mask)[0][:200]:
        a = plan.stream_array(out, int(i))
        assert (a.view(np.uint8) == 0xA5).all(), (name, int(i))
