"""The real (non-dry-run) N-rank bench path on the one-GPU test box: `bench.py --gpus 2 --share-device`
spawns two ranks before anything touches the GPU, both decode their shard of one batch on cuda:0 (gloo
barriers, max-over-ranks timing; then each its own whole batch for the weak figure), and rank 0 prints one line with both ranks' kernel times and the CPU baseline
(north_star: every 1/2/4/8 figure next to the CPU decoder in the same run)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_share_device(gpu_available):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--tiles", "500", "--steps", "3", "--warmup", "1", "--no-props", "--no-assemble",
                        "--no-configs", "--e2e-reps", "0", "--abi-host-reps", "0", "--device-plan-reps", "0",
                        "--cpu-iters", "2"], capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["shared_device"] and "dry_run" not in line
    pr = line["per_rank"]
    # strong scaling (the default, BASELINE config 5): the ranks share ONE 500-tile batch by LPT shards
    assert [r["rank"] for r in pr] == [0, 1] and len({r["seed"] for r in pr}) == 1
    assert all(r["kernel_ms"] > 0 for r in pr) and sum(r["tiles"] for r in pr) == 500
    assert line["scaling"] == "strong" and line["config"]["tiles_total"] == 500
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    w = line["weak"]  # the weak figure beside it: each rank its own 500-tile batch
    assert w["tiles_per_gpu"] == 500 and w["tiles_total"] == 1000 and len(set(w["seeds"])) == 2 and w["value"] > 0
    cb = line["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] >= 1
