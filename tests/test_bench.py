"""bench.py contract on CPU: the N-rank launch (--gpus N spawns N processes, gloo aggregation), the
GPU-count check, the BASELINE config 2-4 stream selections and the CPU-baseline leg."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


def test_gpus2_dry_run_spawns_two_ranks():
    p, lines = _run(["--gpus", "2", "--dry-run", "--tiles", "40", "--steps", "2", "--warmup", "1", "--cpu-iters", "2",
                     "--scaling", "weak"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dry_run"] and line["scaling"] == "weak"
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert len({r["seed"] for r in pr}) == 2  # weak scaling: distinct per-rank batches
    assert all(r["tiles"] == 40 for r in pr)
    assert line["config"]["parallelism"].startswith("dp2")
    assert "weak" not in line  # the weak figure is the headline here
    cb = line["cpu_baseline"]  # rank 0's batch, at every N (north_star: "next to the Java CPU decoder ... in the same run")
    assert cb is not None and cb["value"] > 0 and cb["kind"] == "port"
    # N > 1 field semantics: byte totals are sums over ranks, each rank's own beside them;
    # roofline is per GPU (the slowest rank's own bytes over its own time) with the aggregate against N peaks
    cfg = line["config"]
    assert cfg["stream_bytes_total"] == sum(r["stream_bytes"] for r in pr)
    assert cfg["output_bytes_total"] == sum(r["output_bytes"] for r in pr)
    assert cfg["streams_total"] == sum(r["streams"] for r in pr) and cfg["tiles_total"] == 80
    assert cfg["stream_bytes_per_gpu"] == pr[0]["stream_bytes"]
    assert pr[0]["stream_bytes"] != pr[1]["stream_bytes"]  # distinct batches
    rf = line["roofline"]
    # the slowest rank, by the rounded per-rank fracs: two ranks may round to the same figure
    fmin = min(r["roofline_frac"] for r in pr)
    slow = [r for r in pr if r["roofline_frac"] == fmin]
    assert rf["frac"] == fmin and rf["peak"] == 8000.0
    assert rf["algorithmic_bytes_per_launch"] in {r["stream_bytes"] + r["output_bytes"] for r in slow}
    agg = rf["aggregate"]
    assert agg["peak"] == 16000.0 and agg["algorithmic_bytes_per_launch"] == cfg["stream_bytes_total"] + \
        cfg["output_bytes_total"]
    assert rf["traffic"] is None  # the PMC figure is a one-GPU, one-batch measurement
    assert line["build"]["match"] and line["build"]["library"] == line["build"]["sources"]


def test_gpus2_default_is_strong_scaling():
    """BASELINE config 5 ("10k-tile batch ... sharded across 8xMI355X"): at N > 1
    the default shards ONE batch over the ranks by LPT byte balance; the weak figure rides beside it."""
    import bench

    p, lines = _run(["--gpus", "2", "--dry-run", "--tiles", "41", "--steps", "1", "--warmup", "0", "--no-cpu"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(lines[0])
    assert line["scaling"] == "strong" and "sharded over 2 GPUs" in line["config"]["workload"]
    pr = line["per_rank"]
    assert sum(r["tiles"] for r in pr) == 41 and len({r["seed"] for r in pr}) == 1
    assert line["config"]["tiles_total"] == 41
    # the shards are the LPT split of the one batch: their bytes add up to the whole batch's
    covt = bench.load_covt()
    allp = bench.sample_batch(bench.tile_library(), 41, bench.SEED)
    whole = covt.Plan.from_tiles([t for _, t in allp])
    assert line["config"]["stream_bytes_total"] == whole.in_bytes
    sh = bench.lpt_shards([len(t) for _, t in allp], 2)
    assert sorted(len(s) for s in sh) == sorted(r["tiles"] for r in pr)
    w = line["weak"]
    assert w["tiles_per_gpu"] == 41 and w["tiles_total"] == 82 and len(set(w["seeds"])) == 2
    assert w["value"] > 0


def test_gpus1_default_is_the_whole_batch():
    p, lines = _run(["--dry-run", "--tiles", "25", "--steps", "1", "--warmup", "0", "--no-cpu"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["per_rank"][0]["tiles"] == 25 and "weak" not in line


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="host has >= 2 GPUs")
def test_gpus2_fails_loudly_without_two_gpus():
    p, lines = _run(["--gpus", "2", "--tiles", "10", "--steps", "1"], timeout=120)
    assert p.returncode != 0 and not lines
    assert "GPU" in p.stderr


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


def test_config_selections_match_survey():
    """config 2 = 6 streams / 23,992 B / 137,864 B out; config 3 = 29 tiles, 1,104
    streams, 2,983,091 B; config 4 = 61 tiles, 787 streams, 722,977 B in, 5,167,832 B out."""
    import bench

    covt = bench.load_covt()
    lib = bench.tile_library()
    want = {"config2": (1, 6, 23992, 137864), "config3": (29, 1104, 2983091, 14096776),
            "config4": (61, 787, 722977, 5167832)}
    for name, (nt, ns, ib, ob) in want.items():
        picks = bench.config_tiles(lib, name)
        plan = covt.Plan.from_tiles([t for _, t in picks])
        m = bench.config_mask(plan, name)
        st = plan.streams[m]
        assert (len(picks), int(m.sum()), int(st["byte_length"].sum()),
                int((st["out_elems"] * st["elem_bytes"]).sum())) == (nt, ns, ib, ob), name
        descs, counts, idx = plan.subset_descs(m)
        assert counts.sum() == descs.size // 32 == idx.size  # split chunks + pads included
        assert sorted(idx[idx >= 0].tolist()) == sorted(map(int, m.nonzero()[0]))


def test_cpu_baseline_leg_uses_host_cpus():
    import bench

    p, lines = _run(["--dry-run", "--tiles", "30", "--steps", "1", "--warmup", "0", "--cpu-iters", "3"])
    assert p.returncode == 0, p.stderr[-2000:]
    cb = json.loads(lines[0])["cpu_baseline"]
    n, info = bench.host_cpus()
    assert cb["cores"] == n and cb["host"]["nproc"] == os.cpu_count()
    assert cb["kind"] == "port" and "full bench batch (30 tiles" in cb["sample"]
    assert cb["value"] > 0 and cb["value_1thread"] > 0
    assert "config1" not in cb  # merged into configs.config1 (absent in a dry run)


def test_config1_cpu_leg():
    """BASELINE configs[0]: the oracle decodes omt/5_16_20 whole (walk, 41 Id/Geometry streams, assembly,
    property columns) -- the figure the bench line puts beside the GPU's one-tile latency."""
    import bench

    sys.path.insert(0, ROOT)
    import oracle as O

    lib = bench.tile_library()
    t = bench.config1_tile(lib)
    st, cnt = O.decode_tile_full(t)
    assert st == 0 and cnt["streams"] == 41 and cnt["vertices"] == 19285 and cnt["property_columns"] > 0


def test_kernel_sources_fingerprint():
    """roofline.traffic comes from profiles/pmc_traffic.json only while it was measured on the same decode
    and plan sources: the fingerprint is a stable sha256 over bench.KERNEL_SOURCES."""
    import bench

    a, b = bench.kernel_sources_sha256(), bench.kernel_sources_sha256()
    assert a == b and len(a) == 64
    assert all(os.path.exists(os.path.join(bench.ROOT, p)) for p in bench.KERNEL_SOURCES)
