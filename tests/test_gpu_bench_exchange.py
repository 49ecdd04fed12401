"""The exact N-rank step bench.py runs, rehearsed with one rank on the GPU box.

`python -m torch.distributed.run --nproc-per-node 1 bench.py --exchange` takes bench.py's distributed
branch (RCCL process group, the handle on torch's stream, dist.FrameExchange's double-buffered gather, the
rank-0 assembly with gvrt_unpack_tiles_rgba8) with WORLD_SIZE = 1; the frame rank 0 holds afterwards must be
the single-GPU frame bit for bit (the printed frame_sha1 of view 0), for the view split and the tile split.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--gpus", "1", "--steps", "3", "--warmup", "1", "--no-pmc", "--no-cpu-baseline", "--no-stats", "--no-configs"]


def _bench(args, distributed):
    sys.path.insert(0, ROOT)
    from importlib import import_module
    port = import_module("3dgvrt_lightfield_amd.dist").free_port()
    if distributed:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py", "--exchange", *COMMON, *args]
    else:
        cmd = [sys.executable, "bench.py", *COMMON, *args]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("split,strong", [("views", "bicycle"), ("tiles", "bicycle,truck")])
def test_bench_exchange_step_matches_single_gpu(split, strong):
    """Also the N-rank line's strong-scaling sub-records: the bicycle 1080p frame (and the truck 4K
    frame) tile-split in cost bands through the exact-size exchange, per-rank kernel / exchange / assembly times,
    the exchanged bytes, and the assembled frame equal to rank 0's one-GPU frame."""
    args = ["--config", "bicycle", "--split", split]
    one = _bench(args + ["--strong", "none"], distributed=False)
    ex = _bench(args + ["--strong", strong], distributed=True)
    assert one["frame_sha1"] and ex["frame_sha1"] == one["frame_sha1"], (ex["frame_sha1"], one["frame_sha1"])
    assert ex["n_gpus"] == 1 and ex["config"]["split"] == split
    assert ex["value"] > 0 and ex["ms_per_step"] > 0
    recs = ex["strong_scaling"]
    assert [r["frame"].split()[0] for r in recs] == strong.split(",")
    for r in recs:
        assert r["identical_to_one_gpu"] is True, r
        assert r["ranks"] == 1 and r["layout"] == "cost-bands" and r["ms_per_frame"] > 0 and r["mrays"] > 0
        assert len(r["kernel_ms_per_rank"]) == len(r["exchange_ms_per_rank"]) == 1 and r["kernel_ms_per_rank"][0] > 0
        assert r["exchange_bytes"] == 0 and r["bytes_sent_per_rank"][0] == r["tiles_per_rank"][0] * 256
        assert r["one_gpu_kernel_ms"] > 0 and r["assemble_ms"] >= 0
        assert r["wall_s"] > 0  # each sub-record reports its own wall time


def test_bench_exchange_strong_budget_prints_partial_line():
    """A strong-scaling sub-record starts only within the run's wall-time budget (--strong-budget-s): past it the
    line still prints, the records listed as skipped (an 8-rank run must not run past the driver's
    timeout for lack of a line)."""
    ex = _bench(["--config", "bicycle", "--split", "views", "--strong", "bicycle,truck", "--strong-budget-s", "0"],
                distributed=True)
    assert ex["value"] > 0
    assert [r["frame"] for r in ex["strong_scaling"]] == ["bicycle", "truck"]
    assert all("skipped" in r for r in ex["strong_scaling"])
