"""bench.py's multi-GPU launch path on CPU (gloo): `python bench.py --gpus N` without a torch.distributed
environment must start its N ranks itself (a torch.distributed.run child, before any GPU call), shard the
GLOBAL batch of BASELINE config 5 (65,536 trajectories) with shard_range, take the step time as the max
over ranks and print exactly one JSON line from rank 0 whose rank count comes from the process group.
--dry-run swaps the GPU step for a placeholder and RCCL for gloo; everything else is the bench's code."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--steps", "2", "--warmup", "1",
                        *args], capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 8])
def test_bench_self_launches_strong_scaling(n):
    d = _bench("--gpus", str(n))
    assert d["n_gpus"] == n
    assert d["scaling"] == "strong"
    assert d["config"]["global_batch"] == 65536
    assert d["config"]["batch_per_gpu"] == 65536 // n
    assert d["config"]["parallelism"] == f"dp{n}"
    # value = every rank's trajectories x 31 iterations / the slowest rank's step time
    assert abs(d["value"] - 65536 * 31 / (d["ms_per_step"] * 1e-3)) < 1e-6 * d["value"]
    # every rank reports itself: shard, kernel time, theta wait, wall time, overlap path, lanes
    ranks = d["ranks"]
    assert [r["rank"] for r in ranks] == list(range(n))
    assert sum(r["batch"] for r in ranks) == 65536 and all(r["batch"] == 65536 // n for r in ranks)
    for r in ranks:
        assert r["kernel_ms"] > 0 and r["theta_wait_ms"] >= 0 and r["wall_ms_per_step"] > 0
        assert r["overlap"] is False  # the dry run's placeholder step has no split launch
    assert d["kernel_ms_max_over_ranks"] == max(r["kernel_ms"] for r in ranks)
    assert d["comm"]["backend"] == "gloo" and "all_reduce" in d["comm"]["collective"]
    assert d["comm"]["theta_wait_ms_max_over_ranks"] == max(r["theta_wait_ms"] for r in ranks)
    # beside the strong-scaling line, the same step at 65,536 trajectories per GPU (weak scaling)
    w = d["weak_scaling"]
    assert w["batch_per_gpu"] == 65536 and w["global_batch"] == 65536 * n
    assert abs(w["value"] - 65536 * n * 31 / (w["ms_per_step"] * 1e-3)) < 1e-6 * w["value"]


def test_bench_weak_scaling_flag():
    d = _bench("--gpus", "2", "--weak", "--batch", "1000")
    assert d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 2000 and d["config"]["batch_per_gpu"] == 1000


def test_shard_range_covers_ragged_batches():
    sys.path.insert(0, os.path.join(REPO, "differentiable-tube-mpc_amd"))
    from diff_tube_mpc_strict_pt.core import shard_range

    for B in (65536, 65537, 4097, 8, 7):
        for W in (1, 2, 3, 4, 8):
            if B < W:
                continue
            parts = [shard_range(B, r, W) for r in range(W)]
            assert parts[0][0] == 0 and parts[-1][1] == B
            assert all(parts[r][1] == parts[r + 1][0] for r in range(W - 1))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= 1
