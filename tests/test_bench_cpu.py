"""bench.py's host logic without a GPU: the rank fan-out refuses more ranks
than visible GPUs (unless a gloo rehearsal is asked for) before any GPU call,
and --global-pop splits the population exactly (strong scaling)."""
import os
import pathlib
import subprocess
import sys
import types

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import bench  # noqa: E402


def test_rank_share_weak_and_strong():
    weak = types.SimpleNamespace(global_pop=0, pop=65536)
    assert [bench.rank_share(weak, r, 4) for r in range(4)] == [(65536, r * 65536, 4 * 65536) for r in range(4)]
    for world in (1, 2, 3, 4, 7, 8):
        strong = types.SimpleNamespace(global_pop=262144 + 5, pop=65536)
        parts = [bench.rank_share(strong, r, world) for r in range(world)]
        assert sum(p for p, _, _ in parts) == 262149
        assert all(g == 262149 for _, _, g in parts)
        # contiguous, non-overlapping shards in rank order
        assert [s for _, s, _ in parts] == [sum(p for p, _, _ in parts[:r]) for r in range(world)]
        assert max(p for p, _, _ in parts) - min(p for p, _, _ in parts) <= 1


def test_gpus_above_visible_fails_loudly():
    """No GPU here: --gpus 2 must fail with rc 2 from the parent (no rank started)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TTGA_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-pmc", "--no-cpu", "--steps", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr and r.stdout.strip() == ""


def test_global_pop_below_ranks_rejected():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--global-pop", "3"],
                       cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0 and "--global-pop" in r.stderr
