"""bench.py's contract (the driver's headline line): one JSON line with the
BASELINE metric, whole-job value, roofline and CPU baseline at N = 1, and the
N > 1 path (rehearsed with gloo ranks sharing the GPU)."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = pathlib.Path(__file__).resolve().parent.parent
METRIC = json.loads((REPO / "BASELINE.json").read_text())["metric"]


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_single_gpu_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "20", "--warmup", "2", "--no-pmc",
                        "--cpu-sample", "2048", "--cpu-seconds", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["metric"] == METRIC and d["unit"] == "evals/s" and d["n_gpus"] == 1 and d["steps"] == 20
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["pop_per_gpu"] == 65536 and d["config"]["kernel"] == "eval_tile5_w8"
    rl = d["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and 0 < rl["frac"] < 1
    assert abs(rl["achieved"] - rl["bytes_per_eval"] * 65536 / (rl["kernel_ms"] * 1e-3) / 1e9) < 1e-6 * rl["achieved"]
    cb = d["cpu_baseline"]
    assert cb["kind"] == "reference" or cb["kind"] == "port"
    assert cb["matches_gpu"] is True and cb["value"] > 0 and cb["cores"] >= 1


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_rehearsal():
    env = dict(os.environ, TTGA_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                        "--steps", "10", "--warmup", "2", "--no-pmc", "--no-cpu"],
                       cwd=REPO, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_pop"] == 2 * 65536 and d["value"] > 0
    assert "rehearsal" in d["config"] and "cpu_baseline" not in d
    _assert_ranks(d, 2, "gloo")


def test_bench_rccl_process_group_one_gpu():
    """TTGA_BENCH_FORCE_DIST=1: the nccl (RCCL) process group at world 1, so the
    timing barrier and the MAX all-reduce of the N > 1 path run through RCCL
    on a one-GPU box; the line is the N = 1 line."""
    env = dict(os.environ, TTGA_BENCH_FORCE_DIST="1")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "10", "--warmup", "2", "--no-pmc", "--no-cpu"],
                       cwd=REPO, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["process_group"].startswith("nccl")
    _assert_ranks(d, 1, "nccl")


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` with no launcher: the parent starts the two ranks
    itself (gloo rehearsal on a one-GPU box) and relays rank 0's line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["TTGA_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "10", "--warmup", "2",
                        "--no-pmc", "--no-cpu"], cwd=REPO, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_pop"] == 131072 and d["scaling"] == "weak" and d["value"] > 0
    _assert_ranks(d, 2, "gloo")
    # the launcher parent only starts and relays the ranks: no HIP runtime in it
    assert d["launcher"]["hip_mapped_before_launch"] is False and d["launcher"]["visible_gpus"] >= 1


def _assert_ranks(d, world, backend):
    """Every rank checked a strided sample of its shard against the oracle and
    reported the device it bound (gloo rehearsal: both ranks share the GPU)."""
    rk = d["ranks"]
    assert rk["world"] == world == d["n_gpus"] and rk["backend"] == backend
    assert rk["ranks_verified"] == world and rk["rows_checked"] >= 256 * world, rk
    pairs = {(x["rank"], x["device"]) for x in rk["devices"]}
    assert len(pairs) == world and sorted(r for r, _ in pairs) == list(range(world))
    assert all(x["matches_oracle"] and x["kernel_ms"] > 0 and x["pci"] for x in rk["devices"])


def test_bench_self_launch_global_pop_strong():
    """--global-pop splits one population across the ranks (BASELINE configs[4])."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["TTGA_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--global-pop", "65536", "--steps", "10",
                        "--warmup", "2", "--no-pmc", "--no-cpu"], cwd=REPO, capture_output=True, text=True,
                       timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_pop"] == 65536 and d["config"]["pop_per_gpu"] == 32768
    _assert_ranks(d, 2, "gloo")
