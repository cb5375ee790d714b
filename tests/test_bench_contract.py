"""bench.py driver contract on CPU: launched the way the driver launches it (torch.distributed.run,
one process per rank, 127.0.0.1 rendezvous), rank 0 prints exactly one JSON line whose fields match
the world size. Uses gloo and the tiny model; the GPU run of the same code path is the driver's."""

import json
import os
import subprocess
import sys

import pytest

from cs336_systems.parallel.comm import find_free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(nproc: int, *extra: str) -> list[dict]:
    cmd = [
        sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
        "--master-addr", "127.0.0.1", f"--master-port={find_free_port()}",
        "bench.py", "--gpus", str(nproc), "--steps", "2", "--warmup", "1",
        "--model", "tiny", "--ctx", "32", "--batch", "2", "--dtype", "fp32", "--comm-sweep-mb", "1", "4",
        "--ddp-sweep", "on", *extra,
    ]
    env = dict(os.environ, CS336_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    return [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]


def _gpu_visible() -> bool:
    import torch

    return torch.cuda.device_count() > 0


@pytest.mark.parametrize(
    "nproc,extra",
    [(2, ()), (4, ()), (2, ("--sharded",)), (2, ("--ddp", "zero")), (2, ("--grad-comm-dtype", "bf16"))],
)
def test_bench_multirank_json(nproc, extra):
    lines = _run(nproc, *extra)
    assert len(lines) == 1, lines
    d = lines[0]
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in d
    assert d["n_gpus"] == nproc and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 2 * nproc
    assert d["config"]["parallelism"].startswith(f"dp{nproc}")
    assert d["value"] > 0 and d["ms_per_step"] > 0
    if not _gpu_visible():
        assert "HIP" not in d["config"]["attention"]  # CPU run must not claim the HIP kernels
    assert d["value"] == pytest.approx(2 * nproc * 32 / (d["ms_per_step"] / 1e3), rel=0.02)
    # multi-rank diagnostics (the 8-GPU run must be diagnosable from its own line)
    dd = d["dist"]
    assert dd["pg_world_size"] == nproc and dd["backend"] == "gloo"
    assert dd["comm_wait_ms"] >= 0
    assert dd["n_buckets"] == len(dd["bucket_sizes_mb"]) >= 1
    assert dd["bucket_mb"]["max"] <= 128.0 + 1e-6
    assert "rccl_version" in dd and isinstance(dd["env"], dict)
    # the handout's all-reduce table rides in the same line
    sw = dd["allreduce_sweep_fp32"]
    assert [r["size_mb"] for r in sw] == [1, 4]
    for r in sw:
        assert r["ms"] > 0 and r["algbw_gbs"] > 0
        assert r["busbw_gbs"] == pytest.approx(r["algbw_gbs"] * 2 * (nproc - 1) / nproc, rel=0.01)
    assert dd["coresidency_caps"] == {"TENSILE_STREAMK_MAX_CUS": "248"}  # no RCCL channel cap (rccl_env.py)
    # per-rank CPU affinity
    assert [a["rank"] for a in dd["cpu_affinity"]] == list(range(nproc))
    assert all("cpus" in a and "pinned" in a for a in dd["cpu_affinity"])
    # the handout's DDP-variant table + ZeRO-1 memory; not run under ZeRO-2
    if "zero" not in extra:
        rows = dd["ddp_variants"]
        assert [(r["variant"], r["bucket_mb"]) for r in rows] == [
            ("naive", None), ("flat", None), ("individual", None), ("bucketed", 1.0), ("bucketed", 10.0),
            ("bucketed", 100.0), ("bucketed", 1000.0)]
        for r in rows:
            assert "error" not in r, r
            assert r["ms_per_step"] > 0 and 0 <= r["comm_wait_ms"] <= r["ms_per_step"]
        zm = dd["zero1_memory"]
        assert set(zm["zero1"]) == {"after_init_mib", "peak_before_step_mib", "peak_after_step_mib"}
        assert dd["ddp_sweep"]["world"] == nproc and dd["ddp_sweep"]["wall_s"] < 120
    if "--grad-comm-dtype" in extra:
        assert d["config"]["grad_comm_dtype"] == "bf16" and dd["wire_dtype"] == "bfloat16"
        assert dd["wire_mb_total"] == pytest.approx(dd["bucket_mb"]["total"] / 2, rel=0.01)


def test_bench_ddp_sweep_watchdog():
    """A DDP sweep that outlives ``--ddp-sweep-timeout`` never costs the headline line: rank 0 prints it
    with the sweep marked failed and the job exits 0."""
    lines = _run(2, "--ddp-sweep-timeout", "0.05")
    assert len(lines) == 1, lines
    d = lines[0]
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "error" in d["dist"]["ddp_sweep"] and "ddp_variants" not in d["dist"]


def test_bench_self_launch_without_launcher():
    """``python bench.py --gpus 2`` with no torchrun and no WORLD_SIZE: bench.py launches the two
    ranks itself and reports n_gpus 2 (never a mislabeled 1-GPU number)."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--model", "tiny", "--ctx", "32",
           "--batch", "2", "--dtype", "fp32", "--comm-sweep-mb", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(CS336_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["config"]["parallelism"].startswith("dp2")


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", CS336_DIST_BACKEND="gloo")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--model", "tiny", "--steps", "1"], cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "WORLD_SIZE" in out.stderr


def test_train_applies_coresidency_env():
    """train.py sets the multi-rank co-residency env before torch loads, as bench.py does."""
    from cs336_systems.rccl_env import multi_gpu_env

    code = ("import os, sys, cs336_systems.train as t; "
            "print(sorted((k, os.environ.get(k)) for k in t._CORES_ENV), 'torch' in sys.modules)")
    env = {k: v for k, v in os.environ.items() if k not in ("TENSILE_STREAMK_MAX_CUS", "NCCL_MAX_NCHANNELS")}
    for ws, want in (("2", multi_gpu_env(2)), ("1", {})):
        env["WORLD_SIZE"] = ws
        out = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True,
                             timeout=120)
        assert out.returncode == 0, out.stderr[-2000:]
        assert out.stdout.split(" True")[0].strip() == str(sorted(want.items()))
