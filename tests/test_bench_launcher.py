"""bench.py --gpus N: the N-rank launcher (reference: slurm/train_multi_gpu.sh:26-42 runs one process per GPU
under torchrun; scripts/run.py:39-47 takes the device from LOCAL_RANK).

CPU tests: the per-rank environment, the WORLD_SIZE / --gpus mismatch refusal, the refusal when fewer GPUs are
visible than asked for, and that a failing rank makes the launcher exit non-zero.  The GPU rehearsal
(test_bench_two_ranks_one_gpu) runs the real bench with 2 gloo ranks on one card.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PZ_DEVICE", "PZ_RANKS_PER_GPU", "PZ_VISIBLE_GPUS")}
    e.update(kw)
    return e


def test_rank_envs():
    sys.path.insert(0, ROOT)
    import bench

    envs = bench.rank_envs(3, 29999, base={"KEEP": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
        assert e["KEEP"] == "1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="3", RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr
    assert r.stdout.strip() == ""


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU host: GPUs are visible")
def test_too_few_gpus_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr


def test_visible_gpus_sysfs_count(tmp_path, monkeypatch):
    """the launcher's GPU count reads the KFD topology (no HIP call in the parent) and honours the visibility
    variables"""
    sys.path.insert(0, ROOT)
    import bench

    for var in ("PZ_VISIBLE_GPUS", "ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    n = bench.visible_gpus()
    assert n >= 0
    if not os.path.exists("/dev/kfd"):
        assert n == 0
    monkeypatch.setenv("PZ_VISIBLE_GPUS", "8")
    assert bench.visible_gpus() == 8
    import torch

    assert not torch.cuda.is_initialized()


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU host: the ranks would run")
def test_failing_rank_fails_launcher():
    # PZ_VISIBLE_GPUS claims 2 GPUs on this CPU-only host: the ranks start and fail at torch.cuda.set_device
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-infer", "--no-cpu-baseline"],
                       env=_env(PZ_VISIBLE_GPUS="2"), capture_output=True, text=True, timeout=180)
    assert r.returncode != 0
    assert r.stdout.strip() == ""


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_two_ranks_one_gpu():
    """Rehearsal of the driver's multi-GPU run on one card: bench.py --gpus 2 counts the GPUs from sysfs as the real
    run does (1 here, with PZ_RANKS_PER_GPU=2 ranks per card), spawns 2 ranks (gloo, both on cuda:0), DDP over the
    gradient arena, one JSON line with n_gpus 2 and equal replica weights."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--micro-batch", "4", "--global-batch", "16",
                        "--steps", "1", "--warmup", "1", "--no-infer", "--no-cpu-baseline"],
                       env=_env(PZ_DIST_BACKEND="gloo", PZ_RANKS_PER_GPU="2"), capture_output=True, text=True,
                       timeout=840)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    print(json.dumps({k: out[k] for k in ("n_gpus", "value", "ms_per_step", "ddp", "config")}))
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 16 and out["config"]["grad_accum"] == 2
    dd = out["ddp"]
    assert dd["backend"] == "gloo"
    assert dd["async_rccl_buckets"] == 0  # gloo: synchronous buckets
    assert dd["buckets_reduced_per_step"] >= 2
    assert dd["replica_weights_equal"] is True
    assert out["value"] > 0 and out["loss_mean"] == out["loss_mean"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_four_ranks_one_gpu():
    """The data-parallel path at world size 4 on one card (gloo, PZ_RANKS_PER_GPU=4): the launcher's sysfs count (1
    GPU x 4 ranks), 4 replicas that each run one micro-batch per step, gradient buckets reduced across 4 ranks, equal
    replica weights after the step and a finite loss -- the widest rehearsal of the driver's 8-GPU run one card holds
    (C3 itself needs 8 cards: RCCL refuses two ranks on one device)."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "4", "--micro-batch", "4", "--global-batch", "16",
                        "--steps", "1", "--warmup", "1", "--no-infer", "--no-cpu-baseline"],
                       env=_env(PZ_DIST_BACKEND="gloo", PZ_RANKS_PER_GPU="4"), capture_output=True, text=True,
                       timeout=840)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    print(json.dumps({k: out[k] for k in ("n_gpus", "value", "ms_per_step", "ddp", "config", "loss_per_step")}))
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4"
    assert out["config"]["global_batch"] == 16 and out["config"]["grad_accum"] == 1
    assert out["ddp"]["replica_weights_equal"] is True
    assert all(v == v for v in out["loss_per_step"])
