"""bench.py --gpus N measures N ranks by itself: without a launcher around it
the parent starts the N rank processes (torch.distributed.run as a child, before any library load
or HIP call), each rank takes its own device unless --device shares one, and the printed line
counts distinct devices (`n_gpus`) apart from processes (`ranks`). CPU: the control plane in
--dry-run mode (gloo, no library, no GPU). GPU: two ranks sharing device 0."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable, BENCH] + list(args), cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


def test_launcher_two_ranks_two_devices():
    p, line = _run("--gpus", "2", "--dry-run", "--dry-devices", "2", "--n", "1000")
    assert p.returncode == 0, p.stderr[-3000:]
    assert line["n_gpus"] == 2 and line["ranks"] == 2 and line["devices"] == [0, 1]
    assert line["scaling"] == "weak" and line["shards"] == [[0, 1000], [1000, 1000]]


def test_launcher_shared_device_counts_one_gpu():
    p, line = _run("--gpus", "2", "--device", "0", "--dry-run", "--dry-devices", "1", "--n", "10")
    assert p.returncode == 0, p.stderr[-3000:]
    assert line["n_gpus"] == 1 and line["ranks"] == 2 and line["devices"] == [0, 0]


def test_launcher_refuses_missing_devices():
    p, line = _run("--gpus", "2", "--dry-run", "--dry-devices", "1", "--n", "10")
    assert p.returncode != 0 and line is None
    assert "needs 2 devices, 1 visible" in p.stderr


def test_strong_scaling_splits_the_global_batch():
    # config 5 defaults to strong scaling: BASELINE's 10k states are the batch over all GPUs
    p, line = _run("--gpus", "2", "--config", "5", "--dry-run", "--dry-devices", "2", "--n", "10001")
    assert p.returncode == 0, p.stderr[-3000:]
    assert line["scaling"] == "strong" and line["shards"] == [[0, 5000], [5000, 5001]]


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE is 1" in p.stderr


@pytest.mark.gpu
def test_two_ranks_on_one_card_report_one_gpu():
    """The real bench, two ranks sharing device 0 (the box has one GPU): n_gpus 1, ranks 2."""
    p, line = _run("--gpus", "2", "--device", "0", "--n", "200000", "--steps", "3", "--warmup", "1", "--no-cpu",
                   timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert line["n_gpus"] == 1 and line["ranks"] == 2 and line["devices"] == [0, 0]
    assert line["config"]["statuses"] == {"OK_STR": 200000} and line["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("config,n,scaling", [(4, 400000, "weak"), (5, 600, "strong")], ids=["cfg4-weak", "cfg5-strong"])
def test_two_ranks_check_their_own_shards(config, n, scaling):
    """The multi-rank path of the configs the 8-GPU run scales differently: config 4 weak (every rank
    its own 12.5M-string shape, the fused unescape command), config 5 strong (the states split over
    the ranks). Every rank checks its own shard against the oracle and the line carries every
    rank's kernel time."""
    p, line = _run("--gpus", "2", "--device", "0", "--config", str(config), "--n", str(n), "--steps", "3",
                   "--warmup", "1", "--no-cpu", "--replay", "0", "--check-shard", "20000", timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    assert line["ranks"] == 2 and line["scaling"] == scaling
    checks = line["shard_checks"]
    assert [c["rank"] for c in checks] == [0, 1] and all(c["identical"] for c in checks), checks
    if scaling == "weak":
        assert [c["first_string"] for c in checks] == [0, n]
    else:
        assert [c["first_state"] for c in checks] == [0, n // 2] and sum(c["states"] for c in checks) == n
    r = line["roofline"]
    assert len(r["launch_ms_ranks"]) == 2 and r["launch_ms_max"] >= r["launch_ms_min"] > 0
