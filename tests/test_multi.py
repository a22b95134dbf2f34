"""Multi-GPU paths. CPU: byte-balanced shard bounds. GPU: the library's in-process
multi-device batch (table replicated device-to-device, shards on their own execs; two shards on
device 0 when the box has one GPU) against the oracle, and a world-2 torch.distributed (gloo
control plane) run of one rank per shard, both ranks on device 0, each checked string by string."""
import json
import os
import random
import socket
import subprocess
import sys

import numpy as np
import pytest

import __graft_entry__ as G
from oracle import oracle as O
from tests.conftest import ROOT


def _pkg():
    G.build()
    return G.load_package()


def test_shard_bounds_are_byte_balanced():
    pkg = _pkg()
    rng = np.random.default_rng(3)
    for n in [0, 1, 7, 1000, 12345]:
        lens = rng.integers(0, 200, n).astype(np.uint64)
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        for k in [1, 2, 3, 8]:
            first = pkg.shard_bounds(offs, k)
            assert first[0] == 0 and first[-1] == n and np.all(np.diff(first.astype(np.int64)) >= 0)
            total = int(offs[-1])
            for j in range(1, k):
                f = int(first[j])
                target = total * j // k
                assert int(offs[f]) >= target and (f == 0 or int(offs[f - 1]) < target)


@pytest.mark.gpu
def test_multi_device_batch_vs_oracle():
    pkg = _pkg()
    rng = random.Random(5)
    inserts = {"k%d" % j: rng.choice(["v%d" % j, j, "{k%d}" % ((j + 1) % 50), ["a", j]]) for j in range(50)}
    strings = ["".join(rng.choice(["x", "{k%d}" % rng.randrange(55), " ", "\\{", "é"]) for _ in range(rng.randrange(0, 12)))
               for _ in range(5000)]
    M = pkg.MultiDevice(inserts, [0, 0, 0], clock=(12, 34, 56))
    got = M.run(strings)
    ref = O.Oracle(inserts, "py", clock=(12, 34, 56))
    N = pkg._native
    for s, (st, payload) in zip(strings, got):
        rst, rout, rvid = ref.interpolate(s)
        assert N.STATUS_NAMES[st] == rst, s
        if rst == "OK_STR":
            assert payload == rout, s
        if rst == "OK_VALUE":
            assert payload == rvid, s
    M.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_world2_ranks_on_one_device():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "dist_worker.py"),
           "--device", "0", "--strings", "50000"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r == {"world": 2, "strings": 100000, "mismatches": 0}, r
