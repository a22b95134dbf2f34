"""The N>1 control plane of bench.py on CPU (gloo, world size 2): each rank generates its own shard
of the global synthetic string stream (no data-path collective), and the step time reported is the
max over ranks. The shards must tile the single-process stream exactly."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import __graft_entry__ as G

N_PER_RANK = 3000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_bytes(N, L, synth, first, n):
    offs = np.zeros(n + 1, np.uint64)
    tot = ctypes.c_uint64()
    N.check(L.ie_synth_strings_host(synth, first, n, None, 0, offs.ctypes.data, ctypes.byref(tot)), "len")
    buf = np.zeros(int(tot.value) + 1, np.uint8)
    N.check(L.ie_synth_strings_host(synth, first, n, buf.ctypes.data, buf.size, offs.ctypes.data,
                                    ctypes.byref(tot)), "fill")
    return buf[:int(tot.value)].tobytes()


def _worker(rank, world, port, result_dir, config=3):
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = G.load_package()
    N = pkg._native
    L = N.lib()
    synth = ctypes.c_void_p()
    N.check(L.ie_synth_create(config, 0, ctypes.byref(synth)), "synth")
    mine = _shard_bytes(N, L, synth, bench.shard_first(rank, N_PER_RANK), N_PER_RANK)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    wall = bench.max_over_ranks(0.5 + rank, dist)
    if rank == 0:
        whole = _shard_bytes(N, L, synth, 0, world * N_PER_RANK)
        ok = b"".join(gathered) == whole and wall == 0.5 + (world - 1)
        open(os.path.join(result_dir, "ok"), "w").write("1" if ok else "0")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config", [3, 4])
def test_two_rank_shards_tile_the_stream(tmp_path, config):
    G.build()
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), config), nprocs=2, join=True)
    assert (tmp_path / "ok").read_text() == "1"
