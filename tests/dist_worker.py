"""One rank of the world-2 multi-GPU test (tests/test_multi.py, -m gpu): the library is loaded
before torch (bench.py's order), gloo carries only the control plane, every rank resolves its
own shard of the config-3 synthetic stream on the given device and checks it string by string
against the oracle; rank 0 prints the world's mismatch count as JSON."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--strings", type=int, default=100000)
    args = ap.parse_args()
    import __graft_entry__ as G
    G.check_built()
    pkg = G.load_package()
    N = pkg._native
    L = N.lib()
    import torch.distributed as dist  # after the library (one HIP runtime binding)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from oracle import oracle as O
    synth = ctypes.c_void_p()
    N.check(L.ie_synth_create(3, 0, ctypes.byref(synth)), "synth")
    kvp = ctypes.POINTER(N.KV)()
    nkv = L.ie_synth_kv(synth, ctypes.byref(kvp))
    first = rank * args.strings  # weak scaling: rank r owns strings [r n, (r+1) n)
    offs = np.zeros(args.strings + 1, np.uint64)
    tot = ctypes.c_uint64()
    N.check(L.ie_synth_strings_host(synth, first, args.strings, None, 0, offs.ctypes.data, ctypes.byref(tot)), "len")
    buf = np.zeros(int(tot.value) + 1, np.uint8)
    N.check(L.ie_synth_strings_host(synth, first, args.strings, buf.ctypes.data, buf.size, offs.ctypes.data,
                                    ctypes.byref(tot)), "fill")
    x = N.Exec(args.device)
    table = ctypes.c_void_p()
    clk = N.Clock(12, 34, 56)
    N.check(L.ie_table_build(ctypes.cast(kvp, ctypes.c_void_p), nkv, 0, ctypes.byref(clk), 0, args.device,
                             ctypes.byref(table)), "table")
    res = ctypes.POINTER(N.BatchRes)()
    N.check(L.ie_interpolate_batch(x.h, table, buf.ctypes.data, offs.ctypes.data, args.strings, ctypes.byref(res)), "batch")
    outs, sts, _ = N.batch_to_python(res)
    ref = O.Oracle.from_kv(ctypes.cast(kvp, ctypes.c_void_p), nkv, "py", clock=(12, 34, 56))
    rst = np.zeros(args.strings, np.uint8)
    rln = np.zeros(args.strings, np.uint64)
    rhs = np.zeros(args.strings, np.uint64)
    ref.run_batch(buf, offs, args.strings, 4, rst, rln, rhs, None)
    bad = 0
    for i in range(args.strings):
        h = O.fnv1a(outs[i]) if sts[i] == 0 else 0
        bad += int(sts[i] != rst[i] or len(outs[i]) != int(rln[i]) or h != int(rhs[i]))
    import torch
    t = torch.tensor([bad, args.strings], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world": world, "strings": int(t[1]), "mismatches": int(t[0])}), flush=True)
    L.ie_table_free(table)
    L.ie_synth_free(synth)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
