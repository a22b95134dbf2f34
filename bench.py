#!/usr/bin/env python3
"""Benchmark of the `{key}` interpolation hot path on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic strings already resident in HBM:
  config 3 (default): 10M strings of 48-80 B, 1-2 nested `{q-{iM}}` refs, 100k-entry inserts
  config 2: 1M strings, 1-3 single-level `{kJ}` refs, 1k-entry inserts
  config 4: 12.5M strings per GPU (the 100M batch over 8), mixed-depth chains, escapes,
            brace-bearing values, misses; step = interpolate, then the `unescape` command
            (recursive_unescape + recursive_interpolate, py:1660-1667) on the results
  config 5: text_adventure.json5 forked states (10k per GPU): per state every string one loop
            iteration interpolates (the pre-pass of every executed task tree and the goto_map /
            replace_map first-round strings, from the reference-recorded trees in
            tests/golden/config5_trees.json) against one inserts dict per state, all states in
            one table set, a table id per string
Multi-GPU: one process per GPU, each resolving its own shard (the table is built per rank, no
data-path collective — only the barrier and the max-over-ranks time go over torch.distributed,
gloo on the host). `--gpus N` with N > 1 and no launcher around it starts the N rank processes
itself (child processes with torch.distributed.run's environment, started before this process
loads the library or makes any HIP call); under a launcher WORLD_SIZE must equal N. Rank r drives device LOCAL_RANK unless
`--device` makes ranks share one; `n_gpus` counts distinct devices, `ranks` the processes.
`--scaling weak` (configs 2-4 by default: every rank owns n strings, so config 4 at 8 GPUs is the
100M batch) or `strong` (config 5 by default: the 10k states are the global batch, split by state).

Prints ONE JSON line (rank 0): `value` = interpolated MB/s (input payload, 1 MB = 1e6 B) over
all ranks; `roofline` prices the resolve pipeline against HBM (algorithmic bytes
|in| + |out| + 17 per string); `cpu_baseline` times the C oracle (a literal
restatement of the reference algorithm, oracle/ie_oracle.c) on a bounded sample of the same
workload on this host, single-thread and on every core of this rank's CPU share.
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
CLOCK = (12, 34, 56)
WORKLOADS = {
    2: "cfg2: 1M strings/GPU, 48-80 B, 1-3 single-level {kJ} refs, 1k-entry inserts",
    3: "cfg3: 10M strings/GPU, 48-80 B, 1-2 nested {q-{iM}} refs, 100k-entry inserts",
    4: "cfg4: 12.5M strings/GPU (100M over 8), 48-80 B, 1-2 chain refs of depth 1-4 (40/30/20/10 %), "
       "10 % \\{lit\\} escapes, 2 % brace-bearing values, 1 % missing keys, 100k-entry inserts; "
       "step = interpolate + the unescape command (unescape, interpolate again)",
    5: "cfg5: text_adventure.json5 agent-loop states (10k/GPU), per state every string one loop iteration "
       "interpolates against its dict (the pre-pass of every executed task tree + the goto_map/replace_map "
       "first-round strings, ~180), one inserts dict per state in one table set",
}
DEFAULT_N = {2: 1_000_000, 3: 10_000_000, 4: 12_500_000, 5: 10_000}  # strings (configs 2-4) / states (5)
# the batch BASELINE.json names for each config (weak: per GPU; strong: over all GPUs)
DEFAULT_SCALING = {2: "weak", 3: "weak", 4: "weak", 5: "strong"}


def shard_first(rank, n_per_rank):
    """First global index (string or state) of a rank's shard: every rank owns n (weak scaling)."""
    return rank * n_per_rank


def shard_range(rank, world, n, scaling):
    """(first, count) of a rank's shard of the global unit (string / state) index space: weak
    scaling gives every rank n units, strong scaling splits n units over the world."""
    if scaling == "weak":
        return shard_first(rank, n), n
    lo, hi = rank * n // world, (rank + 1) * n // world
    return lo, hi - lo


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) without a launcher: start the N ranks as child processes with the
    environment torch.distributed.run gives them (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*), wait
    for all of them and return the first non-zero exit code (the others are then stopped). This
    process never loads the library or initialises HIP (no exec from a process that touched the
    GPU); the ranks are the ones that do."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # a failed rank leaves the others waiting at a barrier
                    q.terminate()
        time.sleep(0.05)
    return rc


def rank_devices(args, world, local, ndev):
    """This rank's device, or SystemExit when the request cannot be met: N ranks need N visible
    devices unless --device makes them share one explicitly."""
    if args.device >= 0:
        if args.device >= ndev:
            raise SystemExit("device %d requested, %d visible" % (args.device, ndev))
        return args.device
    if world > ndev:
        raise SystemExit("--gpus %d needs %d devices, %d visible (--device D shares one device)" % (world, world, ndev))
    return local


def max_over_ranks(x, dist):
    """Max of a float over all ranks (the step time the driver compares against its clock)."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(xs, dist):
    """Sums of integers over all ranks (the whole job's bytes and strings)."""
    if dist is None:
        return list(xs)
    import torch
    t = torch.tensor(list(xs), dtype=torch.int64)
    dist.all_reduce(t)
    return [int(v) for v in t.tolist()]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30, help="untimed steps first: the launch time settles over the first ~30 (0.86 -> 0.80 ms at config 3)")
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5])
    ap.add_argument("--n", type=int, default=0, help="strings (configs 2-4) or states (config 5) per GPU")
    ap.add_argument("--device", type=int, default=-1, help="HIP device (default: LOCAL_RANK)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget (wall seconds)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--layout", choices=["views", "packed"], default="",
                    help="output layout (default views; config 4 views runs the fused unescape command): views = each tile claims its "
                         "output range with one atomic (no look-back), packed = input order (look-back)")
    ap.add_argument("--no-packed", action="store_true", help="skip the packed-layout launches beside a views run")
    ap.add_argument("--reserve", type=int, default=32,
                    help="views output: IE_OPT_RESERVE (F x16: tile t writes at F x its input offset, no claim "
                         "atomic; 0 = one claim per tile on one cursor)")
    ap.add_argument("--replay", type=int, default=3,
                    help="config 5: loop iterations replayed after the timed steps, each mutating every state "
                         "(ie_table_set_update) and resolving the batch again (0: none)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="",
                    help="weak: --n units per GPU; strong: --n units over all GPUs (default per config: DEFAULT_SCALING)")
    ap.add_argument("--check-shard", type=int, default=-1,
                    help="strings of every rank's own shard checked against the oracle after the timed steps "
                         "(status, length, FNV-1a per string; config 5: the rank's whole batch); -1: 20000 "
                         "when there are several ranks, 0 otherwise")
    ap.add_argument("--dry-run", action="store_true",
                    help="control plane only (launcher, rank/device assignment, barrier, max over ranks): no library, "
                         "no GPU; --dry-devices devices are taken as visible")
    ap.add_argument("--dry-devices", type=int, default=-1)
    return ap.parse_args(argv)


def cpu_share():
    """Threads this rank may use (the box sets OMP_NUM_THREADS to its CPU share; os.cpu_count()
    shows the whole machine there), and the host's CPU model."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n = min(n, int(os.environ["OMP_NUM_THREADS"]))
    model = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return max(1, n), model


# ------------------------------------------------------------------------------------------
# workloads: device-resident inputs + what the CPU baseline needs
# ------------------------------------------------------------------------------------------
class Synth:
    """Configs 2-4: the library's counter-based generator writes the shard straight into HBM."""

    def __init__(self, N, L, x, cfg, first, n, dev):
        self.N, self.L, self.cfg, self.n = N, L, cfg, n
        self.synth = ctypes.c_void_p()
        N.check(L.ie_synth_create(cfg, 0, ctypes.byref(self.synth)), "ie_synth_create")
        self.kvp = ctypes.POINTER(N.KV)()
        self.nkv = L.ie_synth_kv(self.synth, ctypes.byref(self.kvp))
        self.table = ctypes.c_void_p()
        clk = N.Clock(*CLOCK)
        t0 = time.perf_counter()
        N.check(L.ie_table_build(ctypes.cast(self.kvp, ctypes.c_void_p), self.nkv, 0, ctypes.byref(clk), 0, dev,
                                 ctypes.byref(self.table)), "ie_table_build")
        self.build_s = time.perf_counter() - t0
        self.d_off = N.DeviceBuffer(x, (n + 1) * 8)
        tot = ctypes.c_uint64()
        N.check(L.ie_synth_strings_device(x.h, self.synth, first, n, None, 0, self.d_off.ptr, ctypes.byref(tot)), "synth")
        self.in_bytes = int(tot.value)
        self.d_in = N.DeviceBuffer(x, self.in_bytes + 16)
        N.check(L.ie_synth_strings_device(x.h, self.synth, first, n, self.d_in.ptr, self.d_in.nbytes, self.d_off.ptr,
                                          ctypes.byref(tot)), "synth")
        self.first = first
        self.inserts = int(self.nkv)
        self.d_ids = None

    def host_sample(self, m):
        N, L = self.N, self.L
        offs = np.zeros(m + 1, np.uint64)
        tot = ctypes.c_uint64()
        N.check(L.ie_synth_strings_host(self.synth, self.first, m, None, 0, offs.ctypes.data, ctypes.byref(tot)), "len")
        buf = np.zeros(int(tot.value) + 1, np.uint8)
        N.check(L.ie_synth_strings_host(self.synth, self.first, m, buf.ctypes.data, buf.size, offs.ctypes.data,
                                        ctypes.byref(tot)), "fill")
        return buf, offs

    def close(self):
        self.L.ie_table_free(self.table)
        self.L.ie_synth_free(self.synth)


def iteration_strings(trees):
    """Every string one text_adventure loop iteration interpolates against the state's dict: the
    per-task pre-pass of every executed task tree (recursive_interpolate, py:1501: every str leaf,
    goto_map / replace_map kept whole, py:1471-1477) and the first-round strings of the executed
    goto_map (text, keys, values: py:1692-1699) and replace_map tasks (output_name, item, keys:
    py:1715-1735). The trees are the reference's own (tests/golden/config5_trees.json)."""
    from interpolation_engine_amd import interpolation_engine as IE
    leaves, ids = [], []
    for x in trees:
        IE._tree_leaves({}, x, leaves, ids, 0)
        if x.get("cmd") == "goto_map":
            maps = x["target_maps"]
            leaves += [x["text"]] + [next(iter(d)) for d in maps] + [next(iter(d.values())) for d in maps]
        elif x.get("cmd") == "replace_map":
            leaves += [x["output_name"], x["item"]] + [next(iter(d)) for d in x["wildcard_maps"]]
    return leaves


class States:
    """Config 5: one inserts dict per agent-loop state (interpolation-engine_amd/workloads.py) in
    one table set, and per state every string one loop iteration with that stage interpolates
    (iteration_strings over the reference-recorded task trees, ~180 per state)."""

    def __init__(self, N, L, x, pkg, first, n, dev):
        from interpolation_engine_amd import workloads as Wk
        c5 = json.load(open(os.path.join(ROOT, "tests", "golden", "config5_trees.json"), encoding="utf-8"))
        defaults = json.load(open(os.path.join(ROOT, "tests", "golden", "config5_stream.json"),
                                  encoding="utf-8"))["defaults"]
        self.stream = {}
        for st in c5["states"]:  # the executed tasks of the first recorded state of each stage
            if st["stage"] not in self.stream:
                self.stream[st["stage"]] = iteration_strings([t["x"] for t in st["trees"]])
        self.states = [Wk.state_inserts(defaults, first + j) for j in range(n)]
        strings, ids = [], []
        for j, ins in enumerate(self.states):
            tpl = self.stream[ins["stage"]]
            strings.extend(tpl)
            ids.extend([j] * len(tpl))
        self.ids = np.asarray(ids, dtype=np.uint32)
        self.n = len(strings)
        t0 = time.perf_counter()
        self.tset = pkg.InsertsTableSet(self.states, clock=CLOCK, device=dev, mutable=False)
        self.build_s = time.perf_counter() - t0
        self.table = self.tset.h
        blob, offs = N.pack(strings)
        self.in_bytes = len(blob)
        self.d_in = N.DeviceBuffer.from_numpy(x, np.frombuffer(blob + bytes(16), np.uint8))
        self.d_off = N.DeviceBuffer.from_numpy(x, offs)
        self.d_ids = N.DeviceBuffer.from_numpy(x, self.ids)
        self.blob, self.offs = blob, offs
        self.inserts = len(self.tset.keys)

    def close(self):
        self.tset.close()


def dry_run(args, world, rank, local):
    """The multi-rank control plane without the library or a GPU (tests/test_bench_launch.py):
    device assignment, the barrier and the max-over-ranks time, and the line's rank fields."""
    ndev = args.dry_devices if args.dry_devices >= 0 else world
    dev = rank_devices(args, world, local, ndev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    devs = gather_devices(dev, world, dist)
    cfg = args.config
    scaling = args.scaling or DEFAULT_SCALING[cfg]
    first, n = shard_range(rank, world, args.n or DEFAULT_N[cfg], scaling)
    units = [None] * world
    if dist:
        dist.all_gather_object(units, (first, n))
        dist.barrier()
    else:
        units = [(first, n)]
    wall = max_over_ranks(0.001 * (rank + 1), dist)
    if rank == 0:
        print(json.dumps({"metric": "interpolated MB/s + strings/s on synthetic batches at 1/2/4/8 MI355X", "value": None,
                          "unit": "MB/s", "n_gpus": len(set(devs)), "ranks": world, "devices": devs, "dry_run": True,
                          "scaling": scaling, "shards": units, "wall_max_s": wall}), flush=True)
    if dist:
        dist.destroy_process_group()


def gather_devices(dev, world, dist):
    """Every rank's device (rank order)."""
    if dist is None:
        return [dev]
    out = [None] * world
    dist.all_gather_object(out, dev)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE is %d" % (args.gpus, world))
    if args.dry_run:
        return dry_run(args, world, rank, local)

    # the library (and with it the HIP runtime it links) is loaded before anything imports torch:
    # torch bundles a HIP runtime of the same soname, and which one binds depends on load order
    import __graft_entry__ as G
    G.check_built()  # never compiles here (this process may already hold the GPU, e.g. under rocprofv3)
    pkg = G.load_package()
    N = pkg._native
    L = N.lib()
    ndev = L.ie_device_count()
    if ndev <= 0:
        raise SystemExit("no HIP device visible")
    dev = rank_devices(args, world, local, ndev)

    dist = None
    if world > 1:
        # control plane only (barrier + max-over-ranks time): the shards are independent
        import torch.distributed as dist
        dist.init_process_group("gloo")
    devs = gather_devices(dev, world, dist)

    cfg = args.config
    scaling = args.scaling or DEFAULT_SCALING[cfg]
    # this rank's shard of the global string / state index space
    first, n_units = shard_range(rank, world, args.n or DEFAULT_N[cfg], scaling)
    total_units = n_units * world if scaling == "weak" else (args.n or DEFAULT_N[cfg])
    x = N.Exec(dev)
    # literal-path scratch sized for the workload (the call stays asynchronous; the statuses below
    # prove no string ran out of it)
    N.check(L.ie_exec_set_scratch(x.h, (2 << 30) if cfg == 4 else (256 << 20)), "ie_exec_set_scratch")
    W = Synth(N, L, x, cfg, first, n_units, dev) if cfg != 5 else States(N, L, x, pkg, first, n_units, dev)
    n = W.n
    in_bytes = W.in_bytes
    out_cap = 3 * in_bytes + (64 << 20) if cfg != 5 else 16 * in_bytes + (64 << 20)
    d_out = N.DeviceBuffer(x, out_cap)
    d_ooff = N.DeviceBuffer(x, (n + 1) * 8)
    d_st = N.DeviceBuffer(x, n + 1)
    d_vid = N.DeviceBuffer(x, 4 * n + 4)
    d_tot = N.DeviceBuffer(x, 8)
    ids = W.d_ids.ptr if W.d_ids is not None else None
    cmd = cfg == 4  # the unescape command on the results (py:1660-1667): unescape, interpolate again
    layout = args.layout or "views"
    views = layout == "views"
    d_olen = N.DeviceBuffer(x, 4 * n + 4) if views else None
    reserve = args.reserve if views and (args.reserve * in_bytes) // 16 + (in_bytes >> 2) + (64 << 20) <= out_cap else 0
    N.check(L.ie_exec_set_option(x.h, N.OPT_RESERVE, reserve), "IE_OPT_RESERVE")
    if views:
        o = N.DevViews(d_out.ptr, out_cap, d_ooff.ptr, d_olen.ptr, d_st.ptr, d_vid.ptr, d_tot.ptr)
    else:
        o = N.DevOut(d_out.ptr, out_cap, d_ooff.ptr, d_st.ptr, d_vid.ptr, d_tot.ptr)

    def resolve():
        if views:
            return L.ie_interpolate_device_views(x.h, W.table, ids, W.d_in.ptr, W.d_off.ptr, None, n, ctypes.byref(o))
        return L.ie_interpolate_device_ids(x.h, W.table, ids, W.d_in.ptr, W.d_off.ptr, n, ctypes.byref(o))
    if cmd:
        d_out2 = N.DeviceBuffer(x, out_cap)
        d_ooff2 = N.DeviceBuffer(x, (n + 1) * 8)
        d_st2 = N.DeviceBuffer(x, n + 1)
        d_tot2 = N.DeviceBuffer(x, 8)
        d_olen2 = N.DeviceBuffer(x, 4 * n + 4) if views else None
        if views:  # fused: each tile unescaped in LDS and resolved (no unescaped copy in HBM)
            o2 = N.DevViews(d_out2.ptr, out_cap, d_ooff2.ptr, d_olen2.ptr, d_st2.ptr, d_vid.ptr, d_tot2.ptr)
        else:
            d_u = N.DeviceBuffer(x, out_cap)
            d_uoff = N.DeviceBuffer(x, (n + 1) * 8)
            d_ust = N.DeviceBuffer(x, n + 1)
            d_utot = N.DeviceBuffer(x, 8)
            tmp = N.DevOut(d_u.ptr, out_cap, d_uoff.ptr, d_ust.ptr, d_vid.ptr, d_utot.ptr)
            o2 = N.DevOut(d_out2.ptr, out_cap, d_ooff2.ptr, d_st2.ptr, d_vid.ptr, d_tot2.ptr)

    # HIP events on the exec's stream: config 4 around each of a step's two calls (the resolve is the
    # roofline kernel, the command is reported beside it); the others around the whole timed loop
    # (one pair: no event records between the steps' kernels)
    per_step_marks = cmd

    def step(k=None):
        if k is not None and per_step_marks:
            x.mark(3 * k)
        N.check(resolve(), "resolve")
        if k is not None and per_step_marks:
            x.mark(3 * k + 1)
        if cmd and views:
            N.check(L.ie_unescape_cmd_device_views(x.h, W.table, None, d_out.ptr, d_ooff.ptr, d_olen.ptr, n, d_st.ptr,
                                                   ctypes.byref(o2)), "ie_unescape_cmd_device_views")
        elif cmd:
            N.check(L.ie_unescape_cmd_device(x.h, W.table, None, d_out.ptr, d_ooff.ptr, n, d_st.ptr,
                                             ctypes.byref(tmp), ctypes.byref(o2)), "ie_unescape_cmd_device")
        if k is not None and per_step_marks:
            x.mark(3 * k + 2)

    for _ in range(args.warmup):
        step()
    x.sync()
    out_bytes = int(d_tot.to_numpy(np.uint64, 1)[0])
    assert out_bytes <= out_cap
    st_final = (d_st2 if cmd else d_st).to_numpy(np.uint8, n)
    names = N.STATUS_NAMES
    status_counts = {names[k]: int(c) for k, c in enumerate(np.bincount(st_final, minlength=len(names))[:len(names)]) if c}
    # (diagnostic IE_DEBUG_NOEVAL runs leave statuses unwritten or verbatim: not checked)
    assert "E_OVERFLOW" not in status_counts or os.environ.get("IE_DEBUG_NOEVAL"), "scratch too small"

    if dist:
        dist.barrier()
    x.sync()
    t0 = time.perf_counter()
    assert args.steps <= 341, "HIP event slots: 3 per step, 1024 in all"
    if not per_step_marks:
        x.mark(0)
    for k in range(args.steps):  # HIP events on the exec's stream (above)
        step(k)
    if not per_step_marks:
        x.mark(1)
    x.sync()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    res_ms = ([x.elapsed(3 * k, 3 * k + 1) for k in range(args.steps)] if per_step_marks
              else [x.elapsed(0, 1) / args.steps])
    cmd_ms = [x.elapsed(3 * k + 1, 3 * k + 2) for k in range(args.steps)] if cmd else None
    wall_max = max_over_ranks(wall, dist)

    # the §8b packed layout (offsets[N+1] in input order, what ie_interpolate_device writes) timed on
    # the same batch and build beside the views headline (untimed for `value`; 20 launches)
    packed = None
    if views and cfg in (2, 3) and not args.no_packed:
        op = N.DevOut(d_out.ptr, out_cap, d_ooff.ptr, d_st.ptr, d_vid.ptr, d_tot.ptr)
        for k in range(25):
            if k >= 5:
                x.mark(2 * (k - 5))
            N.check(L.ie_interpolate_device_ids(x.h, W.table, ids, W.d_in.ptr, W.d_off.ptr, n, ctypes.byref(op)),
                    "packed")
            if k >= 5:
                x.mark(2 * (k - 5) + 1)
        x.sync()
        pk_ms = float(np.mean([x.elapsed(2 * k, 2 * k + 1) for k in range(20)]))
        pk_out = int(d_tot.to_numpy(np.uint64, 1)[0])
        pk_alg = in_bytes + pk_out + 17 * n + (4 * n if ids is not None else 0)
        packed = {"launch_ms": round(pk_ms, 4), "frac": round(pk_alg / (pk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                  "launches": 20, "note": "packed offsets[N+1] layout (decoupled look-back), same batch and build"}
        N.check(resolve(), "views again")  # (the views results back in the buffers for the checks below)
        x.sync()

    x.set_timing(True)  # one more call with the library's own events for the telemetry
    if cmd and not views and os.environ.get("IE_DIAG_CMD_RESOLVE"):  # diagnostic: the command's second resolve instead
        N.check(L.ie_interpolate_device(x.h, W.table, d_u.ptr, d_uoff.ptr, n, ctypes.byref(o2)), "timing")
    elif cmd and views and os.environ.get("IE_DIAG_CMD_RESOLVE"):  # diagnostic: the fused command (its stamps)
        N.check(L.ie_unescape_cmd_device_views(x.h, W.table, None, d_out.ptr, d_ooff.ptr, d_olen.ptr, n, d_st.ptr,
                                               ctypes.byref(o2)), "timing")
    else:
        N.check(resolve(), "timing")
    tm = x.timing()
    x.set_timing(False)

    gpu_ms = float(np.mean(res_ms))
    id_bytes = 4 * n if ids is not None else 0
    alg_bytes = in_bytes + out_bytes + 17 * n + id_bytes  # |in| + |out| + 16 (offsets) + 1 (status)
    achieved_gbs = alg_bytes / (gpu_ms * 1e-3) / 1e9
    all_bytes, all_strings = sum_over_ranks([in_bytes, n], dist)
    value = all_bytes / wall_max * args.steps / 1e6  # MB/s over all ranks
    strings_per_s = all_strings * args.steps / wall_max

    cpu = None
    if rank == 0 and not args.no_cpu:
        res = Result(N, n, d_out2 if cmd else d_out, d_ooff2 if cmd else d_ooff, d_st2 if cmd else d_st,
                     d_olen2 if cmd else d_olen, d_tot2 if cmd else d_tot)
        cpu = cpu_baseline(args, W, N, res)

    replay = None
    if rank == 0 and cfg == 5 and args.replay > 0:
        res = Result(N, n, d_out, d_ooff, d_st, d_olen, d_tot)
        replay = replay_states(args, W, x, resolve, res)

    # every rank checks its own shard (the 1 -> 8 GPU runs verify every GPU's results, not rank 0's)
    nchk = args.check_shard if args.check_shard >= 0 else (20000 if world > 1 else 0)
    mine = None
    if nchk:
        res = Result(N, n, d_out2 if cmd else d_out, d_ooff2 if cmd else d_ooff, d_st2 if cmd else d_st,
                     d_olen2 if cmd else d_olen, d_tot2 if cmd else d_tot)
        mine = shard_check(args, W, res, nchk, rank, first)
    checks, launch = [mine], [round(gpu_ms, 4)]
    if dist:
        checks, launch = [None] * world, [None] * world
        dist.all_gather_object(checks, mine)
        dist.all_gather_object(launch, round(gpu_ms, 4))

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic_cfg%d.json" % cfg)
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            # only figures measured on this very build of the kernels count
            bid = L.ie_build_id()
            bid = bid.decode() if isinstance(bid, bytes) else str(bid)
            if pm.get("config") == cfg and pm.get("n") == n and pm.get("build_id") == bid:
                traffic = pm.get("hbm_bytes_per_step")
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        line = {
            "metric": "interpolated MB/s + strings/s on synthetic batches at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "MB/s",
            "n_gpus": len(set(devs)),
            "ranks": world,
            "devices": devs,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (SURVEY §8d generators; configs 2-4 splitmix64 seed 0x1E5EED00+config generated in "
                    "HBM; config 5 seeded states + the reference-recorded call stream)",
            "config": {"workload": WORKLOADS[cfg], "layout": layout,
                       "claim": ("reserved ranges at %g x the input offsets" % (reserve / 16)) if reserve else
                                ("one atomic per tile" if views else "look-back"), "strings_per_gpu": n, "input_bytes_per_gpu": in_bytes,
                       "output_bytes_per_gpu": out_bytes, "inserts": W.inserts, "parallelism": "shard%d" % world,
                       "units_total": total_units, "input_bytes_total": all_bytes,
                       "statuses": status_counts, "table_build_s": round(W.build_s, 3)},
            "strings_per_s": round(strings_per_s, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "k_resolve (single pass: stage, evaluate, %s, emit) + k_emit_windows"
                                   % ("claim the tile's output range" if views else "look-back"),
                         "launch_ms": round(gpu_ms, 4), "alg_bytes_per_launch": alg_bytes,
                         "launch_ms_ranks": launch, "launch_ms_max": max(launch), "launch_ms_min": min(launch),
                         "telemetry": {"kernel_ms": round(tm.resolve_ms, 4), "literal_strings": int(tm.n_complex),
                                       "windowed_tiles": int(tm.n_direct), "exact_strings": int(tm.n_exact),
                                       "chain_failures": int(tm.n_chain_fail), "deferred": int(tm.n_deferred)}},
            "cpu_baseline": cpu,
        }
        if packed:
            line["roofline"]["packed_layout"] = packed
        if nchk:
            line["shard_checks"] = checks
        if cfg == 5:
            line["config"]["states_per_gpu"] = n_units
            line["replay"] = replay
        if cmd:
            ob2 = int(d_tot2.to_numpy(np.uint64, 1)[0])
            ums = float(np.mean(cmd_ms))
            if views:  # fused: read out1 + its views and statuses, write out2 + views + statuses
                ub = None
                ualg = out_bytes + ob2 + 2 * 13 * n
            else:  # unescape: read out1, write tmp; interpolate: read tmp, write out2
                ub = int(d_utot.to_numpy(np.uint64, 1)[0])
                ualg = out_bytes + ub + ub + ob2 + 2 * 17 * n
            line["unescape_cmd"] = {"ms": round(ums, 4), "unescaped_bytes": ub, "output_bytes": ob2,
                                    "fused": views, "achieved_gbs": round(ualg / (ums * 1e-3) / 1e9, 1)}
        print(json.dumps(line), flush=True)
    W.close()
    if dist:
        dist.destroy_process_group()


class Result:
    """The device results of a step in either layout, read back for the checks."""

    def __init__(self, N, n, d_out, d_off, d_st, d_len, d_tot):
        self.N, self.n, self.d_out, self.d_off, self.d_st, self.d_len, self.d_tot = N, n, d_out, d_off, d_st, d_len, d_tot

    def spans(self, m):
        """(starts, lengths) of strings [0, m), uint64"""
        if self.d_len is not None:
            return self.d_off.to_numpy(np.uint64, m), self.d_len.to_numpy(np.uint32, m).astype(np.uint64)
        oo = self.d_off.to_numpy(np.uint64, m + 1)
        return oo[:-1], np.diff(oo)

    def compare(self, m, st, ln, hs, threads):
        """strings [0, m) against the oracle's statuses, lengths and FNV-1a hashes"""
        from oracle import oracle as O
        gst = self.d_st.to_numpy(np.uint8, m)
        starts, lens = self.spans(m)
        if not np.array_equal(gst, st) or not np.array_equal(lens[gst == 0], ln[gst == 0]):
            return False
        total = int(self.d_tot.to_numpy(np.uint64, 1)[0])
        # (views: the results' extent; reserved ranges leave gaps, *total is the sum of lengths)
        ext = int((starts + lens).max()) if m else 0
        blob = self.d_out.to_numpy(np.uint8, max(total, ext))
        return bool(np.array_equal(O.hash_spans(blob, starts, lens, gst, threads), hs))


def cpu_baseline(args, W, N, res):
    """The oracle (a literal C restatement of interpolate_inserts, kind "port") timed on this host
    over a bounded sample of the same workload, single-thread and on every core of this rank's
    share; the GPU's results on the sample are checked against it string by string."""
    from oracle import oracle as O
    threads, model = cpu_share()
    if args.cpu_threads:
        threads = args.cpu_threads
    budget = args.cpu_seconds
    if args.config == 5:
        return cpu_baseline_states(args, W, N, res, model, budget, threads)
    ref = O.Oracle.from_kv(ctypes.cast(W.kvp, ctypes.c_void_p), W.nkv, "py", clock=CLOCK)
    cmd = args.config == 4
    buf, offs = W.host_sample(20000)
    dt1 = ref.run_batch(buf, offs, 20000, 1, unescape_cmd=cmd)  # single-thread calibration
    per_string = max(dt1 / 20000, 1e-9)
    m = int(min(W.n, max(20000, budget * 0.5 * threads / per_string)))
    buf, offs = W.host_sample(m)
    m1 = int(min(m, max(20000, budget * 0.25 / per_string)))
    wall1 = ref.run_batch(buf, offs, m1, 1, unescape_cmd=cmd)
    st = np.zeros(m, np.uint8)
    ln = np.zeros(m, np.uint64)
    hs = np.zeros(m, np.uint64)
    wall = ref.run_batch(buf, offs, m, threads, st, ln, hs, None, unescape_cmd=cmd)
    same = res.compare(m, st, ln, hs, threads)
    return {"value": round(int(offs[m]) / wall / 1e6, 2), "unit": "MB/s", "cores": threads, "kind": "port",
            "value_1t": round(int(offs[m1]) / wall1 / 1e6, 2), "threads_all": threads, "cpu_model": model,
            "nproc_visible": os.cpu_count(), "strings_per_s": round(m / wall, 1),
            "sample": "first %d strings (%d B) of this rank's shard, oracle/ie_oracle.c on %d threads (%.2f s), "
                      "single-thread on the first %d (%.2f s)%s; GPU results identical on all %d: %s"
                      % (m, int(offs[m]), threads, wall, m1, wall1,
                         "; each OK result then through the unescape command" if cmd else "", m, same)}


def shard_check(args, W, res, m, rank, first):
    """This rank's own results against the oracle: the first m strings of its shard (config 4: each
    OK result then through the unescape command; config 5: every string of the rank's states, each
    against its own state's dict), per string status, length and FNV-1a of the bytes."""
    from oracle import oracle as O
    threads, _ = cpu_share()
    if args.config == 5:
        oracles = [O.Oracle(ins, "py", clock=CLOCK) for ins in W.states]
        buf = np.frombuffer(W.blob + bytes(1), np.uint8)
        st, ln, hs = np.zeros(W.n, np.uint8), np.zeros(W.n, np.uint64), np.zeros(W.n, np.uint64)
        O.run_batch_sets(oracles, W.ids, buf, W.offs, threads, st, ln, hs)
        return {"rank": rank, "first_state": first, "states": len(W.states), "strings": W.n,
                "identical": res.compare(W.n, st, ln, hs, threads)}
    m = int(min(m, W.n))
    ref = O.Oracle.from_kv(ctypes.cast(W.kvp, ctypes.c_void_p), W.nkv, "py", clock=CLOCK)
    buf, offs = W.host_sample(m)
    st, ln, hs = np.zeros(m, np.uint8), np.zeros(m, np.uint64), np.zeros(m, np.uint64)
    ref.run_batch(buf, offs, m, threads, st, ln, hs, None, unescape_cmd=args.config == 4)
    return {"rank": rank, "first_string": first, "strings": m, "identical": res.compare(m, st, ln, hs, threads)}


def replay_states(args, W, x, resolve, res):
    """Config 5 as the loop runs it (not a frozen snapshot): between two iterations every state
    takes the stores an iteration makes (set_interpdata, py:470-471; user_input py:1566-1568; the
    model's output and the history replace_maps py:1770-1773): new_user_input, maybe_input, output,
    the appended history_text_llm and length_history. The stores go to the device table set in place
    (ie_table_set_update, no rebuild), then the iteration's strings are resolved again. Per
    iteration: the host's store time (packing + the library call), the library call alone, and the
    resolve; after the last iteration every string is compared with the oracle on the mutated
    states."""
    from interpolation_engine_amd import workloads as Wk
    from oracle import oracle as O
    upd, nat, rsv, nch, arena, split = [], [], [], 0, [], []
    for it in range(args.replay):
        changes = []
        for j, ins in enumerate(W.states):
            r = Wk._Rng(0xC0FFEE ^ (j * 0x9E3779B1) ^ (it << 40))
            inp, out = r.words(2, 8), r.words(15, 55)
            hist = ins["history_text_llm"] + "\n\n<action>" + inp + "</action>\n\n<action-output>" + out + "</action-output>"
            for k, v in (("new_user_input", inp), ("maybe_input", inp), ("output", out), ("history_text_llm", hist),
                         ("length_history", ins["length_history"] + 2)):
                ins[k] = v
                changes.append((j, k, v))
        nch = len(changes)
        t0 = time.perf_counter()
        if not W.tset.update(changes):
            raise RuntimeError("replay: a new key found no placement")
        t1 = time.perf_counter()
        x.sync()
        t2 = time.perf_counter()
        resolve()
        x.sync()
        t3 = time.perf_counter()
        upd.append(t1 - t0)
        nat.append(W.tset.last_update_native_s)
        split.append(W.tset.last_update_split_s)
        rsv.append(t3 - t2)
        arena.append(W.tset.arena_stats())
    threads, _ = cpu_share()
    oracles = [O.Oracle(ins, "py", clock=CLOCK) for ins in W.states]
    buf = np.frombuffer(W.blob + bytes(1), np.uint8)
    st, ln, hs = np.zeros(W.n, np.uint8), np.zeros(W.n, np.uint64), np.zeros(W.n, np.uint64)
    O.run_batch_sets(oracles, W.ids, buf, W.offs, threads, st, ln, hs)
    same = res.compare(W.n, st, ln, hs, threads)
    return {"iterations": args.replay, "stores_per_iteration": nch,
            "store_ms": [round(1e3 * v, 3) for v in upd], "store_library_ms": [round(1e3 * v, 3) for v in nat],
            "store_pack_ms": [round(1e3 * v[0], 3) for v in split],
            "store_values_ms": [round(1e3 * v[2], 3) for v in split],
            "resolve_ms": [round(1e3 * v, 3) for v in rsv],
            "arena_bytes": [a[0] for a in arena], "arena_live_bytes": [a[1] for a in arena],
            "arena_compactions": arena[-1][2] if arena else 0,
            "values_held": len(W.tset.values),
            "identical_to_oracle_after_replay": same,
            "note": "store_ms = InsertsTableSet.update: store_pack_ms (csrc/ie_pack.c: the changes -> ie_kv "
                    "records, texts transcoded across host threads) + store_library_ms (ie_table_set_store) + "
                    "store_values_ms (the value list); resolve_ms = wall time of one batch (launch + sync)"}


def cpu_baseline_states(args, W, N, res, model, budget, threads):
    """Config 5: every state of this rank's batch, each string against its own state's inserts
    (one oracle context per state, built untimed), on all threads of this rank's share and
    single-thread; the GPU's results are compared on the whole batch."""
    from oracle import oracle as O
    oracles = [O.Oracle(ins, "py", clock=CLOCK) for ins in W.states]
    buf = np.frombuffer(W.blob + bytes(1), np.uint8)
    n = W.n
    st, ln, hs = np.zeros(n, np.uint8), np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    wall = O.run_batch_sets(oracles, W.ids, buf, W.offs, threads, st, ln, hs)
    wall1 = O.run_batch_sets(oracles, W.ids, buf, W.offs, 1)
    same = res.compare(n, st, ln, hs, threads)
    return {"value": round(W.in_bytes / max(wall, 1e-9) / 1e6, 2), "unit": "MB/s", "cores": threads, "kind": "port",
            "value_1t": round(W.in_bytes / max(wall1, 1e-9) / 1e6, 2), "threads_all": threads, "cpu_model": model,
            "nproc_visible": os.cpu_count(), "strings_per_s": round(n / max(wall, 1e-9), 1),
            "sample": "all %d states (%d strings, %d B), each string against its own state's dict, "
                      "oracle/ie_oracle.c on %d threads (%.3f s) and single-thread (%.3f s); GPU results "
                      "identical on all: %s" % (len(W.states), n, W.in_bytes, threads, wall, wall1, same)}


if __name__ == "__main__":
    main()
