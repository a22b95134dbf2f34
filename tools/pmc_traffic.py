"""HBM traffic per k_resolve launch from a FETCH_SIZE and a WRITE_SIZE rocprofv3 --pmc pass of
`bench.py --config C` (tools/gpu_round.sh), written to profiles/pmc_traffic_cfgC.json, which
bench.py reads for `roofline.traffic`.

Which dispatches count: the k_resolve dispatches of the batch (the largest grid; the table
build's small pre-resolution dispatch is left out). A views batch of >= 2^19 strings runs a LEAN
first pass and a subset pass per step: the two are summed as one step (per_step_lean). In config 4 every step launches k_resolve
twice (the interpolation, then the unescape command's second resolve): the roofline kernel is the
first, so every other batch-sized dispatch counts, starting with the first. Both counters are in KB.

Reads. gfx950 tallies a wide streaming read at half its bytes (MI355X_MICROARCH.md) but a random
64-byte entry read at its bytes (tools/exp/gather_ubench.hip, profiles/r04/gather_calibration.txt),
and other widths are uncalibrated, so doubling the whole FETCH_SIZE over-counts a kernel that does
both. With a FETCH_SIZE pass of the same batch under IE_DEBUG_NOEVAL (the strings copied verbatim:
the kernel then reads exactly the streamed bytes S = input + offsets (+ table ids), a calibration on
a known byte count in this kernel's own access pattern), the reads are S + (FETCH - FETCH_noeval):
the evaluation's own reads (pilots, entries, arena texts, scratch) counted as tallied. Without that
pass: FETCH_SIZE doubled (the round-3 method, an upper bound). WRITE_SIZE as is.

  python3 tools/pmc_traffic.py C N <fetch_dir> <write_dir> <build_id> [<fetch_noeval_dir> <S bytes>]
"""
import csv
import glob
import re
import json
import os
import sys


def fused_unescape(name):
    """is this k_resolve instance the fused unescape command's (its 4th template flag, UNESC)?"""
    m = re.search(r"k_resolve<([^>]*)>", name)
    if m:
        args = [a.strip() for a in m.group(1).split(",")]
        return len(args) >= 4 and args[3] == "true"
    m = re.search(r"k_resolveILb([01])ELb([01])ELb([01])ELb([01])E", name)
    return bool(m and m.group(4) == "1")


def flags(name):
    """k_resolve's template flags (FAILC, MULTI, VIEWS, UNESC, LK, LEAN) from a kernel name."""
    m = re.search(r"k_resolve<([^>]*)>", name)
    if m:
        f = [a.strip() == "true" for a in m.group(1).split(",")]
    else:
        f = [b == "1" for b in re.findall(r"Lb([01])E", name.split("k_resolve", 1)[-1])]
    return (f + [False] * 6)[:6]


def per_step_lean(big):
    """A views batch that runs the LEAN first pass (the default at >= 2^19 strings): a step is the
    LEAN dispatch plus the subset pass right after it (same grid, not LEAN, not the fused command);
    packed-layout dispatches (not VIEWS) and the fused command are left out."""
    vals, i = [], 0
    while i < len(big):
        v, nm = big[i]
        f = flags(nm)
        if f[5]:
            tot = v
            if i + 1 < len(big):
                f2 = flags(big[i + 1][1])
                if f2[2] and not f2[3] and not f2[5]:
                    tot += big[i + 1][0]
                    i += 1
            vals.append(tot)
        i += 1
    return vals


def per_dispatch(d, counter, cfg):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_resolve" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                k = int(r["Dispatch_Id"])
                g = int(r["Grid_Size"])
                rows.setdefault(k, [g, 0.0, r["Kernel_Name"]])[1] += float(r["Counter_Value"])
    gmax = max(g for g, _, _ in rows.values())
    big = [(v, name) for k, (g, v, name) in sorted(rows.items()) if g == gmax]
    if any(flags(nm)[5] for _, nm in big):
        vals = per_step_lean(big)
    elif cfg == 4 and any(fused_unescape(nm) for _, nm in big):
        # views: each step is the interpolation, the fused command, its deferred subset: the
        # roofline kernel is the dispatch right before each fused one
        vals = [big[i][0] for i in range(len(big) - 1) if not fused_unescape(big[i][1]) and fused_unescape(big[i + 1][1])]
    elif cfg == 4:
        vals = [v for v, _ in big][0::2]  # packed: the interpolation, then the command's second resolve
    else:
        vals = [v for v, _ in big]
    return sum(vals) / len(vals), len(vals)


def main():
    cfg, n, fdir, wdir, bid = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    fetch, nf = per_dispatch(fdir, "FETCH_SIZE", cfg)
    write, nw = per_dispatch(wdir, "WRITE_SIZE", cfg)
    doubled = int(round((2 * fetch + write) * 1024))
    out = {
        "config": cfg,
        "n": n,
        "build_id": bid,
        "k_resolve_launches": [nf, nw],
        "fetch_size_kb": round(fetch),
        "write_size_kb": round(write),
        "hbm_bytes_per_step_fetch_doubled": doubled,
        "source": [os.path.relpath(fdir), os.path.relpath(wdir)],
    }
    if len(sys.argv) > 7:
        ndir, stream = sys.argv[6], int(sys.argv[7])
        fetch0, _ = per_dispatch(ndir, "FETCH_SIZE", cfg)
        reads = stream + (fetch - fetch0) * 1024
        out.update({"fetch_noeval_kb": round(fetch0), "stream_read_bytes": stream, "read_bytes": int(round(reads)),
                    "hbm_bytes_per_step": int(round(reads + write * 1024)),
                    "how": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over bench.py --config %d, "
                           "per k_resolve launch of the batch (config 4: the first resolve of each step); reads = the "
                           "streamed bytes S + (FETCH_SIZE - FETCH_SIZE under IE_DEBUG_NOEVAL), writes = WRITE_SIZE "
                           "(tools/pmc_traffic.py docstring)" % cfg})
        out["source"].append(os.path.relpath(ndir))
    else:
        out.update({"hbm_bytes_per_step": doubled,
                    "how": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over bench.py --config %d; "
                           "per k_resolve launch of the batch; FETCH_SIZE doubled, WRITE_SIZE as is" % cfg})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_traffic_cfg%d.json" % cfg)
    json.dump(out, open(path, "w"), indent=1)
    print(path, out["hbm_bytes_per_step"])


if __name__ == "__main__":
    main()
