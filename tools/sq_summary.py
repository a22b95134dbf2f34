"""Per-wave SQ counter averages of the k_resolve launches in rocprofv3 --pmc counter_collection CSVs
(one line per kernel instance with >= 1e5 waves): VALU / SALU / LDS instructions, the wave's life
(SQ_WAVE_CYCLES, 4-cycle units), the cycles it waited on memory (SQ_WAIT_ANY), issued (ACTIVE_INST_ANY)."""
import collections
import csv
import sys

COLS = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_WAIT_INST_ANY"]


def summary(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "k_resolve" in r["Kernel_Name"]:
            agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    out = []
    for k, d in agg.items():
        if d["SQ_WAVES"] < 1e5:
            continue
        inst = k[k.index("k_resolve<"):k.index(">") + 1]
        out.append("%-50s waves=%.0f %s" % (inst, d["SQ_WAVES"], " ".join(
            "%s=%.0f" % (c[3:], d[c] / d["SQ_WAVES"]) for c in COLS)))
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for line in summary(p):
            print(p.split("/")[-1].replace("_counters.csv", ""), line)
