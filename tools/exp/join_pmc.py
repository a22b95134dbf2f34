"""Join a microbenchmark's printed launch lines (one per dispatch, in launch order) with the
counters a rocprofv3 --pmc pass collected for those dispatches (summed per dispatch and counter).
  python3 tools/exp/join_pmc.py <program stdout> <rocprofv3 output dir> [kernel name filter]
Prints each line with its counters and, where the line carries bytes=, the counter / bytes ratio
(WRITE_SIZE and FETCH_SIZE are in KB)."""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    lines = [ln.strip() for ln in open(sys.argv[1]) if re.match(r"^\d+ ", ln)]
    filt = sys.argv[3] if len(sys.argv) > 3 else ""
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if filt and filt not in row.get("Kernel_Name", ""):
                continue
            per[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    for f in glob.glob(sys.argv[2] + "/**/*.db", recursive=True):  # (rocprofv3's default rocpd output)
        import sqlite3
        for did, name, cn, v in sqlite3.connect(f).execute(
                "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            if filt and filt not in name:
                continue
            per[int(did)][cn] += float(v)
    ids = sorted(per)
    for ln, d in zip(lines, ids):
        c = per[d]
        m = re.search(r"bytes=(\d+)", ln)
        extra = ""
        if m:
            b = int(m.group(1))
            extra = " " + " ".join("%s/bytes=%.3f" % (k, v * 1024 / b) for k, v in sorted(c.items()) if k.endswith("_SIZE"))
        print(ln, {k: round(v) for k, v in sorted(c.items())}, extra)


if __name__ == "__main__":
    main()
