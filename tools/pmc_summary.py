"""Summarise rocprofv3 --pmc counter CSVs for k_resolve: per-dispatch averages and per-wave ratios."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    vals = defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_resolve" not in row.get("Kernel_Name", ""):
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    # one row per (dispatch, counter) after rocprof's per-dimension sum
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    w = avg.get("SQ_WAVES")
    print(d, {k: round(v) for k, v in sorted(avg.items())})
    if w:
        print("   per wave:", {k: round(v / w, 1) for k, v in sorted(avg.items()) if k != "SQ_WAVES"})
