"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel per dispatch."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        m = re.search(r"::(\w+_kernel)", r["Kernel_Name"])
        if not m:
            continue
        agg[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{k:22s} {c:24s} dispatches={len(v):3d} mean={sum(v)/len(v):.6g}")
