"""Copies a profile_round.sh output tree's summaries into profiles/: per
workload its kernel stats and, per PMC pass, each kernel's counters averaged
over its dispatches (the raw per-dispatch CSVs stay in gpurun_out/).
usage: python tools/diag/prof_summaries.py gpurun_out/prof_<tag> profiles/<round>/prof"""
import collections
import csv
import glob
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
for wd in sorted(glob.glob(os.path.join(src, "*", "trace"))):
    w = os.path.basename(os.path.dirname(wd))
    out = os.path.join(dst, w)
    os.makedirs(out, exist_ok=True)
    for f in glob.glob(os.path.join(wd, "*kernel_stats.csv")):
        shutil.copy(f, os.path.join(out, "kernel_stats.csv"))
    for pd in sorted(glob.glob(os.path.join(os.path.dirname(wd), "pmc_*"))):
        if not os.path.isdir(pd):
            continue
        acc = collections.defaultdict(list)
        for f in glob.glob(os.path.join(pd, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
        with open(os.path.join(out, os.path.basename(pd) + "_summary.csv"), "w", newline="") as fh:
            wr = csv.writer(fh)
            wr.writerow(["kernel", "counter", "mean_per_dispatch", "dispatches"])
            for (k, c), v in sorted(acc.items()):
                wr.writerow([k, c, round(sum(v) / len(v), 1), len(v)])
    print(w)
