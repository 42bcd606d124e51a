"""Derive per-launch counters of the feature-transformer kernels from a
rocprofv3 PMC profile (tools/profile.sh) and record them in
profiles/traffic.json, which bench.py reports as roofline.traffic and
roofline.issue.

traffic: gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half
of the bytes of wide coalesced reads -> read bytes = 2 * FETCH_SIZE KiB;
WRITE_SIZE is exact for 16-B-per-lane stores.  Both count traffic leaving L2
toward the fabric, so Infinity-Cache hits are included (an upper bound on HBM
bytes).
issue: SQ_INSTS_VALU / SQ_INSTS_LDS of the dominant kernel (ft_slices), per
launch; bench.py divides by the measured kernel time.

usage: python tools/traffic.py <prof_dir> <key> [kernel-regex]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

prof, key = sys.argv[1], sys.argv[2]
pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else r"plan_|ft_slices|ft_scratch|ft_groups")
dominant = re.compile(r"ft_slices|ft_segments|ft_scratch|ft_groups")
per_kernel = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{prof}/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"::(\w+_kernel)", r["Kernel_Name"])
        if m and pat.search(m.group(1)):
            per_kernel[r["Counter_Name"]][m.group(1)].append(float(r["Counter_Value"]))


def mean_sum(counter, only=None):
    return sum(sum(v) / len(v) for k, v in per_kernel[counter].items() if only is None or only.search(k))


fetch, write = mean_sum("FETCH_SIZE"), mean_sum("WRITE_SIZE")
traffic = (2 * fetch + write) * 1024
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
db = json.load(open(path)) if os.path.exists(path) else {}
db[key] = {"bytes_per_launch": int(traffic), "fetch_kib": fetch, "write_kib": write,
           "kernels": sorted(per_kernel["FETCH_SIZE"]), "source": os.path.relpath(prof),
           "valu_insts_per_launch": mean_sum("SQ_INSTS_VALU", dominant) or None,
           "lds_insts_per_launch": mean_sum("SQ_INSTS_LDS", dominant) or None}
json.dump(db, open(path, "w"), indent=1, sort_keys=True)
print(key, db[key])
