"""Median replay-kernel time per batch count from a rocprofv3 kernel trace
(tools/diag/replay_ab.sh)."""
import collections
import csv
import glob
import sys

name, d = sys.argv[1], sys.argv[2]
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t = collections.defaultdict(list)
size = None
for r in rows:
    n = r["Kernel_Name"]
    if "replay_wave_kernel" not in n:
        continue
    games = int(r["Grid_Size_X"]) // 64
    kind = "V" if "Variant" in n else "C"
    if kind == "C":
        size = games
    t[(size, kind)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = []
for (size, kind), v in sorted(t.items(), key=lambda kv: (kv[0][0] or 0, kv[0][1])):
    v.sort()
    out.append(f"{kind}@{size}:{v[len(v) // 2]:.1f}us")
print(f"{name:12s} " + " ".join(out), flush=True)
