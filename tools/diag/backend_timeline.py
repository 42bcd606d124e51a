"""Timeline of one steady-state fnnue_backend_go call from a rocprofv3 trace
(tools/backend_trace.sh): the actor thread's HIP API calls and every kernel /
copy that started inside the call, in µs from the call's first API call.

usage: python tools/diag/backend_timeline.py <trace dir> <phase index> [phases]
  phases = number of batch-count phases in the run (default 2); the call shown
  is the second-to-last of the given phase
"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
phase = int(sys.argv[2])
nph = int(sys.argv[3]) if len(sys.argv) > 3 else 2


def rows(pattern):
    out = []
    for f in glob.glob(f"{d}/**/{pattern}", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


api = sorted(rows("*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
ker = rows("*kernel_trace.csv")
cpy = rows("*memory_copy_trace.csv")
waits = ("hipStreamSynchronize", "hipEventSynchronize")
actor = collections.Counter(r["Thread_Id"] for r in api if r["Function"] in waits).most_common(1)[0][0]
# device guards / launch bookkeeping between a call's last wait and the next call's first copy
quiet = ("__hipPushCallConfiguration", "__hipPopCallConfiguration", "hipGetLastError", "hipSetDevice",
         "hipGetDevice")
calls, cur, in_wait = [], [], False
for r in api:
    if r["Thread_Id"] != actor:
        continue
    f = r["Function"]
    if f in quiet:
        continue
    # a call ends with its last wait or event poll; the next copy or launch starts the next one
    if f not in waits and in_wait and f in ("hipMemcpyAsync", "hipLaunchKernel") and cur and \
            cur[-1]["Function"] in waits + ("hipEventQuery",):
        calls.append(cur)
        cur = []
    in_wait = f in waits or f == "hipEventQuery"
    cur.append(r)
calls.append(cur)
calls = [c for c in calls if any(r["Function"] in waits + ("hipEventQuery",) for r in c)]
per = len(calls) // nph
c = calls[(phase + 1) * per - 2]
t0 = int(c[0]["Start_Timestamp"])
t1 = int(c[-1]["End_Timestamp"])
print(f"call span {(t1 - t0) / 1e3:.1f} us, {len(c)} API calls on the actor thread")
skip = ("__hipPushCallConfiguration", "__hipPopCallConfiguration", "hipGetLastError", "hipSetDevice", "hipGetDevice")
ev = []
for r in c:
    if r["Function"] in skip:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev.append((s, e, "api", r["Function"]))
for k in ker:
    s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    if t0 <= s <= t1:
        nm = re.sub(r"fnnue::|\(anonymous namespace\)::|void |HIP_vector_type", "", k["Kernel_Name"])
        ev.append((s, e, "ker", nm.split("(")[0][:90] + (" q" + k.get("Queue_Id", "") if "Queue_Id" in k else "")))
for k in cpy:
    s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    if t0 <= s <= t1:
        ev.append((s, e, "cpy", k.get("Direction", "")))
for s, e, kind, name in sorted(ev):
    print(f"  {kind} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name}")
