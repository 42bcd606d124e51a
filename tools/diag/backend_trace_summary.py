"""Per-go() HIP API usage of the backend actor from a rocprofv3 --hip-trace
(tools/backend_trace.sh): the actor thread's calls split into go() calls at
each run of stream synchronisations; per batch-count phase, the steady-state
calls (warm-up excluded): API calls per go(), allocations, host waits.
usage: python tools/diag/backend_trace_summary.py <trace dir> <calls per phase> <phases...>"""
import collections
import csv
import glob
import sys

d, per = sys.argv[1], int(sys.argv[2])
phases = sys.argv[3:]
rows = []
for f in glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
waits = ("hipStreamSynchronize", "hipEventSynchronize")
syncs = collections.Counter(r["Thread_Id"] for r in rows if r["Function"] in waits)
actor = syncs.most_common(1)[0][0]
quiet = ("__hipPushCallConfiguration", "__hipPopCallConfiguration", "hipGetLastError", "hipSetDevice",
         "hipGetDevice")
calls, cur, in_sync = [], [], False
for r in rows:
    if r["Thread_Id"] != actor:
        continue
    f = r["Function"]
    if f not in waits and in_sync and f in ("hipMemcpyAsync", "hipLaunchKernel"):
        calls.append(cur)
        cur = []
    # device guards, launch bookkeeping and event polls leave the state as it is
    if f not in quiet:  # a call ends with its last wait or event poll
        in_sync = f in waits or f == "hipEventQuery"
    cur.append(r)
calls.append(cur)
calls = [c for c in calls if any(r["Function"] in waits + ("hipEventQuery",) for r in c)]
# each phase = warm-up calls + 1 probe + `per` timed calls; the timed ones are the last `per`
n_phase = len(calls) // len(phases)
alloc = ("hipMalloc", "hipFree", "hipHostMalloc", "hipHostFree", "hipMallocAsync", "hipFreeAsync")
for i, name in enumerate(phases):
    timed = calls[(i + 1) * n_phase - per:(i + 1) * n_phase]
    c = collections.Counter(r["Function"] for call in timed for r in call)
    span = [(int(call[-1]["End_Timestamp"]) - int(call[0]["Start_Timestamp"])) / 1e3 for call in timed]
    print(f"{name} batches/go: {len(timed)} steady-state go() calls; per call: " +
          ", ".join(f"{k} {v / len(timed):g}" for k, v in c.most_common()) +
          f"; allocations/frees: {sum(c[a] for a in alloc)}; actor API span median {sorted(span)[len(span) // 2]:.1f} us")
