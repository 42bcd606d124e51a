"""Roofline of the evaluator's kernels from a rocprofv3 profile of the tree
(tools/profile_round.sh): per workload and kernel, the average duration
(kernel trace) and PMC counters per dispatch, and the fraction of each
hardware resource the kernel uses:

  valu   SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x cycles): vector-instruction
         issue.  4 cycles per wave64 instruction is the issue cost of the
         64-bit-encoded VALU forms that dominate these kernels (v_pk_add_u16,
         SDWA, v_perm; measured 1.75x a VOP2 add, tools/diag/valu_bench.hip),
         so the fraction slightly over-states the busy time of VOP2 work.
  lds    SQ_LDS_IDX_ACTIVE / (256 CUs x cycles): LDS-array busy (rocprof's
         LdsUtil); bank-conflict cycles are part of it.
  hbm    (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB / duration / 8 TB/s: bytes past
         L2 (gfx950 FETCH_SIZE counts half of wide reads, MI355X_MICROARCH.md
         §HBM; Infinity-Cache hits included, so an upper bound on HBM bytes).
  mfma   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles): matrix-core busy
         (the stack kernel's L1 / fc_1 contractions, v_mfma_i32_16x16x64_i8).
  cycles = 2.4 GHz (spec clock) x the kernel's average duration from the
  kernel trace, as bench.py prices its live times.  The derived clock
  GRBM_GUI_ACTIVE / 8 / duration (the counter sums the 8 XCDs) is reported
  only as a diagnostic: on dispatches shorter than ~0.3 ms the counter window
  is longer than the kernel and the quotient reads above the part's 2.4 GHz
  (MI355X_MICROARCH.md, DVFS), so a value above 2.4 is flagged, never used.

The binding resource of a kernel is the one with the largest fraction.
Writes <prof>/counters.json and, with --install <key-prefix>, merges it into
profiles/counters.json which bench.py reads (keyed by workload, tagged with
the source hash of the kernels it was measured on).

usage: python tools/roofline.py <prof_dir> [--install]
"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS, SIMDS, XCDS, HBM_PEAK, CLOCK = 256, 1024, 8, 8.0e12, 2.4e9
FOCUS = ("ft_slices_kernel", "ft_segments_kernel", "stack_kernel", "ft_scratch_kernel", "ft_groups_kernel",
         "replay_pair_kernel", "replay_wave_kernel")


def tree_hash() -> str:
    """sha256 over the sources of the evaluation kernels (what their counters depend on)."""
    h = hashlib.sha256()
    src = os.path.join(ROOT, "fishnet_amd", "csrc")
    files = ("kernels.hip", "ft_sliced.hip", "ft_segments.hip", "device_common.h", "sliced_common.h", "kernels.h",
             # the engine actor's replay (backend:<k> workloads)
             "builder.hip", "vbuilder.hip", "replay_wave.h", "board.h", "vboard.h")
    for f in sorted(os.path.join(src, f) for f in files):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def kname(full: str) -> str:
    m = re.search(r"(\w+_kernel)", full)
    return m.group(1) if m else full[:40]


def workload(d: str) -> dict:
    dur = {}
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        k = kname(r["Name"])
        if k in dur:  # several template instances (e.g. the actor's chess and variant nets): keep the busiest
            if float(r["TotalDurationNs"]) <= dur[k]["total_ns"]:
                continue
        dur[k] = {"avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]), "total_ns": float(r["TotalDurationNs"]),
                  "full": r["Name"]}
    # counters per instance; a kernel's are those of the instance its time is (the busiest)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            ctr[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    by_short = collections.defaultdict(list)
    for full in ctr:
        by_short[kname(full)].append(full)
    out = {}
    for k in sorted(set(dur) | set(by_short)):
        full = dur.get(k, {}).get("full")
        if full not in ctr:
            full = by_short[k][0] if len(by_short.get(k, [])) == 1 else None
        c = {n: sum(v) / len(v) for n, v in ctr.get(full, {}).items()} if full else {}
        rec = {"avg_ns": dur.get(k, {}).get("avg_ns"), "calls": dur.get(k, {}).get("calls"), "counters": c}
        if full and len(by_short.get(k, [])) > 1:
            rec["instance"] = full
        t = rec["avg_ns"]
        if k in FOCUS and t and c:
            cyc = CLOCK * t * 1e-9
            fr = {}
            if "SQ_INSTS_VALU" in c:
                fr["valu"] = c["SQ_INSTS_VALU"] * 4 / (SIMDS * cyc)
            if "SQ_LDS_IDX_ACTIVE" in c:
                fr["lds"] = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                fr["mfma"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                hbm_bytes = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
                rec["hbm_bytes"] = hbm_bytes
                fr["hbm"] = hbm_bytes / (t * 1e-9) / HBM_PEAK
            rec["cycles"] = cyc
            if "GRBM_GUI_ACTIVE" in c:
                rec["grbm_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / XCDS / t
                rec["grbm_window_exceeds_kernel"] = rec["grbm_clock_ghz"] > CLOCK / 1e9
            rec["fractions"] = fr
            if fr:
                rec["bound"] = max(fr, key=fr.get)
            if "SQ_WAVE_CYCLES" in c:
                wc = c["SQ_WAVE_CYCLES"]
                rec["wave_states"] = {  # quad-cycles summed over waves (disjoint buckets)
                    "mean_waves_per_cu": wc * 4 / (CUS * cyc),  # at the spec clock: a floor
                    "active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                    "wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                    "wait_inst_lds": c.get("SQ_WAIT_INST_LDS", 0) / wc,
                    "wait_any": c.get("SQ_WAIT_ANY", 0) / wc}
        out[k] = rec
    return out


def main():
    prof = sys.argv[1]
    res = {"tree": tree_hash(), "source": os.path.relpath(prof, ROOT), "workloads": {}}
    for d in sorted(glob.glob(os.path.join(prof, "*", "trace"))):
        wl = os.path.basename(os.path.dirname(d))
        res["workloads"][wl] = workload(os.path.dirname(d))
    json.dump(res, open(os.path.join(prof, "counters.json"), "w"), indent=1, sort_keys=True)
    for wl, ks in res["workloads"].items():
        for k, r in ks.items():
            if "fractions" in r:
                fr = " ".join(f"{n}={v:.3f}" for n, v in r["fractions"].items())
                ws = r.get("wave_states", {})
                clk = r.get("grbm_clock_ghz")
                flag = "" if clk is None else (f" (GRBM {clk:.2f} GHz: window > kernel)" if clk > CLOCK / 1e9
                                               else f" (GRBM {clk:.2f} GHz)")
                print(f"{wl:9s} {k:20s} {r['avg_ns'] / 1e3:8.1f} us  at 2.40 GHz{flag}  {fr}  "
                      f"bound={r.get('bound')}  waves/CU={ws.get('mean_waves_per_cu', 0):.1f}")
    if "--install" in sys.argv:
        path = os.path.join(ROOT, "profiles", "counters.json")
        json.dump(res, open(path, "w"), indent=1, sort_keys=True)
        print("installed", path)


if __name__ == "__main__":
    main()
