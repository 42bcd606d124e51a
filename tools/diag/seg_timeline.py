"""Timeline of ft_segments' (unit, slice) tasks from the diagnostic build
(tools/exp/diag_segtrace.patch -> exp/libfnnue_diag_segtrace.so): which CU /
XCD ran each task, when it started, when each of its 16 waves finished, how
many passes it walked.  Answers where the kernel idles:
CU occupancy over time, the tail, and the spread of wave end times inside a
task (the barrier wait before the next tile).

usage (GPU box): FNNUE_LIB=$PWD/exp/libfnnue_diag_segtrace.so python tools/diag/seg_timeline.py [--hd 1024]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hd", type=int, default=1024)
    ap.add_argument("--games", type=int, default=10_000)
    ap.add_argument("--mode", choices=["games", "children"], default="games")
    ap.add_argument("--out", default="gpurun_out/seg_timeline.json")
    args = ap.parse_args()
    import torch
    import fishnet_amd as F
    from fishnet_amd import _native as N
    lib = N.lib
    lib.fnnue_diag_seg_trace.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    mode = F.PLAYOUT_PLIES if args.mode == "games" else F.PLAYOUT_CHILDREN
    pos, off = F.random_playouts(2, args.games, 0, 160, mode=mode, threads=16)
    if args.mode == "children":
        lim = int(np.searchsorted(off, 1 << 20, side="right") - 1)
        pos, off = pos[: off[lim]], off[: lim + 1]
    ev = F.Evaluator(F.Net.from_bytes(F.synthesize_net(1, args.hd)), 0)
    dev = torch.device("cuda", 0)
    d_pos = torch.from_numpy(pos).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    n = len(pos)
    out = torch.zeros((2, n), dtype=torch.int32, device=dev)
    gmode = F.GROUP_CHAIN if args.mode == "games" else F.GROUP_STAR
    for _ in range(3):
        ev.eval_groups_device(d_pos.data_ptr(), d_off.data_ptr(), len(off) - 1, n, gmode, out[0].data_ptr(),
                              out[1].data_ptr(), None)
    ev.check()
    assert lib.fnnue_diag_seg_trace(None, 0, 1) == 0
    torch.cuda.synchronize()
    ev.eval_groups_device(d_pos.data_ptr(), d_off.data_ptr(), len(off) - 1, n, gmode, out[0].data_ptr(),
                          out[1].data_ptr(), None)
    ev.check()
    tr = np.zeros(((1 << 15), 20), np.uint64)
    assert lib.fnnue_diag_seg_trace(tr.ctypes.data, tr.nbytes, 0) == 0
    live = np.nonzero(tr[:, 0])[0]
    t = tr[live].astype(np.int64)
    t0 = t[:, 0].min()
    start = (t[:, 0] - t0) * 10  # s_memrealtime: 100 MHz -> ns
    ends = (t[:, 2:18] - t0) * 10
    end = ends.max(axis=1)
    hw = t[:, 1] & 0xFFFFFFFF
    xcc = (t[:, 1] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
    span = end.max()
    dur = end - start
    spread = end - ends.min(axis=1)  # first wave done -> last wave done
    passes = t[:, 18] & 0xFFFFFFFF
    items = t[:, 18] >> 32
    ucu = np.unique(cu_key)
    busy = np.zeros(len(ucu))
    for i, k in enumerate(ucu):
        m = cu_key == k
        busy[i] = dur[m].sum()
    res = {
        "hd": args.hd, "mode": args.mode, "positions": int(n), "tasks": int(len(live)), "cus_seen": int(len(ucu)),
        "kernel_span_us": round(span / 1e3, 1),
        "task_us": {"mean": round(dur.mean() / 1e3, 2), "p50": round(np.median(dur) / 1e3, 2),
                    "p90": round(np.percentile(dur, 90) / 1e3, 2), "max": round(dur.max() / 1e3, 2)},
        "cu_busy_frac": {"mean": round(busy.mean() / span, 3), "min": round(busy.min() / span, 3),
                         "max": round(busy.max() / span, 3)},
        "wave_end_spread_frac_of_task": round(float(spread.sum() / dur.sum()), 3),
        "per_xcd_last_end_us": [round(float(end[xcc == x].max()) / 1e3, 1) if np.any(xcc == x) else None
                                for x in range(8)],
        "per_xcd_busy_us": [round(float(dur[xcc == x].sum()) / 1e3, 1) for x in range(8)],
        "last_task_start_us": round(float(start.max()) / 1e3, 1),
        "tasks_ending_after_90pct": int((end > 0.9 * span).sum()),
        "longest_tasks": [{"start_us": round(float(start[i]) / 1e3, 1), "us": round(float(dur[i]) / 1e3, 1),
                           "passes": int(passes[i]), "items": int(items[i]), "xcc": int(xcc[i])}
                          for i in np.argsort(-dur)[:8]],
    }
    # CU occupancy over time (fraction of CUs running a task), 20 bins
    edges = np.linspace(0, span, 21)
    occ = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(end, b) - np.maximum(start, a), 0, None).sum()
        occ.append(round(float(ov / (b - a) / len(ucu)), 3))
    res["cu_occupancy_by_time"] = occ
    S = args.hd // 64
    sl = live % S
    res["task_us_by_slice"] = {"slice0": round(float(dur[sl == 0].mean()) / 1e3, 2),
                               "others": round(float(dur[sl != 0].mean()) / 1e3, 2)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
