"""Rows per item of ft_slices with a per-unit base accumulator.

CPU analysis only, no kernel: over config 2's positions (random playouts,
seed 1, L ~ U[0, 160], as bench.py's default positions workload) cut the
items the way the plan does (plan_count / plan_scatter: key = king block * 33
+ pieces; plan_scan_kernel_t: each king block's items in chunks of
FT_UNIT_ITEMS = 6144 from the block start) and count the feature rows one
item costs

  today:  n - 1 rows (the own king joins the bias, ft_sliced.hip:248-259),
          and a wave sums the longest list of its 8-item pass (the items of a
          unit are sorted by n, so that is about n - 1)
  base:   |item \\ B| + |B \\ item| rows, B = every row present in at least
          half of the unit's items (the optimal single base: a row joins B iff
          that lowers the unit's total), own king included in both; the items
          re-sorted by that count inside the unit, 8-item passes priced at
          their maximum

and prints both means.  VERDICT's bar: build only if the base form is at
least 15 % lower.

  usage: python tools/diag/base_rows.py [--positions 1000000] [--unit 6144] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from fishnet_amd import nnue as F  # noqa: E402

# king block of the own king seen from its perspective (SF 15.1 HalfKAv2_hm
# KingBuckets after the orientation flip; the same table as tests/refpy.py)
KING_BUCKET = np.full(64, -1, dtype=np.int64)
for _sq in range(64):
    _r, _f = divmod(_sq, 8)
    if _f >= 4:
        KING_BUCKET[_sq] = 4 * (7 - _r) + (7 - _f)


def items_of(pos: np.ndarray):
    """Per perspective-item: king block, piece count n, and its n rows (own king included) as a
    boolean matrix over the 704 rows of the block."""
    raw = pos.reshape(-1, 36)
    lo, hi = raw[:, :32] & 15, raw[:, :32] >> 4
    board = np.empty((len(raw), 64), dtype=np.int64)
    board[:, 0::2], board[:, 1::2] = lo, hi
    sq = np.arange(64)
    out = []
    for persp in (0, 1):
        king = 6 if persp == 0 else 14
        ksq = np.argmax(board == king, axis=1)
        flip = (56 if persp else 0) ^ np.where(ksq % 8 < 4, 7, 0)
        kb = KING_BUCKET[ksq ^ flip]
        ptype, colour = board & 7, board >> 3
        plane = np.where(ptype == 6, 10, 2 * (ptype - 1) + (colour != persp))
        row = (sq[None, :] ^ flip[:, None]) + 64 * plane
        present = board != 0
        m = np.zeros((len(raw), 704), dtype=bool)
        r_idx, c_idx = np.nonzero(present)
        m[r_idx, row[r_idx, c_idx]] = True
        out.append((kb, present.sum(axis=1), m))
    kb = np.concatenate([o[0] for o in out])
    n = np.concatenate([o[1] for o in out])
    m = np.concatenate([o[2] for o in out])
    return kb, n, m


def pass_cost(costs_sorted: np.ndarray) -> int:
    """Rows summed by the waves of one unit: 8 items per pass, priced at the pass's maximum."""
    k = len(costs_sorted)
    pad = (-k) % 8
    c = np.concatenate([costs_sorted, np.repeat(costs_sorted[-1:], pad)]) if pad else costs_sorted
    return int(c.reshape(-1, 8).max(axis=1).sum() * 8)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--positions", type=int, default=1_000_000)
    ap.add_argument("--unit", type=int, default=6144)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out")
    a = ap.parse_args()
    pos = F.random_playouts(a.seed, a.positions, 0, 160, threads=8)
    kb, n, m = items_of(pos)
    order = np.lexsort((n, kb))  # counting sort by key kb * 33 + n
    kb, n = kb[order], n[order]
    tot_today = tot_today_pass = tot_base = tot_base_pass = 0
    base_sizes, units = [], 0
    for b in range(32):
        idx = np.nonzero(kb == b)[0]
        for c in range(0, len(idx), a.unit):
            sel = idx[c:c + a.unit]
            mm = m[order[sel]]
            today = n[sel] - 1
            tot_today += int(today.sum())
            tot_today_pass += pass_cost(today)  # already sorted by n inside the block
            freq = mm.sum(axis=0)
            B = freq * 2 >= len(sel)
            inter = mm[:, B].sum(axis=1)
            cost = (n[sel] - inter) + (int(B.sum()) - inter)
            tot_base += int(cost.sum())
            tot_base_pass += pass_cost(np.sort(cost))
            base_sizes.append(int(B.sum()))
            units += 1
    items = len(kb)
    res = {
        "positions": a.positions, "items": items, "units": units, "unit_items": a.unit,
        "rows_per_item_today": tot_today / items, "rows_per_item_today_passes": tot_today_pass / items,
        "rows_per_item_base": tot_base / items, "rows_per_item_base_passes": tot_base_pass / items,
        "base_rows_mean": float(np.mean(base_sizes)),
        "reduction_passes": 1 - tot_base_pass / tot_today_pass,
        "bar": 0.15,
    }
    res["verdict"] = "build" if res["reduction_passes"] >= 0.15 else "no-go"
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
