"""LDS cycles of the feature-transformer row reads, simulated on real plan
lists (would a 32-column slice, 45 KB tile, two
workgroups per CU pay?).

Each ds_read_b128 serves a wave in four 16-lane groups, 256 B (all 64 banks)
per cycle; a group costs as many cycles as the most-used bank has distinct
addresses.  The simulator builds the lists the plan builds (HalfKAv2_hm rows
relative to the king block, own king folded into the bias), sorts items by
(king block, piece count) as plan_scatter does, cuts passes, and counts the
cycles of every row-read step:

  A  64-column slices (the shipped layout): 8 lanes x 16 B per item, two items
     per group; plane stride = 32 (mod 256) B, so row r's chunks sit in bank
     half r & 1; lists parity-ordered (item index & 1 first).  A group costs 1
     cycle when its two rows differ in parity (or are one row), else 2.
  C  32-column slices: 4 lanes x 16 B per item, four items per group; plane
     stride = 64 (mod 256) B, row r's 16 banks set by r & 3; lists ordered by
     class starting at (item index & 3), padded with the zero row of that
     class.  A group costs the largest number of distinct rows in one class.

Also reported: rows per item-step (padding: a pass walks its longest list) and
the resulting LDS cycles per useful row.  The shipped layout's prediction is
checked against the measured SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

usage: python tools/lds_bank_sim.py [positions]
"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import fishnet_amd as F  # noqa: E402


def lists_of(pos: np.ndarray):
    """(king block, rows) per perspective-item, rows relative to the block."""
    b = np.zeros((len(pos), 64), np.int64)
    b[:, 0::2] = pos[:, :32] & 15
    b[:, 1::2] = pos[:, :32] >> 4
    sq = np.arange(64)
    items = []
    for c in (0, 1):
        own_k = 6 if c == 0 else 14
        ksq = np.argmax(b == own_k, axis=1)
        o = (56 if c else 0) ^ np.where((ksq & 7) < 4, 7, 0)
        kb = ((7 - ((ksq ^ o) >> 3)) * 4 + (7 - ((ksq ^ o) & 7)))
        typ = b & 7
        col = b >> 3
        plane = np.where(typ == 6, 10, 2 * (typ - 1) + (col != c))
        row = (sq[None, :] ^ o[:, None]) + 64 * plane
        occ = (b != 0) & ~((sq[None, :] == ksq[:, None]))
        for i in range(len(pos)):
            items.append((int(kb[i]), row[i][occ[i]]))
    return items


def simulate(items, lanes_per_item: int):
    per_group = 16 // lanes_per_item
    per_pass = 64 // lanes_per_item
    ncls = 2 if per_group == 2 else 4
    by_kb = {}
    for kb, rows in items:
        by_kb.setdefault(kb, []).append(rows)
    cycles = steps = useful = 0
    for kb, lst in by_kb.items():
        lst.sort(key=len)
        for p0 in range(0, len(lst), per_pass):
            pas = lst[p0:p0 + per_pass]
            L = max(len(r) for r in pas)
            ordered = []
            for j, rows in enumerate(pas):
                first = (p0 + j) % ncls
                cls = rows % ncls
                order = np.concatenate([rows[cls == (first + k) % ncls] for k in range(ncls)])
                pad = 704 + first if ncls == 4 else 704
                ordered.append(np.concatenate([order, np.full(L - len(order), pad)]))
                useful += len(rows)
            while len(ordered) % per_group:
                ordered.append(ordered[-1])  # clamped lanes repeat the unit's last item
            m = np.stack(ordered)  # items x L
            for g in range(0, len(m), per_group):
                grp = m[g:g + per_group]  # per_group x L
                for k in range(L):
                    rows = np.unique(grp[:, k])
                    cycles += int(np.bincount(rows % ncls, minlength=ncls).max())
                steps += L
            # groups of a wave instruction: a pass has 64 / (16) = 4 groups
    return cycles, steps, useful


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    pos = F.random_playouts(1, n, threads=8)
    items = lists_of(pos)
    res = {}
    for name, lanes in (("A 64-col slices, 8 lanes/item, 2 items/group", 8),
                        ("C 32-col slices, 4 lanes/item, 4 items/group", 4)):
        cyc, steps, useful = simulate(items, lanes)
        # cycles per group-step (1 = conflict-free); the work per useful row:
        # A reads a 128-B row per item-step, C a 64-B half row (twice the slices)
        groups = steps  # one group-step per (group, step)
        per_group = 16 // lanes
        row_bytes = 128 if lanes == 8 else 64
        cyc_per_useful = cyc / useful * (2 if lanes == 4 else 1)  # per full 128-B row of a useful item-row
        res[name] = (cyc / groups, (steps * per_group) / useful, cyc_per_useful)
        print(f"{name}: {cyc / groups:.3f} cycles per group-step (1 = conflict-free), "
              f"{(steps * per_group) / useful:.3f} item-steps per useful row, "
              f"{cyc_per_useful:.3f} LDS cycles per useful {row_bytes * (2 if lanes == 4 else 1)}-B row "
              f"(per 16 lanes)")
    a = res["A 64-col slices, 8 lanes/item, 2 items/group"]
    print(f"predicted conflict share of the shipped layout: {1 - 1 / a[0]:.3f} of row-read cycles")


if __name__ == "__main__":
    main()
