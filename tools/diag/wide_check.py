"""Diagnostic: each FT impl vs the oracle for the wide nets (positions and groups)."""
import sys

import numpy as np

import fishnet_amd as F
from fishnet_amd import _native as N
from oracle.oracle import OracleNet

for seed, hd, flags in ((10, 3072, N.SYNTH_WRAP), (10, 3072, 0), (9, 2560, 0), (8, 1536, 0), (6, 2048, 0)):
    data = F.synthesize_net(seed, hd, flags)
    ev, on = F.Evaluator(F.Net.from_bytes(data), 0), OracleNet(data)
    for n in (3000, 50000):
        pos = F.random_playouts(seed + 7, n, threads=8)
        ops, opo, _ = on.eval_packed(pos, threads=8)
        for impl in (N.FT_SLICED, N.FT_GATHER):
            ev.set_ft_impl(impl)
            ps, po = ev.eval_positions(pos)
            bad = np.nonzero((ps != ops) | (po != opo))[0]
            print(hd, flags, n, "sliced" if impl == N.FT_SLICED else "gather", "bad", len(bad), bad[:8],
                  "psqt-bad", int((ps != ops).sum()), flush=True)
    ev.close()
sys.exit(0)
