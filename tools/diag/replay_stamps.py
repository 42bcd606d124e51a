"""Per-phase cycles of the wave replay for game 0 of a backend call, from the
diagnostic build tools/exp/diag_replay_stamps.patch (run with
FNNUE_LIB=exp/libfnnue_stamps.so): FEN, tokenising, the board chain, the
per-lane check + pack, the tail, the game-end flags (s_memtime cycles)."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import fishnet_amd as F  # noqa: E402
from fishnet_amd import _native as N  # noqa: E402
from fishnet_amd import backend as B  # noqa: E402

stub, actor = B.channel(F.Net.from_bytes(F.synthesize_net(1, 1024, 0)), 0)
bodies = bench.lichess_batches(F, 1, 400, c960=0.0, variants=0.0)
st = (C.c_ulonglong * 8)()
import os
split = bool(os.environ.get("CHAIN_SPLIT"))
names = ["fen", "tokenise", "chain" if not split else "chain:interpret+rest", "check+pack", "tail", "end flags"]
for k in (1, 64, 400):
    rows = []
    for _ in range(20):
        stub.go(bodies[:k])
        assert N.lib.fnnue_diag_replay_stamps(st) == 0
        rows.append(list(st))
    a = np.median(np.array(rows, dtype=np.float64), axis=0)
    extra = f"  chain:play={a[6]:.0f} chain:store={a[7]:.0f}" if split else f" total={a[6]:.0f} cyc moves={int(a[7])}"
    print(f"batches={k:4d} " + "  ".join(f"{n}={v:.0f}" for n, v in zip(names, a[:6])) + extra, flush=True)
actor.close()
