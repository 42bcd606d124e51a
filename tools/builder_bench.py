"""Throughput of the batch builders (host board.cpp vs device builder.hip) on
analysis-batch-shaped input: N random legal games of ~L plies from the start
position, expanded to every ply (PLIES) or every ply + legal children
(CHILDREN).  Prints one JSON line per (builder, mode).  GPU box only.

    python tools/builder_bench.py [--games 4000] [--plies 80]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fishnet_amd as F  # noqa: E402
from fishnet_amd import _native as N  # noqa: E402

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4000)
    ap.add_argument("--plies", type=int, default=80)
    a = ap.parse_args()
    import torch
    games = [(START, F.random_game(77 + i, START, a.plies)) for i in range(a.games)]
    ev = F.Evaluator(F.Net.from_bytes(F.synthesize_net(1, 128, 0)), 0)
    text, fen_off, mv_off = F.pack_games(games)
    dev = torch.device("cuda", 0)
    d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev)
    d_fo = torch.from_numpy(fen_off.astype(np.int32)).to(dev)
    d_mo = torch.from_numpy(mv_off.astype(np.int32)).to(dev)
    import ctypes as C
    for mode, name in ((N.PLAYOUT_PLIES, "plies"), (N.PLAYOUT_CHILDREN, "children")):
        n, g = C.c_size_t(), C.c_size_t()
        rc = N.lib.fnnue_build_batch_device(ev.handle, C.c_void_p(d_text.data_ptr()), C.c_void_p(d_fo.data_ptr()),
                                            C.c_void_p(d_mo.data_ptr()), len(games), mode, None, 0, None, 0,
                                            C.byref(n), C.byref(g), None)
        assert rc == -10, rc
        d_out = torch.empty((n.value, 36), dtype=torch.uint8, device=dev)
        d_off = torch.empty(g.value + 1, dtype=torch.int32, device=dev)

        def run():
            N.check(N.lib.fnnue_build_batch_device(ev.handle, C.c_void_p(d_text.data_ptr()),
                                                   C.c_void_p(d_fo.data_ptr()), C.c_void_p(d_mo.data_ptr()),
                                                   len(games), mode, C.c_void_p(d_out.data_ptr()), n.value,
                                                   C.c_void_p(d_off.data_ptr()), g.value + 1, C.byref(n),
                                                   C.byref(g), None))
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        hn = 0
        for f, m in games[: max(1, len(games) // 10)]:
            hn += len(F.game_positions(f, m) if mode == N.PLAYOUT_PLIES else F.game_children(f, m)[0])
        ht = (time.perf_counter() - t0) * len(games) / max(1, len(games) // 10)
        print(json.dumps({"mode": name, "games": len(games), "positions": n.value,
                          "device_positions_per_s": n.value / dt, "device_ms": dt * 1e3,
                          "host_1thread_positions_per_s": hn * len(games) / max(1, len(games) // 10) / ht}))
    ev.close()


if __name__ == "__main__":
    main()
