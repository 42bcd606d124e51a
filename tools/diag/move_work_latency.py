"""Engine-actor latency of move work (Work::Move, [ref] src/api.rs:160-165:
the position after all moves, a one-ply search over its legal children) at
1 / 8 / 64 move batches per go(), against the oracle's children values.
FNNUE_FT_IMPL=sliced|auto picks the children's feature transformer.
usage: python tools/diag/move_work_latency.py"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fishnet_amd as F  # noqa: E402
from fishnet_amd import backend as B  # noqa: E402
from tests.conftest import net_bytes  # noqa: E402

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
games = json.load(open(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "wcc_games.json")))["games"]
stub, actor = B.channel(F.Net.from_bytes(net_bytes(1, 1024, 0)), 0)
out = {"ft_impl": os.environ.get("FNNUE_FT_IMPL", "auto")}
try:
    for nb in (1, 8, 64):
        bodies = []
        for i in range(nb):
            g = games[i % len(games)]
            mv = g["moves"].split()
            bodies.append(B.AcquireResponseBody(f"m{i}", g["position"], " ".join(mv[:20 + (i % 40)]), work="move"))
        for _ in range(20):
            stub.go(bodies)
        ts = []
        for _ in range(300):
            t = time.perf_counter()
            r = stub.go(bodies)
            ts.append((time.perf_counter() - t) * 1e3)
        assert not any(isinstance(x, B.PositionFailed) for x in r)
        out[f"{nb}_batches_ms_median"] = round(statistics.median(ts), 4)
        out[f"{nb}_children"] = sum(x[0].nodes for x in r)
finally:
    actor.close()
print(json.dumps(out))
