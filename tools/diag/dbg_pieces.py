import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FNNUE_BACKEND_PIECE_PLIES"] = "1024"
import fishnet_amd as F
from fishnet_amd import backend as B
from tests.test_gpu_backend import GAMES, START, ZH_START, ZH
from tests.conftest import net_bytes
data = net_bytes(1, 1024, 0)
stub, actor = B.channel(F.Net.from_bytes(data), 0)
crowded = "rnbqkbnr/pppppppp/pppppppp/8/8/PPPPPPPP/PPPPPPPP/RNBQKBNR w - - 0 1"
bodies = []
for i, g in enumerate(GAMES[:80]):
    bodies.append(B.AcquireResponseBody(str(g["id"]), g["position"], g["moves"]))
    if i in (25, 50):
        bodies.append(B.AcquireResponseBody(f"bad{i}", START, "e2e4 e7e5 e1e3"))
    if i == 40:
        bodies.append(B.AcquireResponseBody("crowded", crowded, "a3a4"))
for call in range(4):
    try:
        res = stub.go(bodies)
        print(call, B.last_stats(actor), [(b.batch_id, r.code) for b, r in zip(bodies, res) if isinstance(r, B.PositionFailed)], flush=True)
    except Exception as e:
        print(call, "ERR", e, flush=True)
actor.close()
