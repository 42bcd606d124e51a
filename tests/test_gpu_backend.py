"""fnnue_backend on the GPU: whole acquired batches through the actor
(device expansion + CHAIN evaluation) against the CPU oracle on the host
builder's positions, bit-exact; per-batch PositionFailed isolation
([ref] src/queue.rs:207-213); move work = 1-ply argmax over the legal
children; skipPositions; concurrent callers on the capacity-1 channel."""
import json
import os
import threading

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import backend as B
from oracle.oracle import OracleNet
from tests.conftest import ROOT, net_bytes

pytestmark = pytest.mark.gpu

GAMES = json.load(open(os.path.join(ROOT, "tests", "golden", "wcc_games.json")))["games"]
START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
C960 = "bqnb1rkr/pp3ppp/3ppn2/2p5/5P2/P2P4/NPP1P1PP/BQ1BNRKR w HFhf - 2 9"


@pytest.fixture(scope="module")
def chan():
    data = net_bytes(1, 1024, 0)
    stub, actor = B.channel(F.Net.from_bytes(data), 0)
    yield stub, OracleNet(data)
    actor.close()


def expect(on, fen, moves):
    pos = F.game_positions(fen, moves)
    ps, po, rc = on.eval_packed(pos, threads=8)
    assert rc == 0
    return ps, po


def cp(ps, po, norm=361):
    v = int((int(ps) + int(po)) / 16)  # C truncation
    return int(v * 100 / norm)


def test_analysis_batches_match_oracle(chan):
    stub, on = chan
    bodies = [B.AcquireResponseBody(str(g["id"]), g["position"], g["moves"]) for g in GAMES[:40]]
    bodies.append(B.AcquireResponseBody("c960", C960, F.random_game(7, C960, 60)))
    bodies.append(B.AcquireResponseBody("root-only", START, ""))
    res = stub.go(bodies)
    assert len(res) == len(bodies)
    for b, rows in zip(bodies, res):
        assert not isinstance(rows, B.PositionFailed), rows
        ps, po = expect(on, b.position, b.moves)
        assert [r.position_id for r in rows] == list(range(len(ps)))
        assert [r.psqt for r in rows] == ps.tolist()
        assert [r.positional for r in rows] == po.tolist()
        assert [r.score.value for r in rows] == [cp(a, c) for a, c in zip(ps, po)]
        assert all(r.depth == 0 and r.nodes == 1 and r.score.kind == "cp" for r in rows)


def test_failed_batches_are_isolated(chan):
    stub, on = chan
    g = GAMES[0]
    good = B.AcquireResponseBody("good", g["position"], g["moves"])
    bodies = [
        B.AcquireResponseBody("badmove", START, "e2e4 e7e5 e1e3"),
        good,
        B.AcquireResponseBody("badfen", "rnbqkbnr/pppppppp/8/8 w", "e2e4"),
        B.AcquireResponseBody("zh", START, "e2e4", variant="crazyhouse"),
        B.AcquireResponseBody("mpv", START, "e2e4", multipv=3),
        B.AcquireResponseBody("threekings", "4k3/8/8/8/8/8/8/K3K3 w - - 0 1", ""),
        B.AcquireResponseBody("good2", START, "d2d4 d7d5 c2c4"),
    ]
    res = stub.go(bodies)
    codes = {b.batch_id: (r.code if isinstance(r, B.PositionFailed) else 0) for b, r in zip(bodies, res)}
    assert codes["badmove"] == -8 and codes["badfen"] == -9
    assert codes["zh"] == -1 and codes["mpv"] == 0  # MultiPV: answered in the matrix form (one line)
    mpv = res[4]
    assert len(mpv) == 2 and all(r.matrix for r in mpv)
    ps, po = expect(on, START, "e2e4")
    assert [r.psqt for r in mpv] == ps.tolist() and [r.positional for r in mpv] == po.tolist()
    m = json.loads(B.into_analysis(mpv))
    assert m[0]["pv"] == [[[]]] and m[0]["score"] == [[{"cp": mpv[0].score.value}]] and m[0]["depth"] == 0
    assert codes["threekings"] != 0
    assert codes["good"] == 0 and codes["good2"] == 0
    for i in (1, 6):
        ps, po = expect(on, bodies[i].position, bodies[i].moves)
        assert [r.psqt for r in res[i]] == ps.tolist() and [r.positional for r in res[i]] == po.tolist()
    with pytest.raises(B.PositionFailed):
        stub.go_one(bodies[0])


def test_skip_positions_and_all_skipped(chan):
    stub, on = chan
    g = GAMES[3]
    n = len(g["moves"].split()) + 1
    skip = [0, 2, 5, n + 10]  # out-of-range ids are ignored (positions.get_mut)
    rows = stub.go_one(B.AcquireResponseBody("s", g["position"], g["moves"], skip_positions=skip))
    ps, po = expect(on, g["position"], g["moves"])
    for r in rows:
        if r.position_id in skip:
            assert r.skipped and r.score is None
        else:
            assert (r.psqt, r.positional) == (ps[r.position_id], po[r.position_id])
    parts = json.loads(B.into_analysis(rows))
    assert parts[0] == {"skipped": True} and parts[1]["score"]["cp"] == cp(ps[1], po[1])
    allskip = stub.go_one(B.AcquireResponseBody("all", START, "e2e4", skip_positions=[0, 1]))
    assert all(r.skipped for r in allskip)


def test_move_work_best_child(chan):
    stub, on = chan
    for k, g in enumerate(GAMES[:6]):
        mv = " ".join(g["moves"].split()[: 10 + 7 * k])
        body = B.AcquireResponseBody(f"m{k}", g["position"], mv, work="move")
        (r,) = stub.go_one(body)
        pos, off = F.game_children(g["position"], mv)
        kids = pos[off[-2] + 1: off[-1]]
        ps, po, rc = on.eval_packed(kids, threads=8)
        vals = [-int((int(a) + int(b)) / 16) for a, b in zip(ps, po)]
        best = int(np.argmax(vals))  # first maximum, as the backend
        assert r.nodes == len(kids) and r.depth == 1
        assert r.score.value == int(vals[best] * 100 / 361)
        after = F.game_positions(g["position"], (mv + " " + r.best_move).strip())[-1]
        assert np.array_equal(after, kids[best]), (r.best_move, best)


def test_concurrent_callers(chan):
    stub, on = chan
    bodies = [B.AcquireResponseBody(str(g["id"]), g["position"], g["moves"]) for g in GAMES[40:60]]
    out = [None] * 4

    def worker(t):
        out[t] = stub.go(bodies[t * 5:(t + 1) * 5])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for t in range(4):
        for b, rows in zip(bodies[t * 5:(t + 1) * 5], out[t]):
            ps, po = expect(on, b.position, b.moves)
            assert [r.psqt for r in rows] == ps.tolist() and [r.positional for r in rows] == po.tolist()
