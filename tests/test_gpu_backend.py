"""fnnue_backend on the GPU: whole acquired batches through the actor
(device expansion + CHAIN evaluation) against the CPU oracles on the host
builder's positions, bit-exact; crazyhouse / atomic batches on their variant
nets ([ref] src/queue.rs:530-539, src/assets.rs:384-391); games that end on
the board answered as the engine answers them (mate 0 / cp 0, no best move,
[ref] src/stockfish.rs:359-376, 418-425); per-batch PositionFailed isolation
([ref] src/queue.rs:207-213); move work = one-ply search over the legal
children (mates first); skipPositions; concurrent callers on the capacity-1
channel."""
import json
import os
import threading

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from fishnet_amd import backend as B
from oracle.oracle import OracleNet, VariantOracleNet
from tests.conftest import ROOT, net_bytes

pytestmark = pytest.mark.gpu

GAMES = json.load(open(os.path.join(ROOT, "tests", "golden", "wcc_games.json")))["games"]
START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
ZH_START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1"
C960 = "bqnb1rkr/pp3ppp/3ppn2/2p5/5P2/P2P4/NPP1P1PP/BQ1BNRKR w HFhf - 2 9"
ZH, AT = N.VARIANT_CRAZYHOUSE, N.VARIANT_ATOMIC
FOOLS_MATE = "f2f3 e7e5 g2g4 d8h4"
STALEMATE = ("7k/5Q2/5K2/8/8/8/8/8 w - - 0 1", "f6g6")
ATOMIC_WIN = "g1f3 e7e6 f3g5 f8e7 g5f7"  # Nxf7 explodes the black king


@pytest.fixture(scope="module")
def chan():
    data = net_bytes(1, 1024, 0)
    zh = F.synthesize_variant_net(5, 512, ZH)
    at = F.synthesize_variant_net(6, 512, AT)
    stub, actor = B.channel(F.Net.from_bytes(data), 0, crazyhouse=F.Net.from_bytes_variant(zh, ZH),
                            atomic=F.Net.from_bytes_variant(at, AT))
    yield stub, {0: OracleNet(data), ZH: VariantOracleNet(zh, ZH), AT: VariantOracleNet(at, AT)}
    actor.close()


def expect(on, fen, moves, variant=0):
    pos = F.game_positions(fen, moves) if variant == 0 else F.game_vpositions(variant, fen, moves)
    ps, po, rc = on[variant].eval_packed(pos, threads=8)
    assert rc == 0
    return ps, po


def cp(ps, po, norm=361):
    v = int((int(ps) + int(po)) / 16)  # C truncation
    return int(v * 100 / norm)


def check_rows(on, body, rows, variant=0):
    """Every ply against the oracle; the last ply of a game that ended on the
    board as the engine answers it."""
    ps, po = expect(on, body.position, body.moves, variant)
    assert [r.position_id for r in rows] == list(range(len(ps)))
    assert [r.psqt for r in rows] == ps.tolist()
    assert [r.positional for r in rows] == po.tolist()
    end = F.game_end(body.position, body.moves, variant)
    for k, r in enumerate(rows):
        if k == len(rows) - 1 and end & F.END_NO_MOVES:
            mated = bool(end & (F.END_CHECK | F.END_EXTINCT))
            assert (r.score.kind, r.score.value, r.depth, r.nodes) == ("mate" if mated else "cp", 0, 0, 0)
            assert r.best_move is None
        else:
            assert (r.score.kind, r.score.value, r.depth, r.nodes) == ("cp", cp(ps[k], po[k]), 0, 1)
    return end


def test_analysis_batches_match_oracle(chan):
    stub, on = chan
    bodies = [B.AcquireResponseBody(str(g["id"]), g["position"], g["moves"]) for g in GAMES[:40]]
    bodies.append(B.AcquireResponseBody("c960", C960, F.random_game(7, C960, 60)))
    bodies.append(B.AcquireResponseBody("root-only", START, ""))
    res = stub.go(bodies)
    assert len(res) == len(bodies)
    for b, rows in zip(bodies, res):
        assert not isinstance(rows, B.PositionFailed), rows
        check_rows(on, b, rows)


def test_games_that_end_on_the_board(chan):
    """Checkmate -> mate 0, stalemate -> cp 0 on the last ply (and a root that
    is already mated), as Stockfish answers `go` there; JSON {"mate":0}."""
    stub, on = chan
    bodies = [B.AcquireResponseBody("mate", START, FOOLS_MATE),
              B.AcquireResponseBody("stalemate", STALEMATE[0], STALEMATE[1], variant="fromPosition"),
              B.AcquireResponseBody("mated-root", "rnb1kbnr/pppp1ppp/8/4p3/6Pq/5P2/PPPPP2P/RNBQKBNR w KQkq - 1 3", "")]
    res = stub.go(bodies)
    ends = [check_rows(on, b, rows) for b, rows in zip(bodies, res)]
    assert ends == [F.END_NO_MOVES | F.END_CHECK, F.END_NO_MOVES, F.END_NO_MOVES | F.END_CHECK]
    assert res[0][-1].score == B.Score("mate", 0) and res[1][-1].score == B.Score("cp", 0)
    parts = json.loads(B.into_analysis(res[0]))
    assert parts[-1]["score"] == {"mate": 0} and parts[-1]["depth"] == 0 and parts[-2]["score"].keys() == {"cp"}


def test_variant_analysis_batches(chan):
    """Crazyhouse and atomic batches on their own nets, every ply against the
    variant oracle; atomic games that end by an explosion answer mate 0 there
    (the kingless last ply no longer fails the batch)."""
    stub, on = chan
    bodies, kinds = [], []
    for i in range(24):
        for variant, name, fen in ((ZH, "crazyhouse", ZH_START), (AT, "atomic", START)):
            moves = F.random_vgame(1000 + i, variant, fen, 30 + 9 * i)
            bodies.append(B.AcquireResponseBody(f"{name}{i}", fen, moves, variant=name))
            kinds.append(variant)
    bodies.append(B.AcquireResponseBody("boom", START, ATOMIC_WIN, variant="atomic"))
    kinds.append(AT)
    bodies.append(B.AcquireResponseBody("chess", START, "e2e4 e7e5"))
    kinds.append(0)
    res = stub.go(bodies)
    extinct = 0
    for b, rows, variant in zip(bodies, res, kinds):
        assert not isinstance(rows, B.PositionFailed), (b.batch_id, rows)
        end = check_rows(on, b, rows, variant)
        extinct += bool(end & F.END_EXTINCT)
    assert extinct >= 2  # the explicit one and random games that ended by an explosion
    assert res[-2][-1].score == B.Score("mate", 0) and (res[-2][-1].psqt, res[-2][-1].positional) == (0, 0)


def test_failed_batches_are_isolated(chan):
    stub, on = chan
    g = GAMES[0]
    good = B.AcquireResponseBody("good", g["position"], g["moves"])
    bodies = [
        B.AcquireResponseBody("badmove", START, "e2e4 e7e5 e1e3"),
        good,
        B.AcquireResponseBody("badfen", "rnbqkbnr/pppppppp/8/8 w", "e2e4"),
        B.AcquireResponseBody("anti", START, "e2e4", variant="antichess"),
        B.AcquireResponseBody("mpv", START, "e2e4", multipv=3),
        B.AcquireResponseBody("threekings", "4k3/8/8/8/8/8/8/K3K3 w - - 0 1", ""),
        B.AcquireResponseBody("good2", START, "d2d4 d7d5 c2c4"),
        B.AcquireResponseBody("zhbad", ZH_START, "e2e4 P@e4", variant="crazyhouse"),
        B.AcquireResponseBody("zhgood", ZH_START, "e2e4 d7d5 e4d5 d8d5 P@e4", variant="crazyhouse"),
    ]
    res = stub.go(bodies)
    codes = {b.batch_id: (r.code if isinstance(r, B.PositionFailed) else 0) for b, r in zip(bodies, res)}
    assert codes["badmove"] == -8 and codes["badfen"] == -9 and codes["zhbad"] == -8
    assert codes["anti"] == -4 and codes["mpv"] == 0  # MultiPV: answered in the matrix form (one line)
    mpv = res[4]
    assert len(mpv) == 2 and all(r.matrix for r in mpv)
    ps, po = expect(on, START, "e2e4")
    assert [r.psqt for r in mpv] == ps.tolist() and [r.positional for r in mpv] == po.tolist()
    m = json.loads(B.into_analysis(mpv))
    assert m[0]["pv"] == [[[]]] and m[0]["score"] == [[{"cp": mpv[0].score.value}]] and m[0]["depth"] == 0
    assert codes["threekings"] != 0
    assert codes["good"] == 0 and codes["good2"] == 0 and codes["zhgood"] == 0
    for i in (1, 6):
        check_rows(on, bodies[i], res[i])
    check_rows(on, bodies[8], res[8], ZH)
    with pytest.raises(B.PositionFailed):
        stub.go_one(bodies[0])


def test_variant_batch_without_its_net():
    """A chess-only backend fails crazyhouse / atomic batches (FNNUE_E_ARCH)
    and evaluates the chess ones; a net in the wrong slot is refused."""
    data = net_bytes(1, 256, 0)
    stub, actor = B.channel(F.Net.from_bytes(data), 0)
    try:
        res = stub.go([B.AcquireResponseBody("zh", ZH_START, "e2e4", variant="crazyhouse"),
                       B.AcquireResponseBody("at", START, "e2e4", variant="atomic"),
                       B.AcquireResponseBody("std", START, "e2e4")])
        assert res[0].code == -4 and res[1].code == -4 and not isinstance(res[2], B.PositionFailed)
    finally:
        actor.close()
    with pytest.raises(F.FnnueError) as e:
        B.channel(None, 0, crazyhouse=F.Net.from_bytes(data))
    assert e.value.name == "FNNUE_E_ARCH"


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


def search1(on, fen, moves, variant=0):
    """The one-ply search the backend runs, restated: mates first, stalemates
    0, else -v(child); first maximum."""
    if variant == 0:
        pos, off = F.game_children(fen, moves)
    else:
        pos, off = F.game_vchildren(variant, fen, moves)
    kids = pos[off[-2] + 1: off[-1]]
    ps, po, rc = on[variant].eval_packed(kids, threads=8)
    return kids, ps, po


def test_move_work_best_child(chan):
    stub, on = chan
    for k, g in enumerate(GAMES[:6]):
        mv = " ".join(g["moves"].split()[: 10 + 7 * k])
        body = B.AcquireResponseBody(f"m{k}", g["position"], mv, work="move")
        (r,) = stub.go_one(body)
        kids, ps, po = search1(on, g["position"], mv)
        vals = [-int((int(a) + int(b)) / 16) for a, b in zip(ps, po)]
        best = int(np.argmax(vals))  # first maximum, as the backend (no mate in one in these positions)
        assert r.nodes == len(kids) and r.depth == 1
        assert r.score == B.Score("cp", int(vals[best] * 100 / 361))
        after = F.game_positions(g["position"], (mv + " " + r.best_move).strip())[-1]
        assert np.array_equal(after, kids[best]), (r.best_move, best)


def test_move_work_mates_and_terminal_roots(chan):
    """Move work: a mate in one is played (score mate 1) whatever the NNUE
    says about the other children; atomic: the exploding capture; a root
    with no legal move has no best move (mate 0 / cp 0)."""
    stub, on = chan
    bodies = [B.AcquireResponseBody("m1", START, "f2f3 e7e5 g2g4", work="move"),
              B.AcquireResponseBody("at1", START, "g1f3 e7e6 f3g5 f8e7", work="move", variant="atomic"),
              B.AcquireResponseBody("mated", START, FOOLS_MATE, work="move"),
              B.AcquireResponseBody("stale", STALEMATE[0], STALEMATE[1], work="move"),
              B.AcquireResponseBody("boom", START, ATOMIC_WIN, work="move", variant="atomic"),
              B.AcquireResponseBody("zh", ZH_START, "e2e4 d7d5 e4d5 d8d5", work="move", variant="crazyhouse")]
    res = [r[0] for r in stub.go(bodies)]
    assert res[0].best_move == "d8h4" and res[0].score == B.Score("mate", 1) and res[0].depth == 1
    assert res[1].score == B.Score("mate", 1)
    assert F.game_end(START, bodies[1].moves + " " + res[1].best_move, AT) & F.END_EXTINCT
    for r, kind in ((res[2], "mate"), (res[3], "cp"), (res[4], "mate")):
        assert r.best_move is None and r.score == B.Score(kind, 0) and (r.depth, r.nodes) == (0, 0)
    kids, ps, po = search1(on, ZH_START, bodies[5].moves, ZH)
    vals = [-int((int(a) + int(b)) / 16) for a, b in zip(ps, po)]
    assert res[5].nodes == len(kids) > 0
    assert res[5].score == B.Score("cp", int(max(vals) * 100 / 361))
    after = F.game_vpositions(ZH, ZH_START, bodies[5].moves + " " + res[5].best_move)[-1]
    assert np.array_equal(after, kids[int(np.argmax(vals))])


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
            check_rows(on, b, rows)


def test_two_channels_on_one_device_at_once(chan):
    """Two channels (fishnet: two workers, each its own engine) on the same
    device, driven from two threads at once, each call a different mix of
    chess, Chess960 and variant batches: each channel's answers equal the same
    batches answered alone on the module's channel, and sampled plies equal the
    oracle (the channels share no buffers, streams or error words)."""
    stub, on = chan
    data = net_bytes(1, 1024, 0)
    stub2, actor2 = B.channel(F.Net.from_bytes(data), 0,
                              crazyhouse=F.Net.from_bytes_variant(F.synthesize_variant_net(5, 512, ZH), ZH),
                              atomic=F.Net.from_bytes_variant(F.synthesize_variant_net(6, 512, AT), AT))
    try:
        mk = lambda off: ([B.AcquireResponseBody(f"g{off + i}", GAMES[(off + i) % len(GAMES)]["position"],
                                                 GAMES[(off + i) % len(GAMES)]["moves"]) for i in range(300)]
                          + [B.AcquireResponseBody(f"c{off}", C960, F.random_game(off + 3, C960, 80), variant="chess960"),
                             B.AcquireResponseBody(f"z{off}", ZH_START, F.random_vgame(off + 4, ZH, ZH_START, 90),
                                                   variant="crazyhouse")])
        sets = [mk(0), mk(300)]
        alone = [stub.go(s) for s in sets]
        out = [[None] * 6 for _ in range(2)]

        def worker(t):
            st = stub if t == 0 else stub2
            for r in range(6):
                out[t][r] = st.go(sets[t])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        key = lambda r: (r.position_id, r.score, r.psqt, r.positional, r.skipped)
        for t in range(2):
            for r in range(6):
                for b, x, y in zip(sets[t], alone[t], out[t][r]):
                    assert not isinstance(y, B.PositionFailed), (t, r, b.batch_id)
                    assert [key(q) for q in x] == [key(q) for q in y], (t, r, b.batch_id)
            for i in range(0, 300, 37):
                check_rows(on, sets[t][i], out[t][5][i])
            check_rows(on, sets[t][301], out[t][5][301], ZH)
    finally:
        actor2.close()


# Positions where a UCI token's meaning is subtle: castling both ways and in
# Chess960 (king already on its destination, rook beside it), en passant
# (legal, and exposing the own king), promotions with and without capture,
# checks, pins.
TOKEN_FENS = [
    START,
    "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
    "r3k2r/p1ppqpb1/bn2pnp1/3PN3/Pp2P3/2N2Q1p/1PPBBPPP/R3K2R b KQkq a3 0 1",
    "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
    "8/8/8/KPp4r/8/8/8/4k3 w - c6 0 1",
    "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1",
    "rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8",
    "4k3/1P6/8/8/8/8/6p1/4K2R b K - 0 1",
    C960,
    "1rk1r3/pppppppp/8/8/8/8/PPPPPPPP/1RK1R3 w BEbe - 0 1",
    "r5kr/pppppppp/8/8/8/8/PPPPPPPP/R5KR w HAha - 0 1",
    "4k3/8/8/8/8/8/4q3/4K2R w K - 0 1",
    "r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1",
    "r3k2r/8/8/8/8/8/8/R3K2R b KQkq - 0 1",
]


def _stm_squares(fen):
    pos = F.pos_from_fen(fen)
    stm = int(pos[32])
    sq = []
    for s in range(64):
        pc = (int(pos[s >> 1]) >> (4 * (s & 1))) & 15
        if pc and (pc >> 3) == stm:
            sq.append(s)
    return sq


def _go_both_replays(stub, bodies):
    """One go() over all the bodies (more than 1024 games: one replay wave per
    game) and the same bodies in go() calls of 1000 (the two-wave replay,
    ADVICE r05): the same batches fail with the same codes, the others give
    the same results."""
    assert len(bodies) > 1024
    res = stub.go(bodies)
    for lo in range(0, len(bodies), 1000):
        part = stub.go(bodies[lo:lo + 1000])
        for i, (a, r) in enumerate(zip(res[lo:lo + 1000], part)):
            if isinstance(a, B.PositionFailed):
                assert isinstance(r, B.PositionFailed) and r.code == a.code, (bodies[lo + i].batch_id, r)
            else:
                assert not isinstance(r, B.PositionFailed), (bodies[lo + i].batch_id, r)
                assert [(x.psqt, x.positional, x.score) for x in a] == [(x.psqt, x.positional, x.score) for x in r]
    return res


def test_every_token_matches_the_host_builder(chan):
    """Every from-square of the side to move x every destination x {none,
    q, n, r, b, k, Q} as a one-move analysis batch: the device replay accepts
    exactly the tokens the host builder (board.cpp parse_uci, perft-pinned)
    accepts, and the position it plays to evaluates like the host's."""
    stub, on = chan
    name = lambda s: "abcdefgh"[s & 7] + "12345678"[s >> 3]
    bodies, host = [], []
    for fi, fen in enumerate(TOKEN_FENS):
        for f in _stm_squares(fen):
            for t in range(64):
                for p in ("", "q", "n", "r", "b", "k", "Q"):
                    tok = name(f) + name(t) + p
                    try:
                        pos = F.game_positions(fen, tok)
                    except F.FnnueError:
                        pos = None
                    bodies.append(B.AcquireResponseBody(f"{fi}:{tok}", fen, tok))
                    host.append(pos)
    res = _go_both_replays(stub, bodies)
    ok = [i for i, p in enumerate(host) if p is not None]
    assert 200 < len(ok) < len(host)
    for i, (b, r) in enumerate(zip(bodies, res)):
        assert isinstance(r, B.PositionFailed) == (host[i] is None), (b.batch_id, r)
    after = np.stack([host[i][1] for i in ok])
    ps, po, rc = on[0].eval_packed(after, threads=8)
    assert rc == 0
    got = np.array([(res[i][1].psqt, res[i][1].positional) for i in ok])
    assert np.array_equal(got[:, 0], ps) and np.array_equal(got[:, 1], po)


VTOKEN_FENS = [
    (ZH, "crazyhouse", ZH_START),
    (ZH, "crazyhouse", "r1bqk2r/ppp2ppp/2n5/2b5/2B5/5N2/PPP2PPP/RNBQK2R[PNPnp] w KQkq - 0 1"),
    (ZH, "crazyhouse", "4k3/1P6/8/3Pp3/8/8/6p1/R3K2R[Nn] w KQ e6 0 1"),
    (ZH, "crazyhouse", "r3k2r/8/8/8/8/8/8/R3K2R[P] b KQkq - 0 1"),
    (AT, "atomic", START),
    (AT, "atomic", "rnbqkbnr/pppp1ppp/8/4p3/4P3/5N2/PPPP1PPP/RNBQKB1R b KQkq - 1 2"),
    (AT, "atomic", "8/8/8/3pP3/8/8/3Kk3/8 w - d6 0 1"),
    (AT, "atomic", "r3k2r/pppq1ppp/8/3pN3/8/8/PPPP1PPP/R3K2R w KQkq - 0 1"),
]


def test_every_variant_token_matches_the_host_builder(chan):
    """As the chess test, for crazyhouse (drops of every piece letter on every
    square, promotions, pockets) and atomic (explosions, king captures,
    adjacent kings, en passant): device acceptance and the position played
    equal vboard.h's host replay."""
    stub, on = chan
    name = lambda s: "abcdefgh"[s & 7] + "12345678"[s >> 3]
    bodies, host, kinds = [], [], []
    for fi, (variant, vname, fen) in enumerate(VTOKEN_FENS):
        pos = F.vpos_from_fen(variant, fen)
        stm = int(pos[32])
        own = [s for s in range(64) if ((int(pos[s >> 1]) >> (4 * (s & 1))) & 15) and
               (((int(pos[s >> 1]) >> (4 * (s & 1))) & 15) >> 3) == stm]
        toks = [name(f) + name(t) + p for f in own for t in range(64) for p in ("", "q", "n", "k", "Q")]
        if variant == ZH:
            toks += [c + "@" + name(t) for c in "PNBRQKpq" for t in range(64)]
        for tok in toks:
            try:
                p = F.game_vpositions(variant, fen, tok)
            except F.FnnueError:
                p = None
            bodies.append(B.AcquireResponseBody(f"{fi}:{tok}", fen, tok, variant=vname))
            host.append(p)
            kinds.append(variant)
    res = _go_both_replays(stub, bodies)
    for i, (b, r) in enumerate(zip(bodies, res)):
        assert isinstance(r, B.PositionFailed) == (host[i] is None), (b.batch_id, r)
    for variant in (ZH, AT):
        ok = [i for i, p in enumerate(host) if p is not None and kinds[i] == variant]
        assert len(ok) > 50
        after = np.stack([host[i][1] for i in ok])
        ps, po, rc = on[variant].eval_packed(after, threads=8)
        assert rc == 0
        got = np.array([(res[i][1].psqt, res[i][1].positional) for i in ok])
        assert np.array_equal(got[:, 0], ps) and np.array_equal(got[:, 1], po)


def test_pieces_with_failures_in_between(monkeypatch):
    """Small pieces (FNNUE_BACKEND_PIECE_PLIES = 1024): a call spans several
    pieces per net, overlapping uploads / replays / evaluations / fills; a
    builder failure and an evaluator failure (a position with more than 32
    pieces, the evaluator's sticky error word) inside middle pieces fail their
    own batches only, every other batch bit-exact, move work in the net's last
    piece."""
    monkeypatch.setenv("FNNUE_BACKEND_PIECE_PLIES", "1024")
    data = net_bytes(1, 1024, 0)
    zh = F.synthesize_variant_net(5, 512, ZH)
    stub, actor = B.channel(F.Net.from_bytes(data), 0, crazyhouse=F.Net.from_bytes_variant(zh, ZH))
    on = {0: OracleNet(data), ZH: VariantOracleNet(zh, ZH)}
    crowded = "rnbqkbnr/pppppppp/pppppppp/8/8/PPPPPPPP/PPPPPPPP/RNBQKBNR w - - 0 1"
    try:
        bodies, kinds = [], []
        for i, g in enumerate(GAMES[:80]):
            bodies.append(B.AcquireResponseBody(str(g["id"]), g["position"], g["moves"]))
            kinds.append(0)
            if i in (25, 50):
                bodies.append(B.AcquireResponseBody(f"bad{i}", START, "e2e4 e7e5 e1e3"))
                kinds.append(-1)
            if i == 40:
                bodies.append(B.AcquireResponseBody("crowded", crowded, "a3a4"))
                kinds.append(-1)
            if i % 8 == 0:
                bodies.append(B.AcquireResponseBody(f"zh{i}", ZH_START, F.random_vgame(77 + i, ZH, ZH_START, 60 + i),
                                                    variant="crazyhouse"))
                kinds.append(ZH)
        bodies.append(B.AcquireResponseBody("mv", GAMES[0]["position"], " ".join(GAMES[0]["moves"].split()[:20]),
                                            work="move"))
        kinds.append(-2)
        res = stub.go(bodies)
        st = B.last_stats(actor)
        assert st["pieces"] >= 5, st
        assert st["rebuilds"] >= 2, st
        for b, rows, kind in zip(bodies, res, kinds):
            if kind == -1:
                assert isinstance(rows, B.PositionFailed), b.batch_id
            elif kind == -2:
                kids, ps, po = search1(on, b.position, b.moves)
                vals = [-int((int(x) + int(y)) / 16) for x, y in zip(ps, po)]
                assert rows[0].nodes == len(kids) and rows[0].score == B.Score("cp", int(max(vals) * 100 / 361))
            else:
                assert not isinstance(rows, B.PositionFailed), (b.batch_id, rows)
                check_rows(on, b, rows, kind)
        # the same call again: pieces and buffers reused, results unchanged
        again = stub.go(bodies)
        for a, r in zip(res, again):
            if isinstance(a, B.PositionFailed):
                assert isinstance(r, B.PositionFailed) and r.code == a.code
            else:
                assert [(x.psqt, x.positional, x.score) for x in a] == [(x.psqt, x.positional, x.score) for x in r]
    finally:
        actor.close()


def test_move_work_isolation(chan):
    """move-work roots whose children the evaluator would reject
    (a chess root with more than 32 pieces; crazyhouse roots whose pockets
    exceed the feature set's limits) fail their own batches with
    FNNUE_E_POSITION, checked on the host before anything reaches the device;
    good analysis and move batches of the same go() are bit-exact
    ([ref] src/queue.rs:207-213: only the failed batch is dropped)."""
    stub, on = chan
    crowded = "rnbqkbnr/pppppppp/pppppppp/8/8/PPPPPPPP/PPPPPPPP/RNBQKBNR w - - 0 1"
    zh_over = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[QQ] w KQkq - 0 1"       # 34 pieces with the hand
    zh_pawns = "4k3/8/8/8/8/8/8/4K3[PPPPPPPPPPPPPPPPPPPPP] w - - 0 1"               # 21 pawns of one type in hand
    g0, g1 = GAMES[5], GAMES[6]
    mv0 = " ".join(g0["moves"].split()[:24])
    bodies = [
        B.AcquireResponseBody("a0", g0["position"], g0["moves"]),
        B.AcquireResponseBody("bad-crowded", crowded, "", work="move"),
        B.AcquireResponseBody("m0", g0["position"], mv0, work="move"),
        B.AcquireResponseBody("bad-zh", zh_over, "", work="move", variant="crazyhouse"),
        B.AcquireResponseBody("zh-good", ZH_START, "e2e4 d7d5 e4d5", work="move", variant="crazyhouse"),
        B.AcquireResponseBody("bad-zh-pawns", zh_pawns, "", work="move", variant="crazyhouse"),
        B.AcquireResponseBody("a1", g1["position"], g1["moves"]),
        B.AcquireResponseBody("zh-a", ZH_START, F.random_vgame(31, ZH, ZH_START, 50), variant="crazyhouse"),
    ]
    res = stub.go(bodies)
    codes = {b.batch_id: (r.code if isinstance(r, B.PositionFailed) else 0) for b, r in zip(bodies, res)}
    assert codes == {"a0": 0, "bad-crowded": -6, "m0": 0, "bad-zh": -6, "zh-good": 0, "bad-zh-pawns": -6,
                     "a1": 0, "zh-a": 0}, codes
    check_rows(on, bodies[0], res[0])
    check_rows(on, bodies[6], res[6])
    check_rows(on, bodies[7], res[7], ZH)
    for i, variant in ((2, 0), (4, ZH)):
        (r,) = res[i]
        kids, ps, po = search1(on, bodies[i].position, bodies[i].moves, variant)
        vals = [-int((int(a) + int(b)) / 16) for a, b in zip(ps, po)]
        assert r.nodes == len(kids) and r.score == B.Score("cp", int(max(vals) * 100 / 361)), bodies[i].batch_id


def _long_game(seed, plies):
    moves = F.random_game(seed, START, plies).split()
    assert len(moves) > 200, len(moves)
    return moves


@pytest.mark.parametrize("fillers", [0, 1100])  # <= 1024 games: the two-wave replay; more: one wave per game
def test_failures_in_late_replay_windows(chan, fillers):
    """Illegal moves in the replay's third and fifth 64-move windows (ADVICE
    r05: the two-wave kernel's double buffers, window count and bad-move
    report past the first windows) fail exactly their batches; the long good
    games around them are bit-exact, in both replay kernels."""
    stub, on = chan
    good = [_long_game(100 + s, 320) for s in range(3)]
    bad3 = list(good[0][:150]) + ["b2b2"] + list(good[0][150:])      # window 2 (plies 129-192)
    bad5 = list(good[1][:270]) + ["a1a1"] + list(good[1][270:])      # window 4 (plies 257-320)
    short = list(good[2][:200]) + ["zz"]                              # unparsable token in window 3
    bodies = [B.AcquireResponseBody("g0", START, " ".join(good[0])),
              B.AcquireResponseBody("bad3", START, " ".join(bad3)),
              B.AcquireResponseBody("g1", START, " ".join(good[1])),
              B.AcquireResponseBody("bad5", START, " ".join(bad5)),
              B.AcquireResponseBody("g2", START, " ".join(good[2])),
              B.AcquireResponseBody("short", START, " ".join(short))]
    bodies += [B.AcquireResponseBody(f"f{i}", START, "e2e4 e7e5" if i % 2 else "d2d4") for i in range(fillers)]
    res = stub.go(bodies)
    # the three rejected games are dropped in one extra pass (each game's flag
    # byte says it failed), not one pass per failure
    assert B.last_stats(stub._actor)["rebuilds"] == 1
    for b, r in zip(bodies, res):
        if b.batch_id in ("bad3", "bad5", "short"):
            assert isinstance(r, B.PositionFailed) and r.code == -8, (b.batch_id, r)
        else:
            assert not isinstance(r, B.PositionFailed), (b.batch_id, r)
    for i in (0, 2, 4):
        check_rows(on, bodies[i], res[i])
    if fillers:
        check_rows(on, bodies[6], res[6])
        check_rows(on, bodies[7], res[7])


def test_go_timeout_breaks_the_channel():
    """The worker's time budget ([ref] src/main.rs:316, 343-351; the engine is
    dropped on expiry, src/stockfish.rs:138): a 16384-batch go() with a 1 ms
    budget returns FNNUE_E_TIMEOUT well within a second, without waiting for
    the device; the batches it had not answered say FNNUE_E_TIMEOUT; the next
    go() on the broken channel fails fast; freeing it does not hang; a new
    channel on the same device answers bit-exact against the oracle."""
    import time
    data = net_bytes(1, 1024, 0)
    on = {0: OracleNet(data)}
    bodies = [B.AcquireResponseBody(f"b{i}", GAMES[i % len(GAMES)]["position"], GAMES[i % len(GAMES)]["moves"])
              for i in range(16384)]
    # answered without the device: their answers stand after a timeout
    hostonly = [B.AcquireResponseBody("allskip", START, "e2e4", skip_positions=[0, 1]),
                B.AcquireResponseBody("mated", START, FOOLS_MATE, work="move")]
    stub, actor = B.channel(F.Net.from_bytes(data), 0)
    try:
        warm = stub.go(bodies[:64])
        assert not any(isinstance(r, B.PositionFailed) for r in warm)
        with pytest.raises(F.FnnueError) as e:
            stub.go(hostonly[:1] + bodies + hostonly[1:], timeout_ms=1)
        assert e.value.name == "FNNUE_E_TIMEOUT", e.value
        assert stub.last_call_s < 1.0, stub.last_call_s
        rc = stub.last_batch_rc
        assert set(np.unique(rc).tolist()) <= {0, -11} and (rc == -11).sum() > 0
        assert rc[0] == 0 and rc[-1] == 0, (rc[0], rc[-1])
        with pytest.raises(F.FnnueError) as e:
            stub.go(bodies[:4])
        assert e.value.name == "FNNUE_E_TIMEOUT" and stub.last_call_s < 0.05
        assert (stub.last_batch_rc == -11).all()
    finally:
        t = time.perf_counter()
        actor.close()
        assert time.perf_counter() - t < 5.0
    stub2, actor2 = B.channel(F.Net.from_bytes(data), 0, timeout_ms=30000)
    try:
        res = stub2.go(bodies[:300])
        for b, rows in zip(bodies[:300], res):
            assert not isinstance(rows, B.PositionFailed), rows
        for i in range(0, 300, 7):
            check_rows(on, bodies[i], res[i])
        big = stub2.go(bodies)  # the full call within its budget on the new channel
        assert not any(isinstance(r, B.PositionFailed) for r in big)
        for i in range(0, 16384, 911):
            check_rows(on, bodies[i], big[i])
    finally:
        actor2.close()


def test_compact_form_equals_full_records(chan):
    """fnnue_backend_go_compact (16 B per position + 24 B per batch) carries
    exactly what the full PositionResponse records do, for every kind of
    batch: analysis (chess, Chess960, crazyhouse, atomic), games ending in
    mate / stalemate / explosion, skipPositions and all-skipped batches,
    MultiPV, move work (best child, mate in one, mated and stalemated roots),
    and failing batches with the same codes."""
    stub, on = chan
    bodies = [B.AcquireResponseBody(str(g["id"]), g["position"], g["moves"]) for g in GAMES[:30]]
    bodies += [B.AcquireResponseBody("c960", C960, F.random_game(7, C960, 60), variant="chess960"),
               B.AcquireResponseBody("mate", START, FOOLS_MATE),
               B.AcquireResponseBody("stalemate", STALEMATE[0], STALEMATE[1], variant="fromPosition"),
               B.AcquireResponseBody("boom", START, ATOMIC_WIN, variant="atomic"),
               B.AcquireResponseBody("zh", ZH_START, F.random_vgame(3, ZH, ZH_START, 70), variant="crazyhouse"),
               B.AcquireResponseBody("skip", GAMES[3]["position"], GAMES[3]["moves"], skip_positions=[0, 2, 5]),
               B.AcquireResponseBody("allskip", START, "e2e4", skip_positions=[0, 1]),
               B.AcquireResponseBody("mpv", START, "e2e4 e7e5", multipv=2),
               B.AcquireResponseBody("mv", GAMES[1]["position"], " ".join(GAMES[1]["moves"].split()[:30]), work="move"),
               B.AcquireResponseBody("m1", START, "f2f3 e7e5 g2g4", work="move"),
               B.AcquireResponseBody("mated", START, FOOLS_MATE, work="move"),
               B.AcquireResponseBody("stale", STALEMATE[0], STALEMATE[1], work="move"),
               B.AcquireResponseBody("zhmv", ZH_START, "e2e4 d7d5 e4d5 d8d5", work="move", variant="crazyhouse"),
               B.AcquireResponseBody("badmove", START, "e2e4 e7e5 e1e3"),
               B.AcquireResponseBody("anti", START, "e2e4", variant="antichess")]
    full = stub.go(bodies)
    comp = stub.go_compact(bodies)
    key = lambda r: (r.position_id, r.score, r.psqt, r.positional, r.depth, r.nodes, r.best_move, r.skipped, r.matrix)
    for b, f, c in zip(bodies, full, comp):
        if isinstance(f, B.PositionFailed):
            assert isinstance(c, B.PositionFailed) and c.code == f.code, b.batch_id
            continue
        assert [key(r) for r in f] == [key(r) for r in c], b.batch_id
        live = [r for r in c if not r.skipped]  # skipped rows carry no time (a skipped row may come first)
        assert all(r.time_ms == live[0].time_ms and r.nps == live[0].nps for r in live), b.batch_id
    for i in range(30):
        check_rows(on, bodies[i], comp[i])
