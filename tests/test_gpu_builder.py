"""GPU tests of the device-side batch builder (fnnue_build_batch*, builder.hip):
record-for-record identical to the host builder (board.cpp, perft-checked,
SURVEY.md §8c), device perft against the published counts, and the error
behaviour of the host path (FEN / illegal move / capacity).  Run with -m gpu."""
import json
import os

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from tests.conftest import ROOT, net_bytes
from tests.positions import CHESS960, FENS, PERFT, START

pytestmark = pytest.mark.gpu

GAMES = json.load(open(os.path.join(ROOT, "tests", "golden", "wcc_games.json")))["games"]


@pytest.fixture(scope="module")
def ev():
    e = F.Evaluator(F.Net.from_bytes(net_bytes(7, 128, 0)), 0)
    yield e
    e.close()


def host_plies(games):
    pos = [F.game_positions(f, m) for f, m in games]
    off = np.concatenate([[0], np.cumsum([len(p) for p in pos])]).astype(np.uint32)
    return np.concatenate(pos), off


def host_children(games):
    pos, off, base = [], [0], 0
    for f, m in games:
        p, o = F.game_children(f, m)
        pos.append(p)
        off += list(base + o[1:].astype(np.int64))
        base += len(p)
    return np.concatenate(pos), np.array(off, dtype=np.uint32)


def random_games(n, plies, seed=11):
    fens = [START, CHESS960, FENS[1], "r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1",
            "1r2k1r1/pppppppp/8/8/8/8/PPPPPPPP/1R2K1R1 w GBgb - 0 1",
            "rnbqkbnr/ppp1p1pp/8/3pPp2/8/8/PPPP1PPP/RNBQKBNR w KQkq f6 0 3", "8/P6k/8/8/8/8/6Kp/8 w - - 0 1"]
    return [(fens[i % len(fens)], F.random_game(seed * 1000 + i, fens[i % len(fens)], plies)) for i in range(n)]


def test_wcc_games_plies_match_host(ev):
    games = [(g["position"], g["moves"]) for g in GAMES]
    pos, off = ev.build_batch(games, N.PLAYOUT_PLIES)
    hpos, hoff = host_plies(games)
    assert np.array_equal(off, hoff)
    assert np.array_equal(pos, hpos)


def test_wcc_games_children_match_host(ev):
    games = [(g["position"], g["moves"]) for g in GAMES[:40]]
    pos, off = ev.build_batch(games, N.PLAYOUT_CHILDREN)
    hpos, hoff = host_children(games)
    assert np.array_equal(off, hoff)
    assert np.array_equal(pos, hpos)


def test_random_games_chess960_ep_promotion_match_host(ev):
    games = random_games(300, 200)
    pos, off = ev.build_batch(games, N.PLAYOUT_PLIES)
    hpos, hoff = host_plies(games)
    assert np.array_equal(off, hoff) and np.array_equal(pos, hpos)
    pos, off = ev.build_batch(games[:60], N.PLAYOUT_CHILDREN)
    hpos, hoff = host_children(games[:60])
    assert np.array_equal(off, hoff) and np.array_equal(pos, hpos)


def test_standard_and_king_takes_rook_castling(ev):
    fen = "r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1"
    a, _ = ev.build_batch([(fen, "e1h1 e8a8")])
    b, _ = ev.build_batch([(fen, "e1g1 e8c8")])
    assert np.array_equal(a, b)
    assert np.array_equal(a, F.game_positions(fen, "e1g1 e8c8"))


def test_fens_without_moves(ev):
    games = [(f, "") for f in FENS]
    pos, off = ev.build_batch(games)
    assert list(np.diff(off)) == [1] * len(FENS)
    assert np.array_equal(pos, np.stack([F.pos_from_fen(f) for f in FENS]))


@pytest.mark.parametrize("fen,counts", PERFT)
def test_device_perft_known_answers(ev, fen, counts):
    for depth, expect in enumerate(counts, start=1):
        if depth <= 4:
            assert ev.perft_device(fen, depth) == expect, (fen, depth)


def test_device_perft_chess960(ev):
    assert [ev.perft_device(CHESS960, d) for d in (1, 2, 3)] == [21, 528, 12189]


def test_illegal_move_names_game_and_ply(ev):
    games = [(START, "e2e4 e7e5"), (START, "e2e4 e7e5 e1g1")]
    with pytest.raises(F.FnnueError) as e:
        ev.build_batch(games)
    assert e.value.name == "FNNUE_E_MOVE" and "ply 3 of game 1" in str(e.value)
    with pytest.raises(F.FnnueError) as e:
        ev.build_batch(games, N.PLAYOUT_CHILDREN)
    assert e.value.name == "FNNUE_E_MOVE"


@pytest.mark.parametrize("bad", ["rnbqkbnr/pppppppp w", "8/8/8/8/8/8/8/8 w - - 0 1",
                                 "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNX w KQkq - 0 1"])
def test_bad_fen(ev, bad):
    with pytest.raises(F.FnnueError) as e:
        ev.build_batch([(START, ""), (bad, "")])
    assert e.value.name == "FNNUE_E_FEN"


def test_empty_batch(ev):
    pos, off = ev.build_batch([])
    assert len(pos) == 0


def test_builder_feeds_evaluator(ev):
    """Device-built CHAIN/STAR groups evaluate like the host-built ones."""
    games = [(g["position"], g["moves"]) for g in GAMES[:20]]
    pos, off = ev.build_batch(games, N.PLAYOUT_PLIES)
    hpos, hoff = host_plies(games)
    a = ev.eval_groups(pos, off, N.GROUP_CHAIN)
    b = ev.eval_groups(hpos, hoff, N.GROUP_CHAIN)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
