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


# Move sequences whose later moves depend on what earlier moves of the same
# replay window did (the lane-parallel chess chain, replay_wave.h /
# ChessRules::lane_chain): castling in both notations followed by the king's
# and the rook's next moves, queenside and Chess960 castling where the king
# stays on its square, en passant taken and expired, promoted pieces moving
# on, and moves from squares emptied earlier (illegal: the first failing ply).
LANE_SEQS = [
    (START, "e2e4 e7e5 g1f3 b8c6 f1c4 g8f6 e1g1 f8c5 f1e1 e8g8 g1h1 c6d4 e1e2 f8e8 h1g1"),
    (START, "e2e4 e7e5 g1f3 b8c6 f1c4 g8f6 e1h1 f8c5 f1e1 e8h8 g1h1 c6d4 e1e2 f8e8 h1g1"),
    (START, "d2d4 d7d5 b1c3 b8c6 c1f4 c8f5 d1d2 d8d7 e1c1 e8c8 d1e1 d8e8 c1b1 c8b8 e1d1"),
    (START, "d2d4 d7d5 b1c3 b8c6 c1f4 c8f5 d1d2 d8d7 e1a1 e8a8 d1e1 d8e8 c1b1 c8b8 e1d1"),
    (START, "e2e4 a7a6 e4e5 d7d5 e5d6 c7d6 d2d4 d6d5"),
    (START, "e2e4 a7a6 e4e5 d7d5 a2a3 a6a5 e5d6"),
    (START, "e2e4 e7e5 e2e3"),
    (START, "e2e4 e7e5 g1f3 b8c6 f1c4 g8f6 e1g1 f8c5 h1g1"),
    (START, "e2e4 e7e5 g1f3 b8c6 f1c4 g8f6 e1e2 f8c5 e2e1 d7d6 e1g1"),
    ("8/P6k/8/8/8/8/6Kp/8 w - - 0 1", "a7a8q h2h1q a8a1 h1a1 g2f2 a1a2 f2e3 a2a8"),
    ("8/P6k/8/8/8/8/6Kp/8 w - - 0 1", "a7a8n h2h1r a8b6 h1h2 g2g3 h2b2 b6d5 b2b3"),
    ("r5kr/pppppppp/8/8/8/8/PPPPPPPP/R5KR w HAha - 0 1", "f2f4 f7f5 g1h1 g8h8 f1f3 f8f6 g1h1 g8h8 a1b1 a8b8"),
    ("1rk1r3/pppppppp/8/8/8/8/PPPPPPPP/1RK1R3 w BEbe - 0 1", "f2f4 f7f5 c1e1 c8e8 f1f3 f8f6 g1h1 g8h8 b1c1 b8c8"),
    ("1rk1r3/pppppppp/8/8/8/8/PPPPPPPP/1RK1R3 w BEbe - 0 1", "d2d4 d7d5 c1b1 c8b8 d1d3 d8d6 c1d1 c8d8 d1c1"),
    ("r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1", "e1g1 e8c8 f1f8 d8f8 g1h1 c8b8 a1a8 b8a8"),
    ("r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1", "a1a8 e8e7 a8h8 h8h1 e1h1"),
    ("r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1", "h1h8 e8d7 e1g1"),
]


def _host_outcome(fen, moves):
    """(positions, None) for a legal game, (None, first failing ply) else."""
    mv = moves.split()
    try:
        return F.game_positions(fen, moves), None
    except F.FnnueError:
        k = 0
        while True:
            try:
                F.game_positions(fen, " ".join(mv[:k + 1]))
                k += 1
            except F.FnnueError:
                return None, k + 1


def test_window_dependent_moves_match_host(ev):
    """Every LANE_SEQS game, from its root and (standard start) after knight
    shuffles of 28 / 56 / 60 plies that move its events across the 64-move
    window boundary: legal games record for record equal to the host builder
    (as one batch: the two-wave replay, and repeated past 1024 games: the
    one-wave replay), illegal ones fail at the host's first failing ply."""
    shuffle = "g1f3 g8f6 f3g1 f6g8"
    games = []
    for fen, moves in LANE_SEQS:
        for r in ((0, 7, 14, 15) if fen == START else (0,)):
            games.append((fen, " ".join([shuffle] * r + [moves]).strip()))
    legal, illegal = [], []
    for fen, moves in games:
        pos, ply = _host_outcome(fen, moves)
        (legal if ply is None else illegal).append((fen, moves, pos, ply))
    assert len(legal) >= 20 and len(illegal) >= 20
    for reps in (1, 1100 // len(legal) + 1):
        batch = [(f, m) for f, m, _, _ in legal] * reps
        pos, off = ev.build_batch(batch)
        hpos, hoff = host_plies(batch)
        assert np.array_equal(off, hoff) and np.array_equal(pos, hpos), reps
    for fen, moves, _, ply in illegal:
        with pytest.raises(F.FnnueError) as e:
            ev.build_batch([(fen, moves)])
        assert e.value.name == "FNNUE_E_MOVE" and f"ply {ply} of game 0" in str(e.value), (moves, str(e.value))
