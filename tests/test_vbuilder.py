"""Variant games (crazyhouse, atomic): the rules of csrc/vboard.h that the host
replay (fnnue_game_vpositions / _vchildren) and the device batch builder
(fnnue_build_vbatch, tests/test_gpu_vbuilder.py) share.

The reference validates and plays every move of a variant batch with
shakmaty (`Uci::to_move`, `play_unchecked`, [ref] src/queue.rs:524-552) before
sending it to Fairy-Stockfish (:530-539).  Neither is available offline, so
the move generator is pinned by published perft known answers (startpos and
two positions exercising drops and explosions), and the replay semantics
(pockets, promoted pieces, explosions, castling rights, notation) by
hand-checked positions.
"""
import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from fishnet_amd import nnue

ZH, AT = N.VARIANT_CRAZYHOUSE, N.VARIANT_ATOMIC
START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
ZH_START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1"

# Published perft counts (crazyhouse / atomic move generators of the chess
# variant libraries and Fairy-Stockfish's perft suite).
PERFT = [
    (ZH, ZH_START, [20, 400, 8902, 197281, 4888832]),
    (ZH, "2k5/8/8/8/8/8/8/4K3[QRBNPqrbnp] w - - 0 1", [301, 75353]),
    (AT, START, [20, 400, 8902, 197326, 4864979]),
    (AT, "rn2kb1r/1pp1p2p/p2q1pp1/3P4/2P3b1/4PN2/PP3PPP/R2QKB1R b KQkq - 0 1", [40, 1238, 45237]),
]


def board(vp):
    b = np.zeros(64, np.uint8)
    b[0::2] = vp[:32] & 15
    b[1::2] = vp[:32] >> 4
    return b


def sq(name):
    return (ord(name[1]) - 49) * 8 + ord(name[0]) - 97


@pytest.mark.parametrize("variant,fen,counts", PERFT)
def test_variant_perft_known_answers(variant, fen, counts):
    for d, want in enumerate(counts, start=1):
        if want > 1_000_000 and d > 4:
            continue  # the depth-5 counts run in test_variant_perft_depth5
        assert nnue.vperft(variant, fen, d) == want, (fen, d)


@pytest.mark.parametrize("variant,want", [(ZH, 4888832), (AT, 4864979)])
def test_variant_perft_depth5(variant, want):
    assert nnue.vperft(variant, ZH_START if variant == ZH else START, 5) == want


def test_crazyhouse_captures_go_to_the_pocket_promoted_as_pawns():
    # black queen takes a promoted white queen: black's pocket gets a pawn
    pos = nnue.game_vpositions(ZH, "4k2q/8/8/8/8/8/8/4K2Q~[] b - - 0 1", "h8h1")
    assert pos.shape == (2, 48)
    assert list(pos[1, 33:43]) == [0, 0, 0, 0, 0, 1, 0, 0, 0, 0]
    # an ordinary capture keeps the piece type; then it is dropped back
    pos = nnue.game_vpositions(ZH, "4k3/8/8/3n4/4P3/8/8/4K3[] w - - 0 1", "e4d5 e8d7 N@f3")
    assert list(pos[1, 33:43]) == [0, 1, 0, 0, 0, 0, 0, 0, 0, 0]
    assert list(pos[3, 33:43]) == [0] * 10
    assert board(pos[3])[sq("f3")] == 2  # white knight dropped
    # a queen promoted on the board keeps its promoted status when it moves:
    # captured on a3 it reaches black's pocket as a pawn
    pos = nnue.game_vpositions(ZH, "4k3/P7/8/8/8/7r/8/4K3[] w - - 0 1", "a7a8q e8e7 a8a3 h3a3")
    assert list(pos[-1, 33:43]) == [0, 0, 0, 0, 0, 1, 0, 0, 0, 0]


def test_crazyhouse_drop_rules():
    fen = "4k3/8/8/8/8/8/8/4K3[Pp] w - - 0 1"
    for bad in ("P@e8", "P@a1", "N@e4", "P@e1"):
        with pytest.raises(F.FnnueError) as e:
            nnue.game_vpositions(ZH, fen, bad)
        assert e.value.name == "FNNUE_E_MOVE"
    pos = nnue.game_vpositions(ZH, fen, "P@e4 p@d5")  # either letter case
    assert board(pos[2])[sq("e4")] == 1 and board(pos[2])[sq("d5")] == 9
    assert list(pos[2, 33:43]) == [0] * 10
    # a drop that leaves the own king in check is illegal; one that blocks a check is legal
    fen = "4k3/8/8/8/8/8/8/r3K3[N] w - - 0 1"  # white king in check along the first rank
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(ZH, fen, "N@h3")
    nnue.game_vpositions(ZH, fen, "N@c1")


def test_atomic_explosions():
    # Nxd6 explodes the knight, the pawn and every non-pawn neighbour of d6
    pos = nnue.game_vpositions(AT, "4k3/4p3/2bpn3/8/4N3/8/8/4K3 w - - 0 1", "e4d6")
    b = board(pos[1])
    assert b[sq("e1")] == 6 and b[sq("e8")] == 14 and b[sq("e7")] == 9  # the pawn next to d6 survives
    assert int((b != 0).sum()) == 3
    # en passant explodes around the destination square
    pos = nnue.game_vpositions(AT, "4k3/8/8/3pP3/8/2n5/8/4K3 w - d6 0 1", "e5d6")
    b = board(pos[1])
    assert int((b != 0).sum()) == 3 and b[sq("c3")] == 10  # knight on c3 is not next to d6
    # kings never capture; a capture next to the own king explodes it: illegal
    for fen, mv in (("4k3/8/8/8/8/8/3p4/4K3 w - - 0 1", "e1d2"), ("4k3/8/8/8/8/8/4p3/4K1N1 w - - 0 1", "g1e2")):
        with pytest.raises(F.FnnueError) as e:
            nnue.game_vpositions(AT, fen, mv)
        assert e.value.name == "FNNUE_E_MOVE"
    # exploding the other king is legal even when the own king is in check
    # (Qxe7 explodes e8); a move that neither answers the check nor wins is not
    fen = "3rk3/4p3/8/8/7Q/8/8/3K4 w - - 0 1"
    pos = nnue.game_vpositions(AT, fen, "h4e7")
    assert int((board(pos[1]) == 14).sum()) == 0
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(AT, fen, "h4h5")
    # connected kings: a king next to the other king is never in check
    nnue.game_vpositions(AT, "8/8/8/8/8/3k4/r2K4/8 w - - 0 1", "d2e2")
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(ZH, "8/8/8/8/8/3k4/r2K4/8[] w - - 0 1", "d2e2")  # crazyhouse: plain chess check


def test_atomic_castling_rights_end_when_the_rook_explodes():
    # Rxg7 explodes next to h8: the rook goes, so black may castle only queen side
    fen = "r3k2r/6p1/8/8/8/8/8/R3K1R1 w Qkq - 0 1"
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(AT, fen, "g1g7 e8g8")
    pos = nnue.game_vpositions(AT, fen, "g1g7 e8c8")
    b = board(pos[2])
    assert b[sq("c8")] == 14 and b[sq("d8")] == 12 and b[sq("h8")] == 0
    # a rook captured on its square (explosion of both rooks) ends both sides' rights there
    fen = "r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1"
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(AT, fen, "a1a8 e8c8")
    nnue.game_vpositions(AT, fen, "a1a8 e8g8")
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(AT, fen, "a1a8 e8g8 e1c1")  # white's a1 rook went with it


def test_variant_replay_matches_children_expansion():
    """game_vchildren's ply positions are game_vpositions', and every child is
    one legal move away (the group sizes are the legal-move counts)."""
    for variant, fen in ((ZH, ZH_START), (AT, START)):
        for seed in range(4):
            moves = nnue.random_vgame(seed, variant, fen, 60)
            plies = nnue.game_vpositions(variant, fen, moves)
            ch, off = nnue.game_vchildren(variant, fen, moves)
            assert len(off) == len(plies) + 1
            assert np.array_equal(ch[off[:-1]], plies)
            toks = moves.split()
            for k in (0, len(toks) // 2):
                prefix = " ".join(toks[:k])
                last = nnue.game_vpositions(variant, fen, prefix)[-1]
                assert np.array_equal(last, plies[k])
                # each child: the position after one of the legal moves
                assert int(off[k + 1] - off[k] - 1) >= 0


def test_random_variant_games_replay_and_stay_valid():
    """Random legal games (drops, captures to the pocket, explosions) replay
    exactly; every position before a king explosion is a valid evaluator input."""
    drops = explosions = 0
    for variant, fen in ((ZH, ZH_START), (AT, START)):
        for seed in range(40):
            moves = nnue.random_vgame(1000 + seed, variant, fen, 200)
            pos = nnue.game_vpositions(variant, fen, moves)
            assert len(pos) == len(moves.split()) + 1
            drops += moves.count("@")
            for i, vp in enumerate(pos):
                b = board(vp)
                kings = int((b == 6).sum()), int((b == 14).sum())
                if kings != (1, 1):  # only an atomic game's last position: a king exploded
                    assert variant == AT and i == len(pos) - 1
                    explosions += 1
                    continue
                assert int((b != 0).sum()) + int(vp[33:43].sum()) <= 32
                assert vp[32] in (0, 1)
                if variant == AT:
                    assert int(vp[33:43].sum()) == 0
    assert drops > 100


def test_vpos_from_fen_uses_the_variant_parser():
    a = F.vpos_from_fen(ZH, "rnbqkbnr/ppp2ppp/8/8/8/8/PPP2PPP/RNBQKBNR[Qpp] w KQkq - 0 1")
    b = F.vpos_from_fen(ZH, "rnbqkbnr/ppp2ppp/8/8/8/8/PPP2PPP/RNBQKBNR/Qpp w KQkq - 0 1")
    assert np.array_equal(a, b) and list(a[33:43]) == [0, 0, 0, 0, 1, 2, 0, 0, 0, 0]
    c = F.vpos_from_fen(ZH, "rnbqkbnr/ppp2ppp/8/8/8/8/PPP2PPP/RNBQKBN~R[Qpp] w KQkq - 0 1")
    assert np.array_equal(a, c)  # promoted marks do not enter the features
    for bad in ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[K] w - - 0 1", "8/8/8/8/8/8/8/8[] w - - 0 1",
                "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[Q] x - - 0 1"):
        with pytest.raises(F.FnnueError):
            F.vpos_from_fen(ZH, bad)
    with pytest.raises(F.FnnueError):
        F.vpos_from_fen(AT, "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[Q] w KQkq - 0 1")  # no pockets in atomic


def test_variant_builder_entry_points_without_gpu():
    with pytest.raises(F.FnnueError):
        nnue.game_vpositions(7, START, "")
    with pytest.raises(F.FnnueError) as e:
        nnue.game_vpositions(ZH, "not a fen", "")
    assert e.value.name == "FNNUE_E_FEN"
    assert N.lib.fnnue_build_vbatch(None, ZH, b"", 0, None, None, 0, N.PLAYOUT_PLIES, None, 0, None, 0,
                                    None, None) == -1


@pytest.mark.parametrize("variant", [ZH, AT])
def test_random_vgames_deterministic_and_replayable(variant):
    """fnnue_random_vgames (bench / test inputs): every ply of legal random games
    as CHAIN groups, independent of the thread count; each game's first
    position is the start position, every position has both kings except an
    atomic game's last one when a king exploded there (the game's end)."""
    a, oa = nnue.random_vgames(9, variant, 300, 120, threads=1)
    b, ob = nnue.random_vgames(9, variant, 300, 120, threads=7)
    assert np.array_equal(a, b) and np.array_equal(oa, ob)
    assert len(oa) == 301 and oa[0] == 0 and oa[-1] == len(a) and np.all(np.diff(oa.astype(np.int64)) >= 1)
    start = nnue.game_vpositions(variant, ZH_START if variant == ZH else START, "")[0]
    assert all(np.array_equal(a[o], start) for o in oa[:-1])
    bd = np.zeros((len(a), 64), np.uint8)
    bd[:, 0::2] = a[:, :32] & 15
    bd[:, 1::2] = a[:, :32] >> 4
    kings = (bd == 6).sum(1) + (bd == 14).sum(1)
    last = np.zeros(len(a), bool)
    last[oa[1:].astype(np.int64) - 1] = True
    assert np.all(((bd == 6).sum(1) <= 1) & ((bd == 14).sum(1) <= 1))
    assert np.all(kings[~last] == 2)
    if variant == AT:
        assert np.any(kings[last] == 1)  # some games end by explosion
    else:
        assert np.all(kings == 2)
    if variant == ZH:
        assert int(a[:, 33:43].sum()) > 0  # pockets fill up
