"""Device batch builder for variant games (fnnue_build_vbatch[_device],
csrc/vbuilder.hip) against the host replay (fnnue_game_vpositions /
_vchildren), record for record: crazyhouse (drops, pockets, promoted pieces)
and atomic (explosions) games from the start position and from FENs with
holdings.  The rules both run are pinned by perft known answers
(tests/test_vbuilder.py).  [ref] src/queue.rs:524-552, :530-539."""
import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from fishnet_amd import nnue
from tests.conftest import net_bytes

pytestmark = pytest.mark.gpu

ZH, AT = N.VARIANT_CRAZYHOUSE, N.VARIANT_ATOMIC
ROOTS = {
    ZH: ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1",
         "r1bqkb1r/pppp1ppp/2n2n2/4p3/2B1P3/5N2/PPPP1PPP/RNBQK2R[] w KQkq - 4 4",
         "2k5/8/8/8/8/8/8/4K3[QRBNPqrbnp] w - - 0 1",
         "rnb1kbnr/ppp2ppp/8/8/8/8/PPP2PPP/RNBQKBNR[Qpp] b KQkq - 0 5"],
    AT: ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
         "rn2kb1r/1pp1p2p/p2q1pp1/3P4/2P3b1/4PN2/PP3PPP/R2QKB1R b KQkq - 0 1",
         "r3k2r/pppppppp/8/8/8/8/PPPPPPPP/R3K2R w KQkq - 0 1"],
}


@pytest.fixture(scope="module")
def ev():
    e = F.Evaluator(F.Net.from_bytes(net_bytes(7, 128, 0)), 0)  # the builder needs a ctx (device, stream) only
    yield e
    e.close()


def _games(variant, count, seed):
    games = []
    for i in range(count):
        fen = ROOTS[variant][i % len(ROOTS[variant])]
        games.append((fen, nnue.random_vgame(seed + i, variant, fen, 40 + (i * 37) % 160)))
    return games


@pytest.mark.parametrize("variant", [ZH, AT])
def test_device_vbuilder_plies_match_host_replay(ev, variant):
    games = _games(variant, 300, 11 if variant == ZH else 23)
    pos, off = ev.build_vbatch(variant, games, N.PLAYOUT_PLIES)
    host = [nnue.game_vpositions(variant, fen, mv) for fen, mv in games]
    assert list(off) == list(np.concatenate([[0], np.cumsum([len(h) for h in host])]))
    assert np.array_equal(pos, np.concatenate(host))
    assert sum(mv.count("@") for _, mv in games) > 100 or variant == AT


@pytest.mark.parametrize("variant", [ZH, AT])
def test_device_vbuilder_children_match_host(ev, variant):
    games = _games(variant, 24, 101 if variant == ZH else 202)
    pos, off = ev.build_vbatch(variant, games, N.PLAYOUT_CHILDREN)
    hp, ho = [], [np.zeros(1, np.int64)]
    base = 0
    for fen, mv in games:
        p, o = nnue.game_vchildren(variant, fen, mv)
        hp.append(p)
        ho.append(o[1:].astype(np.int64) + base)
        base += len(p)
    assert np.array_equal(pos, np.concatenate(hp))
    assert np.array_equal(off.astype(np.int64), np.concatenate(ho))


def test_device_vbuilder_errors_name_the_game(ev):
    fen = ROOTS[ZH][0]
    games = [(fen, "e2e4 e7e5"), (fen, "e2e4 P@e5"), (fen, "g1f3")]  # black has no pawn in hand
    with pytest.raises(F.FnnueError) as e:
        ev.build_vbatch(ZH, games)
    assert e.value.name == "FNNUE_E_MOVE" and "game 1" in str(e.value) and "ply 2" in str(e.value)
    with pytest.raises(F.FnnueError) as e:
        ev.build_vbatch(AT, [(ROOTS[AT][0], "e2e4"), ("8/8/8/8/8/8/8/8 w - - 0 1", "")])
    assert e.value.name == "FNNUE_E_FEN" and "game 1" in str(e.value)
    pos, off = ev.build_vbatch(ZH, [(fen, "")])  # no moves: the root only
    assert len(pos) == 1 and list(off) == [0, 1]
