"""Fairy-Stockfish variant NNUE (BASELINE config 5) on CPU: loader, feature
indices, the CPU restatement's invariances and incremental == refresh.

PARITY UNPINNED: the reference runs variants with Fairy-Stockfish's classical
eval (src/assets.rs:384-391, src/stockfish.rs:248-260), the Fairy-Stockfish
submodule is empty and no variant net is pinned; the feature set is recalled
from Fairy-Stockfish's half_ka_v2_variants (oracle/variant_oracle.c header)."""
import hashlib
import json
import os

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from oracle.oracle import VariantOracleNet, lib as olib, variant_features
from tests.conftest import net_bytes

CZH, ATOMIC = F.VARIANT_CRAZYHOUSE, F.VARIANT_ATOMIC
START_ZH = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1"


def test_variant_loader_checks_feature_set():
    for v, rows in ((CZH, 864), (ATOMIC, 704)):
        data = F.synthesize_variant_net(3, 256, v)
        net = F.Net.from_bytes_variant(data, v)
        assert net.variant == v and net.info()[0] == 256
        assert len(data) > 64 * rows * 256 * 2  # the FT table: 64 king squares x rows x hd int16
        with pytest.raises(F.FnnueError):  # a variant net is not a chess net (feature-set hash)
            F.Net.from_bytes(data)
    with pytest.raises(F.FnnueError):  # crazyhouse net read as atomic: table size / EOF mismatch
        F.Net.from_bytes_variant(F.synthesize_variant_net(3, 256, CZH), ATOMIC)
    with pytest.raises(F.FnnueError):  # chess net read as a variant net
        F.Net.from_bytes_variant(net_bytes(7, 128, 0), CZH)
    leb = F.synthesize_variant_net(4, 256, CZH, N.SYNTH_LEB128)
    assert F.Net.from_bytes_variant(leb, CZH).variant == CZH


def test_variant_feature_indices_known_values():
    # board: orient = rank flip for black, no mirroring; own pawn plane 0, their pawn plane 1, kings 10
    assert olib.voracle_board_index(CZH, 0, 12, 1, 4) == 12 + 864 * 4          # white: own pawn e2, king e1
    assert olib.voracle_board_index(CZH, 1, 12, 1, 60) == (12 ^ 56) + 64 + 864 * (60 ^ 56)
    assert olib.voracle_board_index(ATOMIC, 0, 60, 14, 4) == 60 + 640 + 704 * 4  # their king shares plane 10
    # hand: 704 + 16 * (2 * (pt - 1) + (owner != perspective)) + k
    assert olib.voracle_hand_index(CZH, 0, 0, 1, 0, 4) == 704 + 864 * 4
    assert olib.voracle_hand_index(CZH, 1, 0, 1, 2, 60) == 704 + 16 + 2 + 864 * 4
    assert olib.voracle_hand_index(CZH, 0, 1, 5, 15, 4) == 704 + 16 * 9 + 15 + 864 * 4


def test_vpos_from_fen_holdings():
    a = F.vpos_from_fen(CZH, "r1bqkb1r/ppp2ppp/2n2n2/4p3/4P3/5N2/PPP2PPP/RNBQKB1R[Pp] w KQkq - 0 1")
    b = F.vpos_from_fen(CZH, "r1bqkb1r/ppp2ppp/2n2n2/4p3/4P3/5N2/PPP2PPP/RNBQKB1R/Pp w KQkq - 0 1")
    assert np.array_equal(a, b)
    assert a[33] == 1 and a[38] == 1 and a[33:43].sum() == 2 and a[32] == 0
    c = F.vpos_from_fen(CZH, "r1bqkb1r/ppp2ppp/2n2n2/4p3/4P3/5N2/PPP2PPP/RNBQ~KB1R[QQ] b - - 0 1")
    assert c[37] == 2 and c[32] == 1
    with pytest.raises(F.FnnueError):
        F.vpos_from_fen(ATOMIC, "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[P] w - - 0 1")  # no pockets
    with pytest.raises(F.FnnueError):
        F.vpos_from_fen(CZH, "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[P] w - - 0 1")  # 33 pieces
    s = F.vpos_from_fen(CZH, START_ZH)
    assert s[33:43].sum() == 0


def flip(vpos: np.ndarray) -> np.ndarray:
    """Colour flip: ranks mirrored, piece colours swapped, hands swapped, stm flipped."""
    out = vpos.copy()
    b = np.zeros(64, np.uint8)
    b[0::2] = vpos[:32] & 15
    b[1::2] = vpos[:32] >> 4
    f = np.zeros(64, np.uint8)
    for s in range(64):
        pc = b[s]
        f[s ^ 56] = (pc ^ 8) if pc else 0
    out[:32] = (f[0::2] & 15) | (f[1::2] << 4)
    out[32] = 1 - vpos[32]
    out[33:38], out[38:43] = vpos[38:43].copy(), vpos[33:38].copy()
    return out


@pytest.mark.parametrize("variant", [CZH, ATOMIC])
def test_variant_oracle_colour_flip_invariance(variant):
    """HalfKAv2 variants orient by rank flip only, so the colour-flipped position
    has the same two accumulators in swapped roles: identical outputs."""
    on = VariantOracleNet(F.synthesize_variant_net(3, 256, variant), variant)
    pos = F.random_vpositions(8, variant, 400, 90)
    fl = np.stack([flip(p) for p in pos])
    a, b = on.eval_packed(pos, threads=8), on.eval_packed(fl, threads=8)
    assert a[2] == 0 and b[2] == 0
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    # features: white's list in P == black's list in flip(P)
    for p in pos[:50]:
        assert variant_features(variant, p, 0) == variant_features(variant, flip(p), 1)


@pytest.mark.parametrize("variant", [CZH, ATOMIC])
def test_variant_oracle_incremental_equals_refresh(variant):
    """Accumulators updated along CHAIN (previous position) and STAR (first
    position) groups by feature-set differences (board and pockets), refreshed
    on own-king moves == every position from scratch, bit for bit."""
    on = VariantOracleNet(F.synthesize_variant_net(5, 256, variant), variant)
    pos, off = F.random_vpositions(9, variant, 150, 120, mode=F.PLAYOUT_PLIES)
    ref = on.eval_packed(pos, threads=8)
    assert ref[2] == 0
    for mode in (F.GROUP_CHAIN, F.GROUP_STAR):
        inc = on.eval_groups(pos, off, mode)
        assert inc[2] == 0
        assert np.array_equal(inc[0], ref[0]) and np.array_equal(inc[1], ref[1])


def test_random_vpositions_are_valid():
    pos = F.random_vpositions(3, CZH, 3000, 160)
    hands = pos[:, 33:43].astype(int)
    b = np.zeros((len(pos), 64), np.uint8)
    b[:, 0::2] = pos[:, :32] & 15
    b[:, 1::2] = pos[:, :32] >> 4
    assert hands.max() <= 16 and hands.sum(1).max() > 0
    assert ((b != 0).sum(1) + hands.sum(1)).max() <= 32
    assert np.all((b == 6).sum(1) == 1) and np.all((b == 14).sum(1) == 1)
    at = F.random_vpositions(3, ATOMIC, 3000, 160)
    assert at[:, 33:43].sum() == 0


def numpy_accumulator_bound(data: bytes, hd: int, rows: int, blocks: int, king_row) -> int:
    """The SWAR bound restated over the raw file: per king block and column,
    |bias + own-king row| + the 31 largest |w| of the other rows, over the
    first half's even columns and, doubled, every second-half column."""
    desc_len = int(np.frombuffer(data, np.uint32, 1, 8)[0])
    o = 12 + desc_len + 4  # header, then the FT hash
    cols = np.concatenate([np.arange(0, hd // 2, 2), np.arange(hd // 2, hd)])
    scale = np.where(cols < hd // 2, 1, 2)
    bias = np.frombuffer(data, np.int16, hd, o).astype(np.int64)[cols]
    w = np.frombuffer(data, np.int16, blocks * rows * hd, o + 2 * hd).reshape(blocks, rows, hd)[:, :, cols]
    w = np.abs(w.astype(np.int64))
    worst = 0
    for kb in range(blocks):
        kr = king_row(kb)
        m = w[kb].copy()
        krow = np.frombuffer(data, np.int16, hd, o + 2 * hd + 2 * (kb * rows + kr) * hd).astype(np.int64)[cols]
        base = np.abs(bias + krow)
        m[kr] = 0
        top = -np.sort(-m, axis=0)[:31].sum(axis=0)
        worst = max(worst, int(((base + top) * scale).max()))
    return worst


@pytest.mark.parametrize("variant,rows", [(CZH, 864), (ATOMIC, 704)])
def test_variant_accumulator_bound_covers_the_whole_table(variant, rows):
    """fnnue_net_accumulator_bound of a variant net runs over its 64 king
    blocks of `rows` rows (own king row 640 + king square)."""
    data = F.synthesize_variant_net(4, 256, variant)
    got = F.Net.from_bytes_variant(data, variant).accumulator_bound()
    assert got == numpy_accumulator_bound(data, 256, rows, 64, lambda kb: 640 + kb)
    chess = net_bytes(7, 128, 0)
    assert F.Net.from_bytes(chess).accumulator_bound() == numpy_accumulator_bound(
        chess, 128, 704, 32, lambda kb: 640 + 8 * (7 - (kb >> 2)) + (7 - (kb & 3)))


GOLDEN_V = os.path.join(os.path.dirname(__file__), "golden", "golden_variant_evals.json")


def test_variant_golden_vectors():
    """The restatement against its committed fixture (tests/golden/
    make_variant_fixtures.py): FENs with holdings, atomic positions and a
    digest over 4000 random walks per net."""
    g = json.load(open(GOLDEN_V))
    assert len(g["nets"]) == 4
    for e in g["nets"]:
        v = e["variant"]
        on = VariantOracleNet(F.synthesize_variant_net(e["seed"], e["hd"], v), v)
        pos = np.stack([F.vpos_from_fen(v, f) for f in e["fens"]])
        ps, po, rc = on.eval_packed(pos, threads=4)
        assert rc == 0 and ps.tolist() == e["psqt"] and po.tolist() == e["positional"]
        walks = F.random_vpositions(e["walks_seed"], v, e["walks_count"], e["walks_max_plies"])
        wps, wpo, rc = on.eval_packed(walks, threads=8)
        assert rc == 0
        digest = hashlib.sha256(wps.astype("<i4").tobytes() + wpo.astype("<i4").tobytes()).hexdigest()
        assert digest == e["walks_sha256"]


def test_variant_oracle_atomic_game_over_record():
    """An atomic position with one king exploded is a game-over record: the
    oracle answers (0, 0) without an error (the evaluator does the same on the
    GPU); no king at all, or a missing crazyhouse king, stays invalid."""
    import fishnet_amd as F
    from oracle.oracle import VariantOracleNet
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    pos = F.game_vpositions(ATOMIC, start, "g1f3 e7e6 f3g5 f8e7 g5f7")
    on = VariantOracleNet(F.synthesize_variant_net(3, 256, ATOMIC), ATOMIC)
    ps, po, rc = on.eval_packed(pos)
    assert rc == 0 and ps[-1] == 0 and po[-1] == 0 and np.any(po[:-1])
    gps, gpo, grc = on.eval_groups(pos, np.array([0, len(pos)], np.uint32), 0)
    assert grc == 0 and np.array_equal(gps, ps) and np.array_equal(gpo, po)
    bad = pos[-1:].copy()
    bad[0, :32] &= np.where((bad[0, :32] & 15) == 6, 0xF0, 0xFF).astype(np.uint8)
    bad[0, :32] &= np.where((bad[0, :32] >> 4) == 6, 0x0F, 0xFF).astype(np.uint8)
    assert on.eval_packed(bad)[2] != 0
    onz = VariantOracleNet(F.synthesize_variant_net(3, 256, CZH), CZH)
    zpos = pos[-1:].copy()
    assert onz.eval_packed(zpos)[2] != 0
