"""CPU tests of the oracle itself (oracle/nnue_oracle.c): structure hashes,
agreement with the independent numpy restatement (tests/refpy.py), clamp
regimes, exact symmetries, golden vectors.  No GPU."""
import hashlib
import json
import os

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from oracle import oracle as O
from tests import refpy
from tests.conftest import net_bytes
from tests.positions import FENS

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_structure_hashes_match_survey():
    # HD=1024 -> FT 0x7F2344B8, Net 0x63336A4A, file 0x1C102EF2
    assert O.lib.oracle_ft_hash(1024) == 0x7F2344B8
    assert O.lib.oracle_net_hash(1024) == 0x63336A4A
    assert O.lib.oracle_ft_hash(1024) ^ O.lib.oracle_net_hash(1024) == 0x1C102EF2
    assert refpy.net_hash(1024) == 0x63336A4A and refpy.ft_hash(1024) == 0x7F2344B8


def test_make_index_known_values():
    # White king e1 (sq 4), own pawn e2 (sq 12), white perspective: no flip
    # (king on file e), king bucket of e1 = 31.
    assert O.lib.oracle_make_index(0, 12, 1, 4) == 12 + 0 * 64 + 704 * 31
    # Black perspective, black king e8 (60): orient flips ranks -> e1 -> bucket 31;
    # black pawn e7 (52) is "own" -> plane 0, square 52^56 = 12.
    assert O.lib.oracle_make_index(1, 52, 9, 60) == 12 + 704 * 31
    # King on d1 (file < E): files mirrored: d1 -> e1, a2 (8) -> h2 (15); white knight = plane 2.
    assert O.lib.oracle_make_index(0, 8, 2, 3) == 15 + 2 * 64 + 704 * 31
    # Kings share plane 10; enemy queen = plane 9; H8 king -> bucket 0.
    assert O.lib.oracle_make_index(0, 63, 14, 4) == 63 + 10 * 64 + 704 * 31
    assert O.lib.oracle_make_index(0, 0, 13, 63) == 0 + 9 * 64 + 0
    assert max(refpy.feature(p, s, pc, k) for p in (0, 1) for s in range(64) for pc in (1, 6, 9, 14)
               for k in range(64)) == 22527


def _sample_positions(n=40, seed=5):
    fen_pos = np.stack([F.pos_from_fen(x) for x in FENS])
    return np.concatenate([fen_pos, F.random_playouts(seed, n, threads=2)])


@pytest.mark.parametrize("seed,hd,flags", [(1, 1024, 0), (7, 128, 0), (3, 1024, N.SYNTH_WRAP),
                                           (4, 256, N.SYNTH_FC1_PAD), (8, 1536, 0),
                                           (10, 3072, N.SYNTH_WRAP)])
def test_oracle_matches_numpy_restatement(seed, hd, flags):
    data = net_bytes(seed, hd, flags)
    on = O.OracleNet(data)
    ref = refpy.RefNet(data)
    pos = _sample_positions(24, seed)
    ps, po, rc = on.eval_packed(pos)
    assert rc == 0
    for i, p in enumerate(pos):
        board, stm = O.unpack(p)
        assert refpy.evaluate(ref, board, stm) == (ps[i], po[i]), i


def test_clamp_regimes_are_exercised(oracle_big):
    """The synthetic net must drive every saturation branch, or bit-exactness
    says little: accumulators below 0 / inside / above 127, L1 outputs that
    saturate CReLU (y>>6 > 127) and SqrCReLU (y^2>>19 > 127) and go negative."""
    pos = F.random_playouts(9, 200, threads=2)
    acc_lo = acc_mid = acc_hi = 0
    y_neg = y_sat = y_mid = sq_sat = 0
    for p in pos:
        board, stm = O.unpack(p)
        _, x, y, acc = oracle_big.trace(board, stm)
        acc_lo += int((acc < 0).sum())
        acc_hi += int((acc > 127).sum())
        acc_mid += int(((acc >= 0) & (acc <= 127)).sum())
        y15 = y[:15]
        y_neg += int((y15 < 0).sum())
        y_sat += int(((y15 >> 6) > 127).sum())
        y_mid += int(((y15 >> 6) >= 0).sum() - ((y15 >> 6) > 127).sum())
        sq_sat += int(((y15.astype(np.int64) ** 2 >> 19) > 127).sum())
    tot = 2 * 1024 * len(pos)
    for c in (acc_lo, acc_mid, acc_hi):
        assert c > 0.05 * tot
    for c in (y_neg, y_sat, y_mid, sq_sat):
        assert c > 0.02 * 15 * len(pos)


def _flip_colors(board: np.ndarray) -> np.ndarray:
    out = np.zeros(64, dtype=np.uint8)
    for s in range(64):
        pc = int(board[s])
        if pc:
            out[s ^ 56] = pc ^ 8
    return out


def test_color_flip_and_file_mirror_invariance(oracle_big):
    """HalfKAv2_hm is symmetric: swapping colours + mirroring ranks + flipping
    stm, or mirroring files, leaves both outputs bit-identical."""
    for p in _sample_positions(30, 3):
        board, stm = O.unpack(p)
        base = oracle_big.eval_board(board, stm)
        assert oracle_big.eval_board(_flip_colors(board), 1 - stm) == base
        mirrored = np.array([board[s ^ 7] for s in range(64)], dtype=np.uint8)
        assert oracle_big.eval_board(mirrored, stm) == base


def test_leb128_and_plain_give_identical_results():
    plain = O.OracleNet(net_bytes(2, 512, 0))
    leb = O.OracleNet(net_bytes(2, 512, N.SYNTH_LEB128))
    assert len(net_bytes(2, 512, N.SYNTH_LEB128)) < len(net_bytes(2, 512, 0))
    pos = _sample_positions(50, 8)
    a = plain.eval_packed(pos)
    b = leb.eval_packed(pos)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("mutate", ["version", "hash", "truncate", "trailing", "stack_hash"])
def test_oracle_rejects_corrupt_nets(mutate):
    data = bytearray(net_bytes(5, 128, 0))
    if mutate == "version":
        data[0] ^= 1
    elif mutate == "hash":
        data[4] ^= 1
    elif mutate == "truncate":
        data = data[:-7]
    elif mutate == "trailing":
        data += b"\0"
    elif mutate == "stack_hash":
        dlen = int.from_bytes(data[8:12], "little")
        off = 12 + dlen + 4 + 2 * 128 + 2 * 128 * 22528 + 4 * 8 * 22528
        data[off] ^= 0x10
    with pytest.raises(ValueError):
        O.OracleNet(bytes(data))


def test_golden_vectors():
    g = json.load(open(os.path.join(GOLDEN, "golden_evals.json")))
    pos = np.stack([np.frombuffer(bytes.fromhex(h), dtype=np.uint8) for h in g["positions_hex"]])
    for entry in g["nets"]:
        on = O.OracleNet(net_bytes(entry["seed"], entry["hd"], entry["flags"]))
        assert on.file_hash == entry["file_hash"]
        ps, po, rc = on.eval_packed(pos)
        assert rc == 0
        assert ps.tolist() == entry["psqt"] and po.tolist() == entry["positional"]
        big = F.random_playouts(entry["playouts_seed"], entry["playouts_count"], threads=4)
        bps, bpo, rc = on.eval_packed(big, threads=4)
        digest = hashlib.sha256(bps.astype("<i4").tobytes() + bpo.astype("<i4").tobytes()).hexdigest()
        assert digest == entry["playouts_sha256"]


def test_oracle_game_replay_matches_batch_builder():
    """The oracle's own UCI replay and the product's legal-move batch builder
    must produce the same boards (two independent move appliers)."""
    games = json.load(open(os.path.join(GOLDEN, "wcc_games.json")))["games"]
    on = O.OracleNet(net_bytes(7, 128, 0))
    for g in games[:20]:
        ps_o, po_o = on.eval_game(g["position"], g["moves"])
        pos = F.game_positions(g["position"], g["moves"])
        ps, po, rc = on.eval_packed(pos)
        assert rc == 0
        assert np.array_equal(ps, ps_o) and np.array_equal(po, po_o)


@pytest.fixture(params=["avx2", "avx512"])
def simd_isa(request):
    want = request.param == "avx512"
    got = O.lib.cpu_simd_set_isa(int(want))
    if want and not got:
        pytest.skip("host has no AVX-512 VNNI")
    yield request.param
    O.lib.cpu_simd_set_isa(1)


@pytest.mark.parametrize("hd,flags", [(1024, 0), (128, 0), (512, N.SYNTH_WRAP), (256, N.SYNTH_FC1_PAD),
                                      (1536, 0)])
def test_cpu_baseline_simd_matches_scalar_oracle(hd, flags, simd_isa):
    """oracle/nnue_cpu_simd.c (the cpu_baseline: AVX2 / AVX-512 VNNI,
    register-tiled refresh, incremental CHAIN/STAR updates) is bit-identical
    to the scalar oracle."""
    on = O.OracleNet(net_bytes(11, hd, flags))
    pos = F.random_playouts(21, 3000, threads=4)
    pos = np.concatenate([pos, np.stack([F.pos_from_fen(f) for f in FENS])])
    a, b = on.eval_packed(pos, threads=4), on.simd_eval_packed(pos, threads=4)
    assert a[2] == b[2] == 0
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    for mode, gmode in ((F.PLAYOUT_PLIES, N.GROUP_CHAIN), (F.PLAYOUT_CHILDREN, N.GROUP_STAR)):
        g, off = F.random_playouts(22, 40, mode=mode, threads=4)
        a, b = on.eval_packed(g, threads=4), on.simd_eval_groups(g, off, gmode, threads=4)
        assert a[2] == b[2] == 0
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_cpu_baseline_simd_invalid_positions():
    on = O.OracleNet(net_bytes(11, 128, 0))
    pos = F.random_playouts(23, 20, mode=F.PLAYOUT_PLIES, threads=2)[0][:20].copy()
    pos[5, :32] = 0  # no kings
    ps, po, rc = on.simd_eval_groups(pos, np.array([0, 10, 20], dtype=np.uint32), N.GROUP_CHAIN)
    a = on.eval_packed(pos)
    assert rc != 0 and a[2] != 0
    assert np.array_equal(ps, a[0]) and np.array_equal(po, a[1])


def test_later_sf_transform_equals_sfnnv5_transform():
    """later Stockfish stores the FT weights and biases doubled
    in memory and transforms with clamp(2a, 0, 254) * clamp(2b, 0, 254) >> 9;
    SFNNv5 (this evaluator, the oracle) uses clamp(a, 0, 127) * clamp(b, 0, 127)
    >> 7.  Exhaustive over every int16 accumulator pair whose doubled value
    does not wrap (|a|, |b| < 2^14): the two transforms agree everywhere, so a
    later net evaluates identically here whenever upstream's own doubled int16
    accumulators do not wrap."""
    a = np.arange(-(1 << 14), 1 << 14, dtype=np.int64)
    # the clamp identity per operand, over the whole non-wrapping range
    assert np.array_equal(np.clip(2 * a, 0, 254), 2 * np.clip(a, 0, 127))
    # and the product/shift identity over every pair of clamped values
    x = np.arange(128, dtype=np.int64)
    later = (np.clip(2 * x, 0, 254)[:, None] * np.clip(2 * x, 0, 254)[None, :]) >> 9
    v5 = (x[:, None] * x[None, :]) >> 7
    assert np.array_equal(later, v5)
    assert v5.max() == 126  # the u8 L1 input range both versions feed to fc_0
