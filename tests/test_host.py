"""CPU tests of libfnnue.so's host side: ABI exports, .nnue parsing, board
code (perft known answers, FEN, Chess960), batch building, playouts.  The
device entry points are only checked for their no-GPU error path here."""
import json
import os
import re

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from oracle import oracle as O
from tests.conftest import ROOT, net_bytes
from tests.positions import CHESS960, FENS, PERFT, START


def header_symbols():
    inc = os.path.join(ROOT, "include")
    text = "".join(open(os.path.join(inc, h)).read() for h in sorted(os.listdir(inc)) if h.endswith(".h"))
    return sorted(set(re.findall(r"\b(fnnue_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(N.lib, s), s
        assert s in N.SIGNATURES, f"{s} not bound in _native.py"


def test_abi_version():
    assert N.lib.fnnue_abi_version() >> 16 == 3  # 3.0: the fnnue_multi_*_device calls take streams


def test_net_parse_and_info():
    net = F.Net.from_bytes(net_bytes(1, 1024, 0))
    hd, fh, desc = net.info()
    assert hd == 1024 and fh == 0x1C102EF2 and "synthetic" in desc


def test_leb128_image_identical():
    a = F.Net.from_bytes(net_bytes(2, 512, 0)).image()
    b = F.Net.from_bytes(net_bytes(2, 512, N.SYNTH_LEB128)).image()
    assert np.array_equal(a, b)


@pytest.mark.parametrize("mutate,code", [("version", "FNNUE_E_FORMAT"), ("hash", "FNNUE_E_FORMAT"),
                                         ("truncate", "FNNUE_E_FORMAT"), ("trailing", "FNNUE_E_FORMAT"),
                                         ("stack_hash", "FNNUE_E_FORMAT"), ("empty", "FNNUE_E_FORMAT")])
def test_net_rejects_corruption(mutate, code):
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
        data[12 + dlen + 4 + 2 * 128 + 2 * 128 * 22528 + 4 * 8 * 22528] ^= 0x10
    elif mutate == "empty":
        data = bytearray(b"\0" * 4)
    with pytest.raises(F.FnnueError) as e:
        F.Net.from_bytes(bytes(data))
    assert e.value.name == code


def test_net_load_missing_file():
    with pytest.raises(F.FnnueError) as e:
        F.Net.load("/nonexistent/nn-ad9b42354671.nnue")
    assert e.value.name == "FNNUE_E_IO"


def test_net_file_roundtrip(tmp_path):
    p = tmp_path / "synthetic.nnue"
    p.write_bytes(net_bytes(7, 128, 0))
    assert F.Net.load(str(p)).info()[0] == 128


@pytest.mark.parametrize("hd,flags", [(128, 0), (256, N.SYNTH_LEB128), (512, N.SYNTH_WRAP), (1024, 0)])
def test_net_sha256_matches_hashlib(hd, flags):
    """fnnue_net_sha256 (FIPS 180-4 restated in csrc/sha256.cpp) == hashlib on
    files of several lengths (plain and LEB128 tensors: different tail blocks)."""
    import hashlib
    data = net_bytes(3, hd, flags)
    assert F.Net.from_bytes(data).sha256() == hashlib.sha256(data).hexdigest()


def test_net_identity_from_file_name(tmp_path):
    """[ref] build.rs:7 pins nn-ad9b42354671.nnue; upstream names a net by the
    first 12 hex digits of its SHA-256 and build.rs:100-112 deletes a corrupt
    download.  A file whose nn-<12 hex>.nnue name matches its digest loads; a
    mismatching one fails with FNNUE_E_FORMAT; other names make no claim."""
    import hashlib
    data = net_bytes(7, 128, 0)
    digest = hashlib.sha256(data).hexdigest()
    good = tmp_path / f"nn-{digest[:12]}.nnue"
    good.write_bytes(data)
    net = F.Net.load(str(good))
    assert net.sha256() == digest and net.info()[0] == 128
    wrong = "ad9b42354671" if digest[:12] != "ad9b42354671" else "000000000000"
    bad = tmp_path / f"nn-{wrong}.nnue"
    bad.write_bytes(data)
    with pytest.raises(F.FnnueError) as e:
        F.Net.load(str(bad))
    assert e.value.name == "FNNUE_E_FORMAT" and wrong in str(e.value)
    flipped = bytearray(data)
    flipped[len(data) // 2] ^= 1  # one bit of the weights: same structure, different digest
    corrupt = tmp_path / "sub"
    corrupt.mkdir()
    (corrupt / good.name).write_bytes(bytes(flipped))
    with pytest.raises(F.FnnueError) as e:
        F.Net.load(str(corrupt / good.name))
    assert e.value.name == "FNNUE_E_FORMAT"
    for other in ("nn-AD9B42354671.nnue", "nn-ad9b4235467.nnue", "custom.nnue", "nn-ad9b42354671.bin"):
        (tmp_path / other).write_bytes(data)
        assert F.Net.load(str(tmp_path / other)).sha256() == digest  # no identity claim in the name
    vdata = F.synthesize_variant_net(2, 256, F.VARIANT_ATOMIC)
    vd = hashlib.sha256(vdata).hexdigest()
    (tmp_path / f"nn-{vd[:12]}.nnue").write_bytes(vdata)
    assert F.Net.load_variant(str(tmp_path / f"nn-{vd[:12]}.nnue"), F.VARIANT_ATOMIC).sha256() == vd
    (tmp_path / "nn-0123456789ab.nnue").write_bytes(vdata)
    with pytest.raises(F.FnnueError) as e:
        F.Net.load_variant(str(tmp_path / "nn-0123456789ab.nnue"), F.VARIANT_ATOMIC)
    assert e.value.name == "FNNUE_E_FORMAT"


@pytest.mark.parametrize("fen,counts", PERFT)
def test_perft_known_answers(fen, counts):
    for depth, expect in enumerate(counts, start=1):
        assert F.perft(fen, depth) == expect, (fen, depth)


def test_chess960_perft():
    # Published Chess960 perft (position 1 of the standard 960 perft suite).
    fen = "bqnb1rkr/pp3ppp/3ppn2/2p5/5P2/P2P4/NPP1P1PP/BQ1BNRKR w HFhf - 2 9"
    assert [F.perft(fen, d) for d in (1, 2, 3)] == [21, 528, 12189]


def test_fen_packing_matches_oracle_parser():
    for fen in FENS:
        p = F.pos_from_fen(fen)
        board, stm = O.board_from_fen(fen)
        assert np.array_equal(O.pack(board, stm), p), fen


@pytest.mark.parametrize("bad", ["", "rnbqkbnr/pppppppp w", "8/8/8/8/8/8/8/8 w - - 0 1",
                                 "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNX w KQkq - 0 1"])
def test_bad_fen(bad):
    with pytest.raises(F.FnnueError) as e:
        F.pos_from_fen(bad)
    assert e.value.name == "FNNUE_E_FEN"


def test_game_expansion_matches_oracle_replay():
    games = json.load(open(os.path.join(ROOT, "tests", "golden", "wcc_games.json")))["games"]
    assert len(games) >= 50
    for g in games:
        pos = F.game_positions(g["position"], g["moves"])
        assert len(pos) == len(g["moves"].split()) + 1
        board, stm = O.board_from_fen(g["position"])
        import ctypes as C
        st, ep = C.c_int(stm), C.c_int(-1)
        for i, mv in enumerate(g["moves"].split()):
            assert O.lib.oracle_apply_uci(board.ctypes.data, C.byref(st), C.byref(ep), mv.encode()) == 0
            assert np.array_equal(O.pack(board, st.value), pos[i + 1]), (g["id"], i, mv)


def test_chess960_castling_notation():
    # king-takes-rook castling as fishnet sends it (UCI_Chess960, src/stockfish.rs:213)
    fen = "r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1"
    a = F.game_positions(fen, "e1h1 e8a8")
    b = F.game_positions(fen, "e1g1 e8c8")
    assert np.array_equal(a, b)
    board, _ = O.unpack(a[2])
    assert board[6] == 6 and board[5] == 4 and board[58] == 14 and board[59] == 12
    # Chess960 (Shredder-FEN): "e1g1" is king-takes-rook on g1 -> Kg1, Rf1.
    pos = F.game_positions("1r2k1r1/pppppppp/8/8/8/8/PPPPPPPP/1R2K1R1 w GBgb - 0 1", "e1g1 e8b8")
    board, _ = O.unpack(pos[1])
    assert board[6] == 6 and board[5] == 4 and board[4] == 0
    board, _ = O.unpack(pos[2])
    assert board[58] == 14 and board[59] == 12 and board[57] == 0 and board[60] == 0
    # blocked castling (bishop on d1) is illegal in CHESS960
    with pytest.raises(F.FnnueError):
        F.game_positions(CHESS960, "g1f1")


def test_illegal_move_is_rejected():
    with pytest.raises(F.FnnueError) as e:
        F.game_positions(START, "e2e4 e7e5 e1g1")
    assert e.value.name == "FNNUE_E_MOVE"


def test_en_passant_and_promotion():
    pos = F.game_positions("rnbqkbnr/ppp1p1pp/8/3pPp2/8/8/PPPP1PPP/RNBQKBNR w KQkq f6 0 3", "e5f6")
    board, _ = O.unpack(pos[1])
    assert board[45] == 1 and board[37] == 0
    pos = F.game_positions("8/P6k/8/8/8/8/6Kp/8 w - - 0 1", "a7a8n h2h1q")
    board, _ = O.unpack(pos[2])
    assert board[56] == 2 and board[7] == 13


def test_game_children_groups():
    pos, off = F.game_children(START, "e2e4 e7e5")
    assert list(np.diff(off)) == [21, 21, 30]
    assert np.array_equal(pos[0], F.pos_from_fen(START))


def test_playouts_deterministic_across_threads():
    a = F.random_playouts(3, 300, threads=1)
    b = F.random_playouts(3, 300, threads=7)
    assert np.array_equal(a, b)
    pa, oa = F.random_playouts(4, 20, mode=N.PLAYOUT_PLIES, threads=1)
    pb, ob = F.random_playouts(4, 20, mode=N.PLAYOUT_PLIES, threads=3)
    assert np.array_equal(pa, pb) and np.array_equal(oa, ob)
    assert oa[-1] == len(pa)


def test_playout_positions_are_valid():
    pos = F.random_playouts(1, 2000, threads=4)
    on = O.OracleNet(net_bytes(7, 128, 0))
    _, _, rc = on.eval_packed(pos)
    assert rc == 0
    counts = [int(np.count_nonzero(O.unpack(p)[0])) for p in pos]
    assert min(counts) >= 2 and max(counts) == 32 and 15 < np.mean(counts) < 30


def test_device_entry_points_fail_cleanly_without_gpu():
    if F.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(F.FnnueError) as e:
        F.Evaluator(F.Net.from_bytes(net_bytes(7, 128, 0)), 0)
    assert e.value.name == "FNNUE_E_DEVICE"
    with pytest.raises(F.FnnueError):
        F.selftest_mfma(0)


def test_accumulator_bound_decides_swar():
    """SWAR row sums (ft_slices) are exact only if no reachable accumulator's
    low column leaves int16 range and no doubled second-half column leaves it
    (net.h): realistic synthetic nets qualify, the
    int16-wrap stress net does not (the library then keeps packed adds)."""
    import fishnet_amd as F
    b = F.Net.from_bytes(F.synthesize_net(1, 1024, 0)).accumulator_bound()
    assert 0 < b < 32768
    w = F.Net.from_bytes(F.synthesize_net(3, 1024, N.SYNTH_WRAP)).accumulator_bound()
    assert w >= 32768


def test_playouts_accept_the_full_ply_range():
    """max_plies = 2^32 - 1: the ply-count range is widened before the +1 (no
    division by zero); games still end by mate, stalemate or the 50-move rule."""
    pos = F.random_playouts(5, 2, 0, 2 ** 32 - 1, threads=1)
    assert len(pos) == 2
