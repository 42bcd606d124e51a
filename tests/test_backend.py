"""fnnue_backend host logic (no GPU): batch expansion sizes
(IncomingBatch::from_acquired, [ref] src/queue.rs:518-627) and the submitted
`analysis` JSON (CompletedBatch::into_analysis, queue.rs:715-727; AnalysisPart
and Score serialisation, src/api.rs:355-388)."""
import json

import pytest

from fishnet_amd import _native as N
from fishnet_amd import backend as B

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


def test_batch_size_analysis_and_move():
    assert B.batch_size(B.AcquireResponseBody("a1", START, "")) == 1
    assert B.batch_size(B.AcquireResponseBody("a2", START, "e2e4 e7e5  g1f3\n")) == 4
    assert B.batch_size(B.AcquireResponseBody("a3", START, ["e2e4", "e7e5"])) == 3
    assert B.batch_size(B.AcquireResponseBody("m1", START, "e2e4 e7e5", work="move")) == 1


def test_batch_size_rejects_unknown_work():
    with pytest.raises(N.FnnueError) as e:
        B.batch_size(B.AcquireResponseBody("x", START, "", work="ponder"))
    assert e.value.code == -1


def test_analysis_json_shapes():
    rs = [
        B.PositionResponse(0, B.Score("cp", 23), depth=0, nodes=1, time_ms=4, nps=250),
        B.PositionResponse(1, None, skipped=True),
        B.PositionResponse(2, B.Score("cp", -117), depth=0, nodes=1, time_ms=4, nps=0),
        B.PositionResponse(3, B.Score("mate", -2), depth=1, nodes=20, time_ms=0, nps=7),
    ]
    s = B.into_analysis(rs)
    assert s == ('[{"score":{"cp":23},"depth":0,"nodes":1,"time":4,"nps":250},{"skipped":true},'
                 '{"score":{"cp":-117},"depth":0,"nodes":1,"time":4},'
                 '{"score":{"mate":-2},"depth":1,"nodes":20,"time":0,"nps":7}]')
    parts = json.loads(s)
    assert parts[1] == {"skipped": True} and "pv" not in parts[0] and "nps" not in parts[2]
    assert B.into_analysis([]) == "[]"


def test_analysis_json_matrix_form():
    """A MultiPV batch (Work::matrix_wanted, [ref] src/api.rs:179-187) is
    answered as AnalysisPart::Matrix: pv / score matrices indexed [multipv -
    1][depth] (Matrix::set, src/ipc.rs:77-86); static evaluation fills line 1
    at depth 0 with an empty pv."""
    rs = [B.PositionResponse(0, B.Score("cp", 41), depth=0, nodes=1, time_ms=3, nps=9, matrix=True),
          B.PositionResponse(1, None, skipped=True)]
    s = B.into_analysis(rs)
    assert s == '[{"pv":[[[]]],"score":[[{"cp":41}]],"depth":0,"nodes":1,"time":3,"nps":9},{"skipped":true}]'


def test_analysis_json_capacity():
    import ctypes as C
    arr = (B._Response * 1)()
    n = C.c_size_t()
    buf = C.create_string_buffer(4)
    rc = N.lib.fnnue_backend_analysis_json(arr, 1, buf, len(buf), C.byref(n))
    assert rc == -10 and n.value > 4


def test_game_end_known_positions():
    """fnnue_game_end (host replay): what the engine answers with mate 0 /
    cp 0 and bestmove (none) ([ref] src/stockfish.rs:359-376)."""
    import fishnet_amd as F
    assert F.game_end(START, "f2f3 e7e5 g2g4 d8h4") == F.END_NO_MOVES | F.END_CHECK  # fool's mate
    assert F.game_end("7k/5Q2/5K2/8/8/8/8/8 w - - 0 1", "f6g6") == F.END_NO_MOVES  # stalemate
    assert F.game_end(START, "e2e4 e7e5 d1h5 b8c6") == 0
    assert F.game_end(START, "e2e4 e7e5 d1h5 g7g6 h5e5") == F.END_CHECK  # check, not mate
    # atomic: Nxf7 explodes the black king on e8; the game is over there
    assert F.game_end(START, "g1f3 e7e6 f3g5 f8e7 g5f7", N.VARIANT_ATOMIC) == F.END_NO_MOVES | F.END_EXTINCT
    # crazyhouse: a back-rank mate by a drop (black has nothing in hand to block)
    zh = "7k/6pp/8/8/8/8/8/K7[R] w - - 0 1"
    assert F.game_end(zh, "R@e8", N.VARIANT_CRAZYHOUSE) == F.END_NO_MOVES | F.END_CHECK
    assert F.game_end("7k/6pp/8/8/8/8/8/K7[Rr] w - - 0 1", "R@e8", N.VARIANT_CRAZYHOUSE) == F.END_CHECK  # r@f8 blocks
    with pytest.raises(N.FnnueError) as e:
        F.game_end(START, "e2e5")
    assert e.value.name == "FNNUE_E_MOVE"


def test_channel_nets_slot_checks_without_a_device():
    """fnnue_backend_channel_nets refuses a net in the wrong slot (and no net
    at all) before it touches a device."""
    import ctypes as C
    import fishnet_amd as F
    chess = F.Net.from_bytes(F.synthesize_net(1, 128))
    zh = F.Net.from_bytes_variant(F.synthesize_variant_net(2, 256, N.VARIANT_CRAZYHOUSE), N.VARIANT_CRAZYHOUSE)
    h = C.c_void_p()
    for nets, code in (((None, None, None), -1), ((zh._h, None, None), -4), ((None, chess._h, None), -4),
                       ((None, None, zh._h), -4)):
        rc = N.lib.fnnue_backend_channel_nets(C.byref(B._Nets(*nets)), 0, None, C.byref(h))
        assert rc == code, (nets, rc)


def test_batch_size_counts_tokens_like_the_builder():
    """fnnue_backend_batch_size counts the moves with the 16-byte scan
    (blanks ' ', tab, newline, CR): against Python's split on random texts of
    every length 0..80 at every start alignment 0..15 of the buffer."""
    import ctypes as C
    import random
    rng = random.Random(5)
    blanks = " \t\n\r"
    for length in range(81):
        text = "".join(rng.choice("e2e4q" + blanks) if rng.random() < 0.7 else rng.choice(blanks)
                       for _ in range(length))
        raw = text.encode()
        for shift in range(16):
            buf = C.create_string_buffer(64 + len(raw) + 1)
            base = (-C.addressof(buf)) % 16  # first 16-byte aligned offset
            C.memmove(C.addressof(buf) + base + shift, raw + b"\0", len(raw) + 1)
            a = B._Acquired()
            a.work = 0  # FNNUE_WORK_ANALYSIS
            a.position = START.encode()
            a.moves = C.cast(C.addressof(buf) + base + shift, C.c_char_p)
            n = C.c_size_t()
            N.check(N.lib.fnnue_backend_batch_size(C.byref(a), C.byref(n)))
            assert n.value == len(text.split()) + 1, (repr(text), shift)


def test_compact_layouts_and_argument_checks():
    """The compact answer's records (fnnue_backend.h) have the C layout the
    library writes, and the go() forms reject null arguments without a
    device."""
    import ctypes as C
    assert C.sizeof(B._Compact) == 16 and C.sizeof(B._BatchCompact) == 24
    assert C.sizeof(B._Response) == 56 and C.sizeof(B._Init) == 8
    assert N.lib.fnnue_backend_go_compact(None, None, 0, None, 0, None, None, None, 0) == -1
    assert N.lib.fnnue_backend_go_timeout(None, None, 0, None, 0, None, None, 5) == -1
    assert N.ERRORS[-11] == "FNNUE_E_TIMEOUT"
