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
