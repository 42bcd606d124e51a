"""fnnue_backend (include/fnnue_backend.h) in Python: fishnet's engine-actor
shape over the GPU evaluator.

Mirrors the reference's interface for this path:
  ``stockfish::channel(exe, init, logger) -> (StockfishStub, StockfishActor)``
  ([ref] src/stockfish.rs:23-38) and ``StockfishStub::go(Position) ->
  Result<PositionResponse, PositionFailed>`` (:44-54), with
  ``AcquireResponseBody`` (src/api.rs:293-309), ``PositionResponse`` /
  ``PositionFailed`` (src/ipc.rs:28-39, 100-103), ``Score`` (api.rs:383-388)
  and ``CompletedBatch::into_analysis`` (src/queue.rs:715-727).
Here ``go`` takes whole acquired batches (the GPU wants batches, not single
positions) and returns, per batch, its responses or a ``PositionFailed``.
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _native as N

WORK_ANALYSIS, WORK_MOVE = 0, 1
SCORE_CP, SCORE_MATE = 0, 1


class _Init(C.Structure):
    _fields_ = [("normalize_to_pawn", C.c_int32), ("timeout_ms", C.c_uint32)]


class _Acquired(C.Structure):
    _fields_ = [("batch_id", C.c_char_p), ("work", C.c_int), ("multipv", C.c_int), ("position", C.c_char_p),
                ("variant", C.c_char_p), ("moves", C.c_char_p), ("skip_positions", C.c_void_p),
                ("nskip", C.c_size_t)]


class _Response(C.Structure):
    _fields_ = [("position_id", C.c_uint32), ("skipped", C.c_uint8), ("score_kind", C.c_uint8),
                ("depth", C.c_uint8), ("matrix", C.c_uint8), ("score", C.c_int64), ("psqt", C.c_int32),
                ("positional", C.c_int32), ("nodes", C.c_uint64), ("time_ms", C.c_uint64), ("nps", C.c_uint32),
                ("best_move", C.c_char * 8)]


class _Compact(C.Structure):
    _fields_ = [("psqt", C.c_int32), ("positional", C.c_int32), ("score", C.c_int32), ("score_kind", C.c_uint8),
                ("depth", C.c_uint8), ("flags", C.c_uint8), ("reserved", C.c_uint8)]


class _BatchCompact(C.Structure):
    _fields_ = [("time_ms", C.c_uint64), ("nps", C.c_uint32), ("nodes", C.c_uint32), ("best_move", C.c_char * 8)]


COMPACT_SKIPPED, COMPACT_MATRIX, COMPACT_NO_MOVES = 1, 2, 4


@dataclass
class AcquireResponseBody:
    """One acquired batch: work type + id, root FEN, variant, UCI moves, skipPositions."""
    batch_id: str
    position: str
    moves: str | Sequence[str] = ""
    work: str = "analysis"            # "analysis" | "move"
    variant: str = "standard"
    skip_positions: Sequence[int] = ()
    multipv: int | None = None


@dataclass
class Score:
    kind: str   # "cp" | "mate"
    value: int


@dataclass
class PositionResponse:
    position_id: int
    score: Score | None               # None for Skip::Skip
    psqt: int = 0
    positional: int = 0
    depth: int = 0
    nodes: int = 0
    time_ms: int = 0
    nps: int = 0
    best_move: str | None = None
    skipped: bool = False
    matrix: bool = False              # AnalysisPart::Matrix (the batch asked for multipv)


@dataclass
class PositionFailed(Exception):
    batch_id: str
    code: int = 0
    message: str = field(default="")

    def __str__(self) -> str:
        return f"PositionFailed({self.batch_id}): {N.ERRORS.get(self.code, self.code)} {self.message}"


def batch_size(body: AcquireResponseBody) -> int:
    """Responses the batch expands to (IncomingBatch::from_acquired): moves + 1, or 1 for move work."""
    a, _keep = _acquired([body])
    n = C.c_size_t()
    N.check(N.lib.fnnue_backend_batch_size(C.byref(a[0]), C.byref(n)))
    return n.value


def _acquired(bodies: Sequence[AcquireResponseBody]):
    arr = (_Acquired * max(1, len(bodies)))()
    keep = []
    for i, b in enumerate(bodies):
        moves = b.moves if isinstance(b.moves, str) else " ".join(b.moves)
        skip = np.ascontiguousarray(np.asarray(list(b.skip_positions), dtype=np.uint32))
        keep.append(skip)
        strs = [s.encode() for s in (b.batch_id, b.position, b.variant or "", moves)]
        keep += strs
        work = {"analysis": WORK_ANALYSIS, "move": WORK_MOVE}.get(b.work, -1)
        arr[i] = _Acquired(strs[0], work, int(b.multipv or 0), strs[1], strs[2], strs[3],
                           skip.ctypes.data if len(skip) else None, len(skip))
    return arr, keep


class GpuEvalActor:
    """The actor half: owns the worker thread and the evaluator (fnnue_backend)."""

    def __init__(self, handle: C.c_void_p):
        self._h = handle

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            N.lib.fnnue_backend_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        if N is not None and getattr(N, "lib", None) is not None:
            self.close()


class GpuEvalStub:
    """StockfishStub for the GPU backend: ``go`` sends batches over the channel."""

    def __init__(self, actor: GpuEvalActor):
        self._actor = actor

    def go(self, bodies: Sequence[AcquireResponseBody],
           timeout_ms: int = 0) -> list[list[PositionResponse] | PositionFailed]:
        """One go() over whole batches, within `timeout_ms` (0: the channel's
        budget).  A call that overruns it raises FnnueError FNNUE_E_TIMEOUT and
        breaks the channel (fnnue_backend_go_timeout); `last_batch_rc` then
        says which batches had been answered."""
        nb = len(bodies)
        if nb == 0:
            return []
        a, _keep = _acquired(bodies)
        cap = 0
        for b in bodies:
            moves = b.moves if isinstance(b.moves, str) else " ".join(b.moves)
            cap += 1 if b.work == "move" else len(moves.split()) + 1
        out = (_Response * max(1, cap))()
        off = np.zeros(nb + 1, dtype=np.uint32)
        rc = np.zeros(nb, dtype=np.int32)
        self.last_batch_rc = rc
        t0 = time.perf_counter()
        ret = N.lib.fnnue_backend_go_timeout(self._actor._h, a, nb, out, cap, N.ptr(off), N.ptr(rc), int(timeout_ms))
        self.last_call_s = time.perf_counter() - t0  # the C call alone (not the ctypes marshalling around it)
        N.check(ret)
        res: list[list[PositionResponse] | PositionFailed] = []
        for i, b in enumerate(bodies):
            if rc[i]:
                res.append(PositionFailed(b.batch_id, int(rc[i])))
                continue
            rows = []
            for k in range(int(off[i]), int(off[i + 1])):
                r = out[k]
                if r.skipped:
                    rows.append(PositionResponse(r.position_id, None, skipped=True))
                    continue
                rows.append(PositionResponse(
                    r.position_id, Score("mate" if r.score_kind == SCORE_MATE else "cp", int(r.score)), r.psqt,
                    r.positional, r.depth, r.nodes, r.time_ms, r.nps, r.best_move.decode() or None,
                    matrix=bool(r.matrix)))
            res.append(rows)
        return res

    def go_compact(self, bodies: Sequence[AcquireResponseBody],
                   timeout_ms: int = 0) -> list[list[PositionResponse] | PositionFailed]:
        """go() through the compact form (fnnue_backend_go_compact: 16 B per
        position + 24 B per batch), expanded here into the same
        PositionResponses the full form gives."""
        nb = len(bodies)
        if nb == 0:
            return []
        a, _keep = _acquired(bodies)
        cap = sum(1 if b.work == "move" else len((b.moves if isinstance(b.moves, str) else " ".join(b.moves)).split()) + 1
                  for b in bodies)
        out = (_Compact * max(1, cap))()
        bout = (_BatchCompact * nb)()
        off = np.zeros(nb + 1, dtype=np.uint32)
        rc = np.zeros(nb, dtype=np.int32)
        self.last_batch_rc = rc
        t0 = time.perf_counter()
        ret = N.lib.fnnue_backend_go_compact(self._actor._h, a, nb, out, cap, bout, N.ptr(off), N.ptr(rc),
                                             int(timeout_ms))
        self.last_call_s = time.perf_counter() - t0
        N.check(ret)
        res: list[list[PositionResponse] | PositionFailed] = []
        for i, b in enumerate(bodies):
            if rc[i]:
                res.append(PositionFailed(b.batch_id, int(rc[i])))
                continue
            bt = bout[i]
            rows = []
            for k in range(int(off[i]), int(off[i + 1])):
                r = out[k]
                pid = k - int(off[i])
                if r.flags & COMPACT_SKIPPED:
                    rows.append(PositionResponse(pid, None, skipped=True))
                    continue
                move = b.work == "move"
                nodes = 0 if r.flags & COMPACT_NO_MOVES else (bt.nodes if move else 1)
                rows.append(PositionResponse(
                    pid, Score("mate" if r.score_kind == SCORE_MATE else "cp", int(r.score)), r.psqt, r.positional,
                    r.depth, nodes, bt.time_ms, bt.nps, (bt.best_move.decode() or None) if move else None,
                    matrix=bool(r.flags & COMPACT_MATRIX)))
            res.append(rows)
        return res

    def go_one(self, body: AcquireResponseBody) -> list[PositionResponse]:
        """One batch; raises PositionFailed like StockfishStub::go's Err."""
        r = self.go([body])[0]
        if isinstance(r, PositionFailed):
            raise r
        return r


class _Stats(C.Structure):
    _fields_ = [("prep_ms", C.c_double), ("device_ms", C.c_double), ("fill_ms", C.c_double), ("total_ms", C.c_double),
                ("positions", C.c_uint64), ("stream_syncs", C.c_uint32), ("rebuilds", C.c_uint32),
                ("host_threads", C.c_uint32), ("pieces", C.c_uint32)]


def last_stats(actor: "GpuEvalActor") -> dict:
    """fnnue_backend_last_stats: where the last go() spent its time."""
    st = _Stats()
    N.check(N.lib.fnnue_backend_last_stats(actor._h, C.byref(st)))
    return {k: getattr(st, k) for k, _ in _Stats._fields_}


class _Nets(C.Structure):
    _fields_ = [("chess", C.c_void_p), ("crazyhouse", C.c_void_p), ("atomic", C.c_void_p)]


def channel(net=None, device: int = 0, normalize_to_pawn: int = 0, *, crazyhouse=None,
            atomic=None, timeout_ms: int = 0) -> tuple[GpuEvalStub, GpuEvalActor]:
    """stockfish::channel for the GPU evaluator.  `net` (a fishnet_amd.Net)
    goes to the slot of its variant; `crazyhouse` / `atomic` add variant nets
    (fnnue_backend_channel_nets): each batch is evaluated by its variant's net.
    `timeout_ms`: the budget of each go() (0: 60 s, [ref] src/main.rs:316)."""
    h = C.c_void_p()
    init = _Init(normalize_to_pawn, timeout_ms)
    if crazyhouse is None and atomic is None:
        N.check(N.lib.fnnue_backend_channel(net._h, device, C.byref(init), C.byref(h)))
    else:
        nets = _Nets(net._h if net is not None else None, crazyhouse._h if crazyhouse is not None else None,
                     atomic._h if atomic is not None else None)
        N.check(N.lib.fnnue_backend_channel_nets(C.byref(nets), device, C.byref(init), C.byref(h)))
    actor = GpuEvalActor(h)
    return GpuEvalStub(actor), actor


def into_analysis(responses: Sequence[PositionResponse]) -> str:
    """The `analysis` JSON array of a completed analysis batch (fnnue_backend_analysis_json)."""
    arr = (_Response * max(1, len(responses)))()
    for i, r in enumerate(responses):
        if r.skipped:
            arr[i] = _Response(r.position_id, 1)
            continue
        kind = SCORE_MATE if r.score.kind == "mate" else SCORE_CP
        arr[i] = _Response(r.position_id, 0, kind, r.depth, 1 if r.matrix else 0, r.score.value, r.psqt,
                           r.positional, r.nodes, r.time_ms, r.nps, (r.best_move or "").encode())
    n = C.c_size_t()
    N.lib.fnnue_backend_analysis_json(arr, len(responses), None, 0, C.byref(n))
    buf = C.create_string_buffer(n.value + 1)
    N.check(N.lib.fnnue_backend_analysis_json(arr, len(responses), buf, len(buf), C.byref(n)))
    return buf.value.decode()
