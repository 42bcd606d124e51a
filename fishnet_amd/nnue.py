"""Host-side API of the MI355X NNUE evaluator over the C ABI.

Mirrors what the reference does on its static-evaluation path:

* ``Net.load(path)`` — ``setoption name EvalFile value <path>``
  ([ref] src/stockfish.rs:209-211; net file from src/assets.rs:128-133).
* ``Evaluator(net, device)`` — one engine per worker becomes one context per
  GPU ([ref] src/stockfish.rs:23-38 ``channel``; src/main.rs:158-170).
* ``Evaluator.eval_positions`` / ``eval_groups`` — batched replacement for one
  ``position fen ... moves ...`` round trip per position
  ([ref] src/stockfish.rs:274-283).
* ``game_positions`` — the per-ply expansion of an analysis batch
  ([ref] src/queue.rs:543-600, ``IncomingBatch::from_acquired``).

Errors raise :class:`FnnueError`; the caller treats any of them as
``PositionFailed`` for the whole batch ([ref] src/queue.rs:207-213).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from ._native import FnnueError  # noqa: F401  (re-export)


class Net:
    """A parsed and validated .nnue network (immutable, shareable)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @classmethod
    def load(cls, path: str) -> "Net":
        h = C.c_void_p()
        N.check(N.lib.fnnue_net_load(path.encode(), C.byref(h)))
        return cls(h.value)

    @classmethod
    def load_variant(cls, path: str, variant: int) -> "Net":
        """A Fairy-Stockfish variant net (VARIANT_CRAZYHOUSE / VARIANT_ATOMIC)."""
        h = C.c_void_p()
        N.check(N.lib.fnnue_net_load_variant(path.encode(), variant, C.byref(h)))
        return cls(h.value)

    @classmethod
    def from_bytes_variant(cls, data: bytes, variant: int) -> "Net":
        h = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        N.check(N.lib.fnnue_net_load_variant_mem(buf, len(data), variant, C.byref(h)))
        return cls(h.value)

    @property
    def variant(self) -> int:
        v = C.c_int()
        N.check(N.lib.fnnue_net_variant(self._h, C.byref(v)))
        return v.value

    @classmethod
    def from_bytes(cls, data: bytes) -> "Net":
        h = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        N.check(N.lib.fnnue_net_load_mem(buf, len(data), C.byref(h)))
        return cls(h.value)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def info(self) -> tuple[int, int, str]:
        hd, fh, desc = C.c_uint32(), C.c_uint32(), C.c_char_p()
        N.check(N.lib.fnnue_net_info(self._h, C.byref(hd), C.byref(fh), C.byref(desc)))
        return hd.value, fh.value, desc.value.decode(errors="replace")

    def sha256(self) -> str:
        """SHA-256 of the file bytes, lowercase hex (net identity)."""
        d = (C.c_uint8 * 32)()
        N.check(N.lib.fnnue_net_sha256(self._h, d))
        return bytes(d).hex()

    def accumulator_bound(self) -> int:
        """Largest possible |sum| of an even accumulator column (< 2^15: SWAR rows exact)."""
        b = C.c_int32()
        N.check(N.lib.fnnue_net_accumulator_bound(self._h, C.byref(b)))
        return b.value

    def image(self) -> np.ndarray:
        size = C.c_size_t()
        N.check(N.lib.fnnue_net_image_size(self._h, C.byref(size)))
        buf = np.zeros(size.value, dtype=np.uint8)
        N.check(N.lib.fnnue_net_image_pack(self._h, N.ptr(buf), size.value))
        return buf

    def __del__(self):
        # at interpreter shutdown the module globals may already be gone
        lib = getattr(N, "lib", None) if N is not None else None
        if lib is not None and getattr(self, "_h", None) and self._h.value:
            lib.fnnue_net_free(self._h)
            self._h = C.c_void_p()


def synthesize_net(seed: int, hd: int = 1024, flags: int = 0) -> bytes:
    """Deterministic synthetic net in the exact .nnue format."""
    buf, size = C.c_void_p(), C.c_size_t()
    N.check(N.lib.fnnue_net_synthesize(seed, hd, flags, C.byref(buf), C.byref(size)))
    try:
        return C.string_at(buf.value, size.value)
    finally:
        N.lib.fnnue_buffer_free(buf)


def synthesize_variant_net(seed: int, hd: int, variant: int, flags: int = 0) -> bytes:
    """Deterministic synthetic Fairy-Stockfish variant net in the .nnue format."""
    buf, size = C.c_void_p(), C.c_size_t()
    N.check(N.lib.fnnue_net_synthesize_variant(seed, hd, variant, flags, C.byref(buf), C.byref(size)))
    try:
        return C.string_at(buf.value, size.value)
    finally:
        N.lib.fnnue_buffer_free(buf)


def vpos_from_fen(variant: int, fen: str) -> np.ndarray:
    out = N.vpositions_array(1)
    N.check(N.lib.fnnue_vpos_from_fen(variant, fen.encode(), N.ptr(out)))
    return out[0]


def random_vpositions(seed: int, variant: int, count: int, max_plies: int = 120, mode: int = N.PLAYOUT_FINAL):
    """Seeded pseudo-legal random walks of a variant (test inputs).  FINAL ->
    positions; PLIES -> (positions, CHAIN group offsets)."""
    cap = count if mode == N.PLAYOUT_FINAL else count * (max_plies + 1)
    out = N.vpositions_array(cap)
    off = np.zeros(count + 1, dtype=np.uint32)
    n, g = C.c_size_t(), C.c_size_t()
    N.check(N.lib.fnnue_random_vpositions(seed, variant, count, max_plies, mode, N.ptr(out), cap, N.ptr(off), len(off),
                                          C.byref(n), C.byref(g)))
    if mode == N.PLAYOUT_FINAL:
        return out[: n.value]
    return out[: n.value], off[: g.value + 1]


def game_vpositions(variant: int, fen: str, moves: str | list[str]) -> np.ndarray:
    """Root + the position after every move of a variant game (host replay)."""
    if not isinstance(moves, str):
        moves = " ".join(moves)
    n = C.c_size_t()
    cap = moves.count(" ") + 2 if moves.strip() else 1
    out = N.vpositions_array(cap)
    N.check(N.lib.fnnue_game_vpositions(variant, fen.encode(), moves.encode(), N.ptr(out), cap, C.byref(n)))
    return out[: n.value]


def game_vchildren(variant: int, fen: str, moves: str | list[str]) -> tuple[np.ndarray, np.ndarray]:
    """Every ply of a variant game plus its legal children (drops included), STAR groups."""
    if not isinstance(moves, str):
        moves = " ".join(moves)
    nply = (moves.count(" ") + 2) if moves.strip() else 1
    n, g = C.c_size_t(), C.c_size_t()
    off = np.zeros(nply + 1, dtype=np.uint32)
    rc = N.lib.fnnue_game_vchildren(variant, fen.encode(), moves.encode(), None, 0, N.ptr(off), len(off),
                                    C.byref(n), C.byref(g))
    if rc != -10:
        N.check(rc)
    out = N.vpositions_array(n.value)
    N.check(N.lib.fnnue_game_vchildren(variant, fen.encode(), moves.encode(), N.ptr(out), len(out), N.ptr(off),
                                       len(off), C.byref(n), C.byref(g)))
    return out[: n.value], off[: g.value + 1]


END_NO_MOVES, END_CHECK, END_EXTINCT = 1, 2, 4


def game_end(fen: str, moves: str | list[str] = "", variant: int = 0) -> int:
    """FNNUE_END_* flags of the position after `moves` (host replay): no legal
    move, side to move in check, its king exploded (atomic)."""
    if not isinstance(moves, str):
        moves = " ".join(moves)
    flags = C.c_int()
    N.check(N.lib.fnnue_game_end(variant, fen.encode(), moves.encode(), C.byref(flags)))
    return flags.value


def vperft(variant: int, fen: str, depth: int) -> int:
    nodes = C.c_uint64()
    N.check(N.lib.fnnue_vperft(variant, fen.encode(), depth, C.byref(nodes)))
    return nodes.value


def random_vgame(seed: int, variant: int, fen: str, plies: int) -> str:
    """Up to `plies` random legal moves of a variant game as UCI (drops "N@f3")."""
    n = C.c_size_t()
    buf = C.create_string_buffer(8 * plies + 16)
    N.check(N.lib.fnnue_random_vgame(seed, variant, fen.encode(), plies, buf, len(buf), C.byref(n)))
    return buf.value.decode()


def random_vgames(seed: int, variant: int, count: int, max_plies: int = 160, threads: int = 8):
    """Every ply of seeded random legal variant games, CHAIN groups -> (positions, offsets)."""
    cap = count * (max_plies + 1)
    out = N.vpositions_array(cap)
    off = np.zeros(count + 1, dtype=np.uint32)
    n, g = C.c_size_t(), C.c_size_t()
    N.check(N.lib.fnnue_random_vgames(seed, variant, count, max_plies, threads, N.ptr(out), cap, N.ptr(off), len(off),
                                      C.byref(n), C.byref(g)))
    return out[: n.value], off[: g.value + 1]


def device_count() -> int:
    n = C.c_int()
    N.check(N.lib.fnnue_device_count(C.byref(n)))
    return n.value


class Evaluator:
    """A net resident on one GPU (one per process/GPU)."""

    def __init__(self, net: Net | None, device: int = 0, *, image_ptr: int | None = None,
                 image_bytes: int = 0, hd: int = 0):
        h = C.c_void_p()
        if net is not None:
            N.check(N.lib.fnnue_ctx_create(net.handle, device, C.byref(h)))
        else:
            N.check(N.lib.fnnue_ctx_create_from_image(device, hd, C.c_void_p(image_ptr), image_bytes, C.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def device_image(self) -> tuple[int, int]:
        p, s = C.c_void_p(), C.c_size_t()
        N.check(N.lib.fnnue_ctx_image(self._h, C.byref(p), C.byref(s)))
        return p.value, s.value

    def eval_positions(self, pos: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, N.POS_BYTES)
        n = pos.shape[0]
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_eval_positions(self._h, N.ptr(pos), n, N.ptr(psqt), N.ptr(positional)))
        return psqt, positional

    def eval_groups(self, pos: np.ndarray, off: np.ndarray, mode: int = N.GROUP_CHAIN):
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, N.POS_BYTES)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        if len(off) < 1:
            raise ValueError("off needs at least one entry (off[0] = 0)")
        n = pos.shape[0]
        if int(off[-1]) != n:
            raise ValueError(f"off[-1] = {int(off[-1])} but {n} positions were given")
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_eval_groups(self._h, N.ptr(pos), n, N.ptr(off), len(off) - 1, mode,
                                        N.ptr(psqt), N.ptr(positional)))
        return psqt, positional

    def eval_vpositions(self, vpos: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """Fairy-Stockfish variant positions (fnnue_vpos, 48 B) on a variant-net context."""
        vpos = np.ascontiguousarray(vpos, dtype=np.uint8).reshape(-1, N.VPOS_BYTES)
        n = vpos.shape[0]
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_eval_vpositions(self._h, N.ptr(vpos), n, N.ptr(psqt), N.ptr(positional)))
        return psqt, positional

    def eval_vgroups(self, vpos: np.ndarray, off: np.ndarray, mode: int = N.GROUP_CHAIN):
        """Variant positions in CHAIN / STAR groups, accumulators carried along (incremental)."""
        vpos = np.ascontiguousarray(vpos, dtype=np.uint8).reshape(-1, N.VPOS_BYTES)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        if len(off) < 1 or int(off[-1]) != vpos.shape[0]:
            raise ValueError("off must have >= 1 entry and end at the number of positions")
        n = vpos.shape[0]
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_eval_vgroups(self._h, N.ptr(vpos), n, N.ptr(off), len(off) - 1, mode, N.ptr(psqt),
                                         N.ptr(positional)))
        return psqt, positional

    def eval_vgroups_device(self, d_pos: int, d_off: int, ngroups: int, npos: int, mode: int, d_psqt: int,
                            d_positional: int, stream: int | None):
        N.check(N.lib.fnnue_eval_vgroups_device(self._h, C.c_void_p(d_pos), C.c_void_p(d_off), ngroups, npos, mode,
                                                C.c_void_p(d_psqt), C.c_void_p(d_positional), C.c_void_p(stream)))

    def eval_vpositions_device(self, d_pos: int, n: int, d_psqt: int, d_positional: int, stream: int | None):
        N.check(N.lib.fnnue_eval_vpositions_device(self._h, C.c_void_p(d_pos), n, C.c_void_p(d_psqt),
                                                   C.c_void_p(d_positional), C.c_void_p(stream)))

    # Device-pointer entry points (inputs resident in HBM; asynchronous).
    def eval_positions_device(self, d_pos: int, n: int, d_psqt: int, d_positional: int, stream: int | None):
        N.check(N.lib.fnnue_eval_positions_device(self._h, C.c_void_p(d_pos), n, C.c_void_p(d_psqt),
                                                  C.c_void_p(d_positional), C.c_void_p(stream)))

    def eval_groups_device(self, d_pos: int, d_off: int, ngroups: int, npos: int, mode: int, d_psqt: int,
                           d_positional: int, stream: int | None):
        N.check(N.lib.fnnue_eval_groups_device(self._h, C.c_void_p(d_pos), C.c_void_p(d_off), ngroups, npos, mode,
                                               C.c_void_p(d_psqt), C.c_void_p(d_positional), C.c_void_p(stream)))

    def eval_groups_dual_device(self, small: "Evaluator", d_pos: int, d_off: int, ngroups: int, npos: int, mode: int,
                                d_psqt: int, d_positional: int, d_psqt_small: int, d_positional_small: int,
                                stream: int | None):
        """This (big) net and `small` over the same groups, one plan (fnnue_eval_groups_dual_device)."""
        N.check(N.lib.fnnue_eval_groups_dual_device(self._h, small._h, C.c_void_p(d_pos), C.c_void_p(d_off), ngroups,
                                                    npos, mode, C.c_void_p(d_psqt), C.c_void_p(d_positional),
                                                    C.c_void_p(d_psqt_small), C.c_void_p(d_positional_small),
                                                    C.c_void_p(stream)))

    def eval_groups_dual(self, small: "Evaluator", pos: np.ndarray, off: np.ndarray, mode: int = N.GROUP_CHAIN):
        """Host-buffer convenience over eval_groups_dual_device (torch for the device buffers)."""
        import torch
        dev = torch.device("cuda", self.device)
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, N.POS_BYTES)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = len(pos)
        d_pos = torch.from_numpy(pos).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        out = torch.zeros((4, max(n, 1)), dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        self.eval_groups_dual_device(small, d_pos.data_ptr(), d_off.data_ptr(), len(off) - 1, n, mode,
                                     out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), None)
        self.check()
        small.check()
        o = out[:, :n].cpu().numpy()
        return o[0], o[1], o[2], o[3]

    def check(self) -> None:
        N.check(N.lib.fnnue_ctx_check(self._h))

    # Device-side batch builder (fnnue_build_batch): games = [(fen, "uci uci ..."), ...].
    def build_batch(self, games, mode: int = N.PLAYOUT_PLIES) -> tuple[np.ndarray, np.ndarray]:
        text, fen_off, mv_off = pack_games(games)
        n, g = C.c_size_t(), C.c_size_t()
        rc = N.lib.fnnue_build_batch(self._h, text, len(text), N.ptr(fen_off), N.ptr(mv_off), len(games), mode,
                                     None, 0, None, 0, C.byref(n), C.byref(g))
        if rc != -10:  # FNNUE_E_CAPACITY reports the sizes; anything else is final
            N.check(rc)
            return N.positions_array(0), np.zeros(1, dtype=np.uint32)
        out = N.positions_array(n.value)
        off = np.zeros(g.value + 1, dtype=np.uint32)
        N.check(N.lib.fnnue_build_batch(self._h, text, len(text), N.ptr(fen_off), N.ptr(mv_off), len(games), mode,
                                        N.ptr(out), len(out), N.ptr(off), len(off), C.byref(n), C.byref(g)))
        return out[: n.value], off[: g.value + 1]

    # Variant games on the device (fnnue_build_vbatch): games = [(fen, "uci ..."), ...].
    def build_vbatch(self, variant: int, games, mode: int = N.PLAYOUT_PLIES) -> tuple[np.ndarray, np.ndarray]:
        text, fen_off, mv_off = pack_games(games)
        n, g = C.c_size_t(), C.c_size_t()
        rc = N.lib.fnnue_build_vbatch(self._h, variant, text, len(text), N.ptr(fen_off), N.ptr(mv_off), len(games),
                                      mode, None, 0, None, 0, C.byref(n), C.byref(g))
        if rc != -10:
            N.check(rc)
            return N.vpositions_array(0), np.zeros(1, dtype=np.uint32)
        out = N.vpositions_array(n.value)
        off = np.zeros(g.value + 1, dtype=np.uint32)
        N.check(N.lib.fnnue_build_vbatch(self._h, variant, text, len(text), N.ptr(fen_off), N.ptr(mv_off),
                                         len(games), mode, N.ptr(out), len(out), N.ptr(off), len(off), C.byref(n),
                                         C.byref(g)))
        return out[: n.value], off[: g.value + 1]

    def perft_device(self, fen: str, depth: int) -> int:
        nodes = C.c_uint64()
        N.check(N.lib.fnnue_perft_device(self._h, fen.encode(), depth, C.byref(nodes)))
        return nodes.value

    def set_ft_impl(self, impl: int) -> None:
        """FT_AUTO (default: gather for chess position calls of at most FT_GATHER_MAX positions,
        sliced otherwise and for every grouped call), FT_SLICED (LDS-stationary tiles) or
        FT_GATHER (per-position / per-group row gather)."""
        N.check(N.lib.fnnue_ctx_set_ft_impl(self._h, impl))

    def swar(self) -> tuple[bool, int]:
        """(SWAR row sums on, the net's accumulator bound)."""
        e, b = C.c_int(), C.c_int32()
        N.check(N.lib.fnnue_ctx_swar(self._h, C.byref(e), C.byref(b)))
        return bool(e.value), b.value

    def set_swar(self, enable: bool) -> None:
        N.check(N.lib.fnnue_ctx_set_swar(self._h, 1 if enable else 0))

    def set_timing(self, enable, ft_only: bool = False) -> None:
        """Events around every phase (plan / FT kernel / stacks), or with ft_only
        only the two around the FT main kernel (FNNUE_TIMING_FT: each event
        record costs the stream a few microseconds)."""
        N.check(N.lib.fnnue_ctx_set_timing(self._h, (N.TIMING_FT if ft_only else N.TIMING_ALL) if enable else N.TIMING_OFF))

    def timing_phases(self) -> tuple[int, float, float, float]:
        """(timed launches, summed ms of the FT plan kernels, of the FT main kernel, of the layer stacks); resets."""
        n, a, b, c = C.c_uint32(), C.c_double(), C.c_double(), C.c_double()
        N.check(N.lib.fnnue_ctx_timing_phases(self._h, C.byref(n), C.byref(a), C.byref(b), C.byref(c)))
        return n.value, a.value, b.value, c.value

    def timing_read(self) -> tuple[int, float, float]:
        """(timed launches, summed feature-transformer ms, summed layer-stack ms); resets."""
        n, a, b = C.c_uint32(), C.c_double(), C.c_double()
        N.check(N.lib.fnnue_ctx_timing_read(self._h, C.byref(n), C.byref(a), C.byref(b)))
        return n.value, a.value, b.value

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            N.lib.fnnue_ctx_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        if N is not None and getattr(N, "lib", None) is not None:
            self.close()


class _BorrowedEvaluator(Evaluator):
    """The context of one device of a MultiEvaluator (owned by it)."""

    def __init__(self, handle: C.c_void_p, device: int):  # noqa: D401  (no ctx creation)
        self._h = handle
        self.device = device

    def close(self) -> None:
        self._h = C.c_void_p()


def _ptrs(vals) -> C.Array:
    return (C.c_void_p * len(vals))(*[C.c_void_p(v) for v in vals])


def _sizes(vals) -> C.Array:
    return (C.c_size_t * len(vals))(*vals)


def _streams(vals):
    return None if vals is None else _ptrs([v or 0 for v in vals])


class MultiEvaluator:
    """Several GPUs from one process (fnnue_multi_*): the net is RCCL-broadcast
    from devices[0]; batches are sharded without a data-path collective.  The
    reference's one-engine-per-core parallelism ([ref] src/main.rs:156-170)."""

    def __init__(self, net: Net, devices):
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        N.check(N.lib.fnnue_multi_create(net.handle, devs, len(devices), C.byref(h)))
        self._h = h
        self.devices = list(devices)

    def __len__(self) -> int:
        return len(self.devices)

    def ctx(self, i: int) -> Evaluator:
        h = C.c_void_p()
        N.check(N.lib.fnnue_multi_ctx(self._h, i, C.byref(h)))
        return _BorrowedEvaluator(h, self.devices[i])

    def eval_positions(self, pos: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, N.POS_BYTES)
        n = pos.shape[0]
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_multi_eval_positions(self._h, N.ptr(pos), n, N.ptr(psqt), N.ptr(positional)))
        return psqt, positional

    def eval_vpositions(self, vpos: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        vpos = np.ascontiguousarray(vpos, dtype=np.uint8).reshape(-1, N.VPOS_BYTES)
        n = vpos.shape[0]
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_multi_eval_vpositions(self._h, N.ptr(vpos), n, N.ptr(psqt), N.ptr(positional)))
        return psqt, positional

    def eval_groups(self, pos: np.ndarray, off: np.ndarray, mode: int = N.GROUP_CHAIN):
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, N.POS_BYTES)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        if len(off) < 1 or int(off[-1]) != pos.shape[0]:
            raise ValueError("off must have >= 1 entry and end at the number of positions")
        n = pos.shape[0]
        psqt = np.zeros(n, dtype=np.int32)
        positional = np.zeros(n, dtype=np.int32)
        N.check(N.lib.fnnue_multi_eval_groups(self._h, N.ptr(pos), n, N.ptr(off), len(off) - 1, mode,
                                              N.ptr(psqt), N.ptr(positional)))
        return psqt, positional

    # device-resident shards: one pointer / count per device (asynchronous; then
    # sync()).  streams: one hipStream_t handle per device (e.g. torch's
    # current stream of each device) or None for the contexts' own streams.
    def eval_positions_device(self, d_pos, n, d_psqt, d_positional, streams=None) -> None:
        N.check(N.lib.fnnue_multi_eval_positions_device(self._h, _ptrs(d_pos), _sizes(n), _ptrs(d_psqt),
                                                        _ptrs(d_positional), _streams(streams)))

    def eval_vpositions_device(self, d_pos, n, d_psqt, d_positional, streams=None) -> None:
        N.check(N.lib.fnnue_multi_eval_vpositions_device(self._h, _ptrs(d_pos), _sizes(n), _ptrs(d_psqt),
                                                         _ptrs(d_positional), _streams(streams)))

    def eval_vgroups_device(self, d_pos, d_off, ngroups, npos, mode, d_psqt, d_positional, streams=None) -> None:
        N.check(N.lib.fnnue_multi_eval_vgroups_device(self._h, _ptrs(d_pos), _ptrs(d_off), _sizes(ngroups),
                                                      _sizes(npos), mode, _ptrs(d_psqt), _ptrs(d_positional),
                                                      _streams(streams)))

    def eval_groups_device(self, d_pos, d_off, ngroups, npos, mode, d_psqt, d_positional, streams=None) -> None:
        N.check(N.lib.fnnue_multi_eval_groups_device(self._h, _ptrs(d_pos), _ptrs(d_off), _sizes(ngroups),
                                                     _sizes(npos), mode, _ptrs(d_psqt), _ptrs(d_positional),
                                                     _streams(streams)))

    def sync(self) -> None:
        N.check(N.lib.fnnue_multi_sync(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            N.lib.fnnue_multi_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        if N is not None and getattr(N, "lib", None) is not None:
            self.close()


def partition_groups(off: np.ndarray, nparts: int) -> np.ndarray:
    """Whole groups into nparts contiguous runs of about equal position counts
    (fnnue_partition_groups): part k = groups [cut[k], cut[k + 1])."""
    off = np.ascontiguousarray(off, dtype=np.uint32)
    cut = np.zeros(nparts + 1, dtype=np.uint32)
    N.check(N.lib.fnnue_partition_groups(N.ptr(off), len(off) - 1, nparts, N.ptr(cut)))
    return cut


def pos_from_fen(fen: str) -> np.ndarray:
    out = N.positions_array(1)
    N.check(N.lib.fnnue_pos_from_fen(fen.encode(), N.ptr(out)))
    return out[0]


def game_positions(fen: str, moves: str | list[str]) -> np.ndarray:
    """Root + the position after every move (analysis batch expansion)."""
    if not isinstance(moves, str):
        moves = " ".join(moves)
    n = C.c_size_t()
    cap = moves.count(" ") + 2 if moves.strip() else 1
    out = N.positions_array(cap)
    N.check(N.lib.fnnue_game_positions(fen.encode(), moves.encode(), N.ptr(out), cap, C.byref(n)))
    return out[: n.value]


def game_children(fen: str, moves: str | list[str]) -> tuple[np.ndarray, np.ndarray]:
    """Every ply plus its legal 1-ply children, as STAR groups."""
    if not isinstance(moves, str):
        moves = " ".join(moves)
    nply = (moves.count(" ") + 2) if moves.strip() else 1
    cap = nply * 256
    out = N.positions_array(cap)
    off = np.zeros(nply + 1, dtype=np.uint32)
    n, g = C.c_size_t(), C.c_size_t()
    N.check(N.lib.fnnue_game_children(fen.encode(), moves.encode(), N.ptr(out), cap, N.ptr(off), len(off),
                                      C.byref(n), C.byref(g)))
    return out[: n.value], off[: g.value + 1]


def random_playouts(seed: int, count: int, min_plies: int = 0, max_plies: int = 160,
                    mode: int = N.PLAYOUT_FINAL, threads: int = 8, cap: int | None = None):
    """Seeded random-playout positions.  FINAL -> positions;
    PLIES / CHILDREN -> (positions, group offsets)."""
    if cap is None:
        per = {N.PLAYOUT_FINAL: 1, N.PLAYOUT_PLIES: max_plies + 1, N.PLAYOUT_CHILDREN: (max_plies + 1) * 40}[mode]
        cap = count * per
    offcap = count * (max_plies + 1) + 1 if mode != N.PLAYOUT_FINAL else 1
    for _ in range(2):
        out = N.positions_array(cap)
        off = np.zeros(offcap, dtype=np.uint32)
        n, g = C.c_size_t(), C.c_size_t()
        rc = N.lib.fnnue_random_playouts(seed, count, min_plies, max_plies, mode, threads, N.ptr(out), cap,
                                         N.ptr(off), len(off), C.byref(n), C.byref(g))
        if rc == -10 and n.value > cap:  # FNNUE_E_CAPACITY: retry with the exact size
            cap = n.value
            continue
        N.check(rc)
        break
    if mode == N.PLAYOUT_FINAL:
        return out[: n.value]
    return out[: n.value], off[: g.value + 1]


def pack_games(games) -> tuple[bytes, np.ndarray, np.ndarray]:
    """[(fen, moves)] -> the builder's text layout: FEN g in [fen_off[g], mv_off[g]),
    its moves in [mv_off[g], fen_off[g + 1])."""
    parts, fen_off, mv_off, pos = [], [], [], 0
    for fen, moves in games:
        if not isinstance(moves, str):
            moves = " ".join(moves)
        f, m = fen.encode(), b" " + moves.encode()
        fen_off.append(pos)
        mv_off.append(pos + len(f))
        parts += [f, m]
        pos += len(f) + len(m)
    fen_off.append(pos)
    return b"".join(parts), np.array(fen_off, dtype=np.uint32), np.array(mv_off, dtype=np.uint32)


def random_game(seed: int, fen: str, plies: int) -> str:
    """Up to `plies` random legal moves from `fen` as space-separated UCI (test inputs)."""
    n = C.c_size_t()
    buf = C.create_string_buffer(8 * plies + 16)
    N.check(N.lib.fnnue_random_game(seed, fen.encode(), plies, buf, len(buf), C.byref(n)))
    return buf.value.decode()


def perft(fen: str, depth: int) -> int:
    nodes = C.c_uint64()
    N.check(N.lib.fnnue_perft(fen.encode(), depth, C.byref(nodes)))
    return nodes.value


def selftest_mfma(device: int = 0) -> None:
    N.check(N.lib.fnnue_selftest_mfma(device))
