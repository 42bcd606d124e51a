"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

CPU restatement of Stockfish 15.1 NNUE (see nnue_oracle.c header: parity
unpinned — the reference's Stockfish submodule and net are absent).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build() -> None:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def _load() -> C.CDLL:
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    vp = C.c_void_p
    lib.oracle_net_load_mem.argtypes = [vp, C.c_size_t, C.POINTER(vp)]
    lib.oracle_net_load_mem.restype = C.c_int
    lib.oracle_net_free.argtypes = [vp]
    lib.oracle_net_hd.argtypes = [vp]
    lib.oracle_net_hd.restype = C.c_uint32
    lib.oracle_net_file_hash.argtypes = [vp]
    lib.oracle_net_file_hash.restype = C.c_uint32
    lib.oracle_net_hash.argtypes = [C.c_uint32]
    lib.oracle_net_hash.restype = C.c_uint32
    lib.oracle_ft_hash.argtypes = [C.c_uint32]
    lib.oracle_ft_hash.restype = C.c_uint32
    lib.oracle_eval_board.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    lib.oracle_eval_board.restype = C.c_int
    lib.oracle_eval_packed.argtypes = [vp, vp, C.c_size_t, vp, vp, C.c_int]
    lib.oracle_eval_packed.restype = C.c_int
    lib.cpu_simd_eval_packed.argtypes = [vp, vp, C.c_size_t, vp, vp, C.c_int]
    lib.cpu_simd_eval_packed.restype = C.c_int
    lib.cpu_simd_eval_groups.argtypes = [vp, vp, vp, C.c_size_t, C.c_int, vp, vp, C.c_int]
    lib.cpu_simd_eval_groups.restype = C.c_int
    lib.cpu_simd_eval_games.argtypes = [vp, C.c_char_p, vp, vp, C.c_size_t, vp, vp, vp, C.c_int]
    lib.cpu_simd_eval_games.restype = C.c_int
    lib.cpu_simd_isa512.restype = C.c_int
    lib.cpu_simd_set_isa.argtypes = [C.c_int]
    lib.cpu_simd_set_isa.restype = C.c_int
    lib.oracle_eval_game.argtypes = [vp, C.c_char_p, C.c_char_p, vp, vp, C.c_long]
    lib.oracle_eval_game.restype = C.c_long
    lib.oracle_features.argtypes = [vp, C.c_int, vp]
    lib.oracle_features.restype = C.c_int
    lib.oracle_make_index.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
    lib.oracle_make_index.restype = C.c_int
    lib.oracle_eval_trace.argtypes = [vp, vp, C.c_int, vp, vp, vp]
    lib.oracle_eval_trace.restype = C.c_int
    lib.oracle_board_from_fen.argtypes = [C.c_char_p, vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.oracle_board_from_fen.restype = C.c_int
    lib.oracle_apply_uci.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p]
    lib.oracle_apply_uci.restype = C.c_int
    lib.oracle_net_load_variant_mem.argtypes = [vp, C.c_size_t, C.c_int, C.POINTER(vp)]
    lib.oracle_net_load_variant_mem.restype = C.c_int
    lib.voracle_eval_packed.argtypes = [vp, vp, C.c_size_t, vp, vp, C.c_int]
    lib.voracle_eval_packed.restype = C.c_int
    lib.voracle_eval_groups.argtypes = [vp, vp, vp, C.c_size_t, C.c_int, vp, vp]
    lib.voracle_eval_groups.restype = C.c_int
    lib.voracle_features.argtypes = [C.c_int, vp, C.c_int, vp]
    lib.voracle_features.restype = C.c_int
    lib.voracle_board_index.argtypes = [C.c_int] * 5
    lib.voracle_board_index.restype = C.c_int
    lib.voracle_hand_index.argtypes = [C.c_int] * 6
    lib.voracle_hand_index.restype = C.c_int
    return lib


lib = _load()

VARIANT_CRAZYHOUSE, VARIANT_ATOMIC = 1, 2
VPOS_BYTES = 48


class OracleNet:
    def __init__(self, data: bytes):
        self._h = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        rc = lib.oracle_net_load_mem(buf, len(data), C.byref(self._h))
        if rc != 0:
            raise ValueError(f"oracle rejected net (code {rc})")
        self.hd = lib.oracle_net_hd(self._h)
        self.file_hash = lib.oracle_net_file_hash(self._h)

    def eval_packed(self, pos: np.ndarray, threads: int = 1) -> tuple[np.ndarray, np.ndarray, int]:
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, 36)
        n = pos.shape[0]
        ps = np.zeros(n, dtype=np.int32)
        po = np.zeros(n, dtype=np.int32)
        rc = lib.oracle_eval_packed(self._h, pos.ctypes.data, n, ps.ctypes.data, po.ctypes.data, threads)
        return ps, po, rc

    def simd_eval_packed(self, pos: np.ndarray, threads: int = 1) -> tuple[np.ndarray, np.ndarray, int]:
        """AVX2 restatement of the engine's evaluation (nnue_cpu_simd.c): the cpu_baseline."""
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, 36)
        n = pos.shape[0]
        ps = np.zeros(n, dtype=np.int32)
        po = np.zeros(n, dtype=np.int32)
        rc = lib.cpu_simd_eval_packed(self._h, pos.ctypes.data, n, ps.ctypes.data, po.ctypes.data, threads)
        return ps, po, rc

    def simd_eval_groups(self, pos: np.ndarray, off: np.ndarray, mode: int,
                         threads: int = 1) -> tuple[np.ndarray, np.ndarray, int]:
        """Incremental accumulators along CHAIN (mode 0) / STAR (mode 1) groups, AVX2."""
        pos = np.ascontiguousarray(pos, dtype=np.uint8).reshape(-1, 36)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = pos.shape[0]
        assert len(off) >= 1 and int(off[-1]) == n
        ps = np.zeros(n, dtype=np.int32)
        po = np.zeros(n, dtype=np.int32)
        rc = lib.cpu_simd_eval_groups(self._h, pos.ctypes.data, off.ctypes.data, len(off) - 1, mode,
                                      ps.ctypes.data, po.ctypes.data, threads)
        return ps, po, rc

    def simd_eval_games(self, text: bytes, fen_off: np.ndarray, mv_off: np.ndarray, out_off: np.ndarray,
                        threads: int = 1) -> tuple[np.ndarray, np.ndarray, int]:
        """Whole analysis batches on the CPU: FEN parse + UCI replay + every ply
        evaluated along the game (fishnet_amd.pack_games text layout; out_off =
        per-game result offsets), AVX2 / AVX-512."""
        fen_off = np.ascontiguousarray(fen_off, dtype=np.uint32)
        mv_off = np.ascontiguousarray(mv_off, dtype=np.uint32)
        out_off = np.ascontiguousarray(out_off, dtype=np.uint32)
        n = int(out_off[-1])
        ps = np.zeros(max(n, 1), dtype=np.int32)
        po = np.zeros(max(n, 1), dtype=np.int32)
        rc = lib.cpu_simd_eval_games(self._h, text, fen_off.ctypes.data, mv_off.ctypes.data, len(mv_off),
                                     out_off.ctypes.data, ps.ctypes.data, po.ctypes.data, threads)
        return ps[:n], po[:n], rc

    def eval_board(self, board: np.ndarray, stm: int) -> tuple[int, int]:
        board = np.ascontiguousarray(board, dtype=np.uint8)
        a, b = C.c_int32(), C.c_int32()
        if lib.oracle_eval_board(self._h, board.ctypes.data, stm, C.byref(a), C.byref(b)) != 0:
            raise ValueError("invalid board")
        return a.value, b.value

    def eval_game(self, fen: str, moves: str) -> tuple[np.ndarray, np.ndarray]:
        cap = moves.count(" ") + 2
        ps = np.zeros(cap, dtype=np.int32)
        po = np.zeros(cap, dtype=np.int32)
        k = lib.oracle_eval_game(self._h, fen.encode(), moves.encode(), ps.ctypes.data, po.ctypes.data, cap)
        if k < 0:
            raise ValueError(f"oracle game replay failed ({k})")
        return ps[:k], po[:k]

    def trace(self, board: np.ndarray, stm: int):
        board = np.ascontiguousarray(board, dtype=np.uint8)
        x = np.zeros(self.hd, dtype=np.uint8)
        y = np.zeros(16, dtype=np.int32)
        acc = np.zeros(2 * self.hd, dtype=np.int16)
        b = lib.oracle_eval_trace(self._h, board.ctypes.data, stm, x.ctypes.data, y.ctypes.data, acc.ctypes.data)
        return b, x, y, acc

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and lib is not None:
            lib.oracle_net_free(self._h)
            self._h = C.c_void_p()


class VariantOracleNet:
    """Fairy-Stockfish variant net (variant_oracle.c restatement; parity unpinned)."""

    def __init__(self, data: bytes, variant: int):
        self._h = C.c_void_p()
        buf = C.create_string_buffer(data, len(data))
        rc = lib.oracle_net_load_variant_mem(buf, len(data), variant, C.byref(self._h))
        if rc != 0:
            raise ValueError(f"oracle rejected variant net (code {rc})")
        self.variant = variant
        self.hd = lib.oracle_net_hd(self._h)

    def eval_packed(self, vpos: np.ndarray, threads: int = 1):
        vpos = np.ascontiguousarray(vpos, dtype=np.uint8).reshape(-1, VPOS_BYTES)
        n = vpos.shape[0]
        ps, po = np.zeros(n, np.int32), np.zeros(n, np.int32)
        rc = lib.voracle_eval_packed(self._h, vpos.ctypes.data, n, ps.ctypes.data, po.ctypes.data, threads)
        return ps, po, rc

    def eval_groups(self, vpos: np.ndarray, off: np.ndarray, mode: int):
        vpos = np.ascontiguousarray(vpos, dtype=np.uint8).reshape(-1, VPOS_BYTES)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = vpos.shape[0]
        ps, po = np.zeros(n, np.int32), np.zeros(n, np.int32)
        rc = lib.voracle_eval_groups(self._h, vpos.ctypes.data, off.ctypes.data, len(off) - 1, mode,
                                     ps.ctypes.data, po.ctypes.data)
        return ps, po, rc

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value and lib is not None:
            lib.oracle_net_free(self._h)
            self._h = C.c_void_p()


def variant_features(variant: int, vpos48: np.ndarray, persp: int) -> list[int]:
    out = np.zeros(64, dtype=np.int32)
    p = np.ascontiguousarray(vpos48, dtype=np.uint8)
    k = lib.voracle_features(variant, p.ctypes.data, persp, out.ctypes.data)
    if k < 0:
        raise ValueError("invalid variant position")
    return sorted(out[:k].tolist())


def unpack(pos36: np.ndarray) -> tuple[np.ndarray, int]:
    b = np.zeros(64, dtype=np.uint8)
    b[0::2] = pos36[:32] & 15
    b[1::2] = pos36[:32] >> 4
    return b, int(pos36[32])


def pack(board: np.ndarray, stm: int) -> np.ndarray:
    p = np.zeros(36, dtype=np.uint8)
    p[:32] = (board[0::2] & 15) | ((board[1::2] & 15) << 4)
    p[32] = stm
    return p


def features(board: np.ndarray, persp: int) -> list[int]:
    out = np.zeros(64, dtype=np.int32)
    board = np.ascontiguousarray(board, dtype=np.uint8)
    k = lib.oracle_features(board.ctypes.data, persp, out.ctypes.data)
    if k < 0:
        raise ValueError("invalid board")
    return sorted(out[:k].tolist())


def board_from_fen(fen: str) -> tuple[np.ndarray, int]:
    b = np.zeros(64, dtype=np.uint8)
    stm, ep = C.c_int(), C.c_int()
    if lib.oracle_board_from_fen(fen.encode(), b.ctypes.data, C.byref(stm), C.byref(ep)) != 0:
        raise ValueError("bad fen")
    return b, stm.value
