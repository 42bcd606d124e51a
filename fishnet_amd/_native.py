"""ctypes binding of libfnnue.so — the C ABI declared in include/fnnue.h.

The library is built in-tree (``fishnet_amd/libfnnue.so``, see
``fishnet_amd/csrc/Makefile`` / ``__graft_entry__.build``).  There is no
fallback: if the library cannot be loaded, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

LIB_PATH = os.environ.get("FNNUE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfnnue.so")

FNNUE_OK = 0
ERRORS = {
    -1: "FNNUE_E_ARG", -2: "FNNUE_E_IO", -3: "FNNUE_E_FORMAT", -4: "FNNUE_E_ARCH",
    -5: "FNNUE_E_DEVICE", -6: "FNNUE_E_POSITION", -7: "FNNUE_E_OOM", -8: "FNNUE_E_MOVE",
    -9: "FNNUE_E_FEN", -10: "FNNUE_E_CAPACITY", -11: "FNNUE_E_TIMEOUT",
}
SYNTH_LEB128, SYNTH_WRAP, SYNTH_FC1_PAD = 1, 2, 4
GROUP_CHAIN, GROUP_STAR = 0, 1
TIMING_OFF, TIMING_ALL, TIMING_FT = 0, 1, 2  # fnnue_ctx_set_timing
FT_SLICED, FT_GATHER, FT_AUTO = 0, 1, 2
FT_GATHER_MAX = 16384  # FNNUE_FT_AUTO gathers chess positions calls up to this size
PLAYOUT_FINAL, PLAYOUT_PLIES, PLAYOUT_CHILDREN = 0, 1, 2
VARIANT_CHESS, VARIANT_CRAZYHOUSE, VARIANT_ATOMIC = 0, 1, 2
POS_BYTES = 36
VPOS_BYTES = 48


class FnnueError(RuntimeError):
    """A nonzero FNNUE_E_* return code (maps to fishnet's PositionFailed)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"{ERRORS.get(code, code)}: {message}")
        self.code = code
        self.name = ERRORS.get(code, str(code))


def _load() -> C.CDLL:
    # libfnnue.so and torch's bundled ROCm runtime share the soname
    # libamdhip64.so.7; whichever loads first serves the whole process.  Load
    # torch's first (when torch is installed) so that tensors allocated by
    # torch and the library's kernels live in one HIP runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run `make -C fishnet_amd/csrc` or __graft_entry__.build()")
    return C.CDLL(LIB_PATH)


lib = _load()

_vp, _sz, _u32, _u64, _i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int
_P = C.POINTER

SIGNATURES = {
    "fnnue_last_error": ([], C.c_char_p),
    "fnnue_abi_version": ([], _u32),
    "fnnue_net_load": ([C.c_char_p, _P(_vp)], _i32),
    "fnnue_net_load_mem": ([_vp, _sz, _P(_vp)], _i32),
    "fnnue_net_info": ([_vp, _P(_u32), _P(_u32), _P(C.c_char_p)], _i32),
    "fnnue_net_free": ([_vp], None),
    "fnnue_net_sha256": ([_vp, _vp], _i32),
    "fnnue_net_synthesize": ([_u64, _u32, _u32, _P(_vp), _P(_sz)], _i32),
    "fnnue_buffer_free": ([_vp], None),
    "fnnue_device_count": ([_P(_i32)], _i32),
    "fnnue_ctx_create": ([_vp, _i32, _P(_vp)], _i32),
    "fnnue_net_image_size": ([_vp, _P(_sz)], _i32),
    "fnnue_net_image_pack": ([_vp, _vp, _sz], _i32),
    "fnnue_ctx_create_from_image": ([_i32, _u32, _vp, _sz, _P(_vp)], _i32),
    "fnnue_ctx_image": ([_vp, _P(_vp), _P(_sz)], _i32),
    "fnnue_ctx_free": ([_vp], None),
    "fnnue_eval_positions": ([_vp, _vp, _sz, _vp, _vp], _i32),
    "fnnue_eval_groups": ([_vp, _vp, _sz, _vp, _sz, _i32, _vp, _vp], _i32),
    "fnnue_eval_positions_device": ([_vp, _vp, _sz, _vp, _vp, _vp], _i32),
    "fnnue_eval_groups_device": ([_vp, _vp, _vp, _sz, _sz, _i32, _vp, _vp, _vp], _i32),
    "fnnue_eval_groups_dual_device": ([_vp, _vp, _vp, _vp, _sz, _sz, _i32, _vp, _vp, _vp, _vp, _vp], _i32),
    "fnnue_ctx_check": ([_vp], _i32),
    "fnnue_pos_from_fen": ([C.c_char_p, _vp], _i32),
    "fnnue_game_positions": ([C.c_char_p, C.c_char_p, _vp, _sz, _P(_sz)], _i32),
    "fnnue_game_children": ([C.c_char_p, C.c_char_p, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)], _i32),
    "fnnue_random_playouts": ([_u64, _sz, _u32, _u32, _i32, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)], _i32),
    "fnnue_perft": ([C.c_char_p, _i32, _P(_u64)], _i32),
    "fnnue_selftest_mfma": ([_i32], _i32),
    "fnnue_ctx_set_timing": ([_vp, _i32], _i32),
    "fnnue_ctx_set_ft_impl": ([_vp, _i32], _i32),
    "fnnue_net_accumulator_bound": ([_vp, _P(C.c_int32)], _i32),
    "fnnue_ctx_swar": ([_vp, _P(_i32), _P(C.c_int32)], _i32),
    "fnnue_ctx_set_swar": ([_vp, _i32], _i32),
    "fnnue_ctx_timing_read": ([_vp, _P(_u32), _P(C.c_double), _P(C.c_double)], _i32),
    "fnnue_ctx_timing_phases": ([_vp, _P(_u32), _P(C.c_double), _P(C.c_double), _P(C.c_double)], _i32),
    "fnnue_build_batch_device": ([_vp, _vp, _vp, _vp, _sz, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz), _vp], _i32),
    "fnnue_build_batch": ([_vp, C.c_char_p, _sz, _vp, _vp, _sz, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)], _i32),
    "fnnue_perft_device": ([_vp, C.c_char_p, _i32, _P(_u64)], _i32),
    "fnnue_random_game": ([_u64, C.c_char_p, _u32, C.c_char_p, _sz, _P(_sz)], _i32),
    "fnnue_multi_create": ([_vp, _P(_i32), _i32, _P(_vp)], _i32),
    "fnnue_multi_free": ([_vp], None),
    "fnnue_multi_size": ([_vp, _P(_i32)], _i32),
    "fnnue_multi_ctx": ([_vp, _i32, _P(_vp)], _i32),
    "fnnue_multi_eval_positions": ([_vp, _vp, _sz, _vp, _vp], _i32),
    "fnnue_multi_eval_groups": ([_vp, _vp, _sz, _vp, _sz, _i32, _vp, _vp], _i32),
    "fnnue_multi_eval_positions_device": ([_vp, _P(_vp), _P(_sz), _P(_vp), _P(_vp), _P(_vp)], _i32),
    "fnnue_multi_eval_groups_device": ([_vp, _P(_vp), _P(_vp), _P(_sz), _P(_sz), _i32, _P(_vp), _P(_vp), _P(_vp)],
                                       _i32),
    "fnnue_multi_sync": ([_vp], _i32),
    "fnnue_multi_eval_vpositions": ([_vp, _vp, _sz, _vp, _vp], _i32),
    "fnnue_multi_eval_vpositions_device": ([_vp, _P(_vp), _P(_sz), _P(_vp), _P(_vp), _P(_vp)], _i32),
    "fnnue_multi_eval_vgroups_device": ([_vp, _P(_vp), _P(_vp), _P(_sz), _P(_sz), _i32, _P(_vp), _P(_vp), _P(_vp)],
                                        _i32),
    "fnnue_partition_groups": ([_vp, _sz, _i32, _vp], _i32),
    "fnnue_net_load_variant": ([C.c_char_p, _i32, _P(_vp)], _i32),
    "fnnue_net_load_variant_mem": ([_vp, _sz, _i32, _P(_vp)], _i32),
    "fnnue_net_variant": ([_vp, _P(_i32)], _i32),
    "fnnue_net_synthesize_variant": ([_u64, _u32, _i32, _u32, _P(_vp), _P(_sz)], _i32),
    "fnnue_vpos_from_fen": ([_i32, C.c_char_p, _vp], _i32),
    "fnnue_random_vpositions": ([_u64, _i32, _sz, _u32, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)], _i32),
    "fnnue_game_vpositions": ([_i32, C.c_char_p, C.c_char_p, _vp, _sz, _P(_sz)], _i32),
    "fnnue_game_vchildren": ([_i32, C.c_char_p, C.c_char_p, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)], _i32),
    "fnnue_vperft": ([_i32, C.c_char_p, _i32, _P(_u64)], _i32),
    "fnnue_game_end": ([_i32, C.c_char_p, C.c_char_p, _P(_i32)], _i32),
    "fnnue_random_vgame": ([_u64, _i32, C.c_char_p, _u32, C.c_char_p, _sz, _P(_sz)], _i32),
    "fnnue_random_vgames": ([_u64, _i32, _sz, _u32, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)], _i32),
    "fnnue_build_vbatch_device": ([_vp, _i32, _vp, _vp, _vp, _sz, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz), _vp],
                                  _i32),
    "fnnue_build_vbatch": ([_vp, _i32, C.c_char_p, _sz, _vp, _vp, _sz, _i32, _vp, _sz, _vp, _sz, _P(_sz), _P(_sz)],
                           _i32),
    "fnnue_eval_vpositions": ([_vp, _vp, _sz, _vp, _vp], _i32),
    "fnnue_eval_vpositions_device": ([_vp, _vp, _sz, _vp, _vp, _vp], _i32),
    "fnnue_eval_vgroups": ([_vp, _vp, _sz, _vp, _sz, _i32, _vp, _vp], _i32),
    "fnnue_eval_vgroups_device": ([_vp, _vp, _vp, _sz, _sz, _i32, _vp, _vp, _vp], _i32),
    # include/fnnue_backend.h
    "fnnue_backend_channel": ([_vp, _i32, _vp, _P(_vp)], _i32),
    "fnnue_backend_channel_nets": ([_vp, _i32, _vp, _P(_vp)], _i32),
    "fnnue_backend_free": ([_vp], None),
    "fnnue_backend_batch_size": ([_vp, _P(_sz)], _i32),
    "fnnue_backend_go": ([_vp, _vp, _sz, _vp, _sz, _vp, _vp], _i32),
    "fnnue_backend_go_timeout": ([_vp, _vp, _sz, _vp, _sz, _vp, _vp, _u32], _i32),
    "fnnue_backend_go_compact": ([_vp, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _u32], _i32),
    "fnnue_backend_analysis_json": ([_vp, _sz, C.c_char_p, _sz, _P(_sz)], _i32),
    "fnnue_backend_last_stats": ([_vp, _vp], _i32),
}

for _name, (_args, _res) in SIGNATURES.items():
    _fn = getattr(lib, _name)  # AttributeError here = symbol missing from the build
    _fn.argtypes = _args
    _fn.restype = _res


def check(rc: int) -> None:
    if rc != FNNUE_OK:
        raise FnnueError(rc, (lib.fnnue_last_error() or b"").decode(errors="replace"))


def ptr(a) -> int | None:
    """Host numpy array -> void* (None for None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def positions_array(n: int) -> np.ndarray:
    return np.zeros((n, POS_BYTES), dtype=np.uint8)


def vpositions_array(n: int) -> np.ndarray:
    return np.zeros((n, VPOS_BYTES), dtype=np.uint8)
