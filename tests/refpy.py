"""Second, independent restatement of SF 15.1 NNUE in numpy (test-only).

Used to cross-check the C oracle (oracle/nnue_oracle.c) on small cases, so a
slip in one restatement shows up as a disagreement.  Written from the same
upstream description (SURVEY.md §8a rows a1–a8) but structured differently:
vectorised numpy, explicit dtype wraparound.
"""
from __future__ import annotations

import struct

import numpy as np

VERSION = 0x7AF32F20
FEATURES = 22528
M32 = 0xFFFFFFFF


def _affine_hash(prev: int, out: int) -> int:
    return ((0xCC03DAE4 + out) ^ (prev >> 1) ^ (prev << 31)) & M32


def net_hash(hd: int) -> int:
    h = 0xEC42E90D ^ (2 * hd)
    h = _affine_hash(h, 16)
    h = (0x538D24C7 + h) & M32
    h = _affine_hash(h, 32)
    h = (0x538D24C7 + h) & M32
    return _affine_hash(h, 1)


def ft_hash(hd: int) -> int:
    return 0x7F234CB8 ^ (2 * hd)


class RefNet:
    """Plain-format parser (no LEB128; the C oracle covers that)."""

    def __init__(self, data: bytes):
        off = 0

        def take(dtype, count):
            nonlocal off
            a = np.frombuffer(data, dtype=dtype, count=count, offset=off)
            off += a.nbytes
            return a

        version, fhash, dlen = struct.unpack_from("<III", data, 0)
        assert version == VERSION
        off = 12 + dlen
        fth = struct.unpack_from("<I", data, off)[0]
        off += 4
        hd = (fth ^ 0x7F234CB8) // 2
        assert ft_hash(hd) == fth and fhash == ft_hash(hd) ^ net_hash(hd)
        self.hd = hd
        self.bias = take("<i2", hd).astype(np.int64)
        self.w = take("<i2", hd * FEATURES).reshape(FEATURES, hd).astype(np.int64)
        self.psqt = take("<i4", 8 * FEATURES).reshape(FEATURES, 8).astype(np.int64)
        self.stacks = []
        for _ in range(8):
            assert struct.unpack_from("<I", data, off)[0] == net_hash(hd)
            off += 4
            b0 = take("<i4", 16).astype(np.int64)
            w0 = take("i1", 16 * hd).reshape(16, hd).astype(np.int64)
            b1 = take("<i4", 32).astype(np.int64)
            w1 = take("i1", 32 * 32).reshape(32, 32).astype(np.int64)
            b2 = int(take("<i4", 1)[0])
            w2 = take("i1", 32).astype(np.int64)
            self.stacks.append((b0, w0, b1, w1, b2, w2))
        assert off == len(data)


KING_BUCKET = [-1] * 64
for _sq in range(64):
    _r, _f = divmod(_sq, 8)
    if _f >= 4:
        KING_BUCKET[_sq] = 4 * (7 - _r) + (7 - _f)


def feature(persp: int, sq: int, pc: int, ksq: int) -> int:
    flip = (56 if persp else 0) ^ (7 if (ksq % 8) < 4 else 0)
    ptype, color = pc & 7, pc >> 3
    plane = 10 if ptype == 6 else 2 * (ptype - 1) + (color != persp)
    return (sq ^ flip) + 64 * plane + 704 * KING_BUCKET[ksq ^ flip]


def _wrap16(a: np.ndarray) -> np.ndarray:
    return ((a + 32768) % 65536) - 32768


def _trunc_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def evaluate(net: RefNet, board: list[int] | np.ndarray, stm: int) -> tuple[int, int]:
    board = [int(x) for x in board]
    wk, bk = board.index(6), board.index(14)
    pieces = [(s, pc) for s, pc in enumerate(board) if pc]
    acc, psq = [], []
    for persp, ksq in ((0, wk), (1, bk)):
        idx = [feature(persp, s, pc, ksq) for s, pc in pieces]
        acc.append(_wrap16(net.bias + net.w[idx].sum(axis=0)))
        psq.append(net.psqt[idx].sum(axis=0))
    bucket = (len(pieces) - 1) // 4
    psqt = _trunc_div(int(psq[stm][bucket] - psq[1 - stm][bucket]), 2)
    half = net.hd // 2
    xs = []
    for persp in (stm, 1 - stm):
        a = np.clip(acc[persp][:half], 0, 127)
        b = np.clip(acc[persp][half:], 0, 127)
        xs.append((a * b) // 128)
    x = np.concatenate(xs)
    b0, w0, b1, w1, b2, w2 = net.stacks[bucket]
    y = b0 + w0 @ x
    sq = np.minimum(127, (y * y >> 12) // 128)
    cr = np.clip(y >> 6, 0, 127)
    x1 = np.concatenate([sq[:15], cr[:15], [0, 0]])
    z = b1 + w1 @ x1
    x2 = np.clip(z >> 6, 0, 127)
    out = b2 + int(w2 @ x2)
    fwd = _trunc_div(int(y[15]) * 9600, 8128)
    return psqt, out + fwd
