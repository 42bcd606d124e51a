"""Incremental (grouped) evaluation of Fairy-Stockfish variant positions
(fnnue_eval_vgroups[_device]: the segment machinery of ft_segments.hip over
the variant feature sets, pocket changes as row adds / removes) against the
from-scratch GPU path and the CPU oracle (oracle/variant_oracle.c), bit-exact,
and end to end from the device batch builder.  Parity unpinned against
Fairy-Stockfish itself.  [ref] src/queue.rs:524-552 (every ply of
a variant game is evaluated), :530-539."""
import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from fishnet_amd import nnue
from oracle.oracle import VariantOracleNet

pytestmark = pytest.mark.gpu

ZH, AT = N.VARIANT_CRAZYHOUSE, N.VARIANT_ATOMIC
START = {ZH: "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1",
         AT: "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"}


@pytest.fixture(scope="module")
def vc():
    cache = {}

    def get(variant, hd=512, seed=5):
        key = (variant, hd, seed)
        if key not in cache:
            data = F.synthesize_variant_net(seed, hd, variant)
            cache[key] = (F.Evaluator(F.Net.from_bytes_variant(data, variant), 0), VariantOracleNet(data, variant))
        return cache[key]

    yield get
    for ev, _ in cache.values():
        ev.close()


def legal_games(variant, count, seed, plies=160):
    games = [(START[variant], nnue.random_vgame(seed + i, variant, START[variant], 20 + (i * 53) % plies))
             for i in range(count)]
    parts = [nnue.game_vpositions(variant, f, m) for f, m in games]
    off = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.uint32)
    return games, np.concatenate(parts), off


def kings(pos):
    b = np.zeros((len(pos), 64), np.uint8)
    b[:, 0::2] = pos[:, :32] & 15
    b[:, 1::2] = pos[:, :32] >> 4
    return (b == 6).sum(1) + (b == 14).sum(1)


def check_game_over(variant, pos, ps, po):
    """Atomic game-over records (one king exploded) are kept and answered with
    (0, 0); crazyhouse never loses a king."""
    k = kings(pos)
    if variant == AT:
        assert np.any(k == 1)
        assert not np.any(ps[k == 1]) and not np.any(po[k == 1])
    else:
        assert np.all(k == 2)


@pytest.mark.parametrize("variant", [ZH, AT])
@pytest.mark.parametrize("hd", [256, 1024])
def test_vgroups_chain_legal_games_match_oracle(vc, variant, hd):
    """CHAIN along legal random games (drops, pockets, explosions): every ply
    equals the from-scratch GPU path and the oracle."""
    ev, on = vc(variant, hd)
    _, pos, off = legal_games(variant, 400, 7 * hd + variant)
    # atomic games that end by an explosion keep their last ply
    gs, go = ev.eval_vgroups(pos, off, N.GROUP_CHAIN)
    check_game_over(variant, pos, gs, go)
    ss, so = ev.eval_vpositions(pos)
    assert np.array_equal(gs, ss) and np.array_equal(go, so)
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert rc == 0 and np.array_equal(gs, ops) and np.array_equal(go, opo)


@pytest.mark.parametrize("variant", [ZH, AT])
def test_vgroups_star_children_match_oracle(vc, variant):
    """STAR: every ply of legal games and all its legal children (drops
    included), children derived from the parent's accumulator."""
    ev, on = vc(variant)
    parts, offs, base = [], [np.zeros(1, np.int64)], 0
    for i in range(12):
        moves = nnue.random_vgame(300 + i, variant, START[variant], 60)
        p, o = nnue.game_vchildren(variant, START[variant], moves)
        parts.append(p)
        offs.append(o[1:].astype(np.int64) + base)
        base += len(p)
    pos, off = np.concatenate(parts), np.concatenate(offs).astype(np.uint32)
    # atomic: every child that captures next to the enemy king is a game-over
    # record inside its STAR group (kept, answered (0, 0))
    gs, go = ev.eval_vgroups(pos, off, N.GROUP_STAR)
    check_game_over(variant, pos, gs, go)
    ss, so = ev.eval_vpositions(pos)
    assert np.array_equal(gs, ss) and np.array_equal(go, so)
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert rc == 0 and np.array_equal(gs, ops) and np.array_equal(go, opo)


@pytest.mark.parametrize("variant", [ZH, AT])
def test_vgroups_random_walks_incremental_equals_refresh(vc, variant):
    """Pseudo-legal random walks (fnnue_random_vpositions PLIES: teleporting
    pieces, many-square changes) as CHAIN and as STAR groups: the deltas or the
    refresh fallback always reproduce the from-scratch results."""
    ev, on = vc(variant)
    pos, off = F.random_vpositions(41, variant, 3000, 120, mode=N.PLAYOUT_PLIES)
    ss, so = ev.eval_vpositions(pos)
    for mode in (N.GROUP_CHAIN, N.GROUP_STAR):
        gs, go = ev.eval_vgroups(pos, off, mode)
        assert np.array_equal(gs, ss) and np.array_equal(go, so), mode
    idx = np.arange(0, len(pos), 7)
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert np.array_equal(ss[idx], ops) and np.array_equal(so[idx], opo)


@pytest.mark.parametrize("variant", [ZH, AT])
@pytest.mark.parametrize("n", [97, 2048, 2049])
def test_vgroups_either_side_of_the_one_workgroup_plan(vc, variant, n):
    """Calls of at most 2048 positions take the one-workgroup segment plan,
    larger ones the kernel chain: both give the from-scratch results (CHAIN
    and STAR over the same legal games, the last game cut short)."""
    ev, on = vc(variant)
    _, pos, off = legal_games(variant, 40, 900 + variant)
    assert len(pos) >= n
    pos = pos[:n]
    off = np.concatenate([off[off < n], [n]]).astype(np.uint32)
    ss, so = ev.eval_vpositions(pos)
    for mode in (N.GROUP_CHAIN, N.GROUP_STAR):
        gs, go = ev.eval_vgroups(pos, off, mode)
        assert np.array_equal(gs, ss) and np.array_equal(go, so), mode
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert rc == 0 and np.array_equal(ss, ops) and np.array_equal(so, opo)


def test_vgroups_device_end_to_end_from_the_device_builder(vc):
    """fnnue_build_vbatch_device -> fnnue_eval_vgroups_device: crazyhouse games
    never leave HBM as positions; every ply against the oracle."""
    import ctypes as C
    import torch
    ev, on = vc(ZH, 1024)
    games, hpos, hoff = legal_games(ZH, 300, 901)
    text, fo, mo = F.pack_games(games)
    dev = torch.device("cuda", 0)
    d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(dev)
    d_fo = torch.from_numpy(fo.view(np.int32)).to(dev)
    d_mo = torch.from_numpy(mo.view(np.int32)).to(dev)
    n, g = len(hpos), len(games)
    d_pos = torch.zeros((n, 48), dtype=torch.uint8, device=dev)
    d_off = torch.zeros(g + 1, dtype=torch.int32, device=dev)
    no, ng = C.c_size_t(), C.c_size_t()
    stream = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    N.check(N.lib.fnnue_build_vbatch_device(ev.handle, ZH, C.c_void_p(d_text.data_ptr()), C.c_void_p(d_fo.data_ptr()),
                                            C.c_void_p(d_mo.data_ptr()), g, N.PLAYOUT_PLIES,
                                            C.c_void_p(d_pos.data_ptr()), n, C.c_void_p(d_off.data_ptr()), g + 1,
                                            C.byref(no), C.byref(ng), C.c_void_p(stream)))
    assert no.value == n and ng.value == g
    ps = torch.zeros(n, dtype=torch.int32, device=dev)
    po = torch.zeros(n, dtype=torch.int32, device=dev)
    ev.eval_vgroups_device(d_pos.data_ptr(), d_off.data_ptr(), g, n, N.GROUP_CHAIN, ps.data_ptr(), po.data_ptr(),
                           stream)
    ev.check()
    assert np.array_equal(d_pos.cpu().numpy(), hpos)
    ops, opo, rc = on.eval_packed(hpos, threads=8)
    assert rc == 0 and np.array_equal(ps.cpu().numpy(), ops) and np.array_equal(po.cpu().numpy(), opo)


def test_vgroups_above_one_workspace_and_errors(vc):
    """> 2^20 crazyhouse positions in CHAIN groups (chunks cut on the device),
    malformed offsets latched as FNNUE_E_ARG, wrong-net entry points refused."""
    import torch
    ev, on = vc(ZH, 256)
    pos, off = F.random_vpositions(77, ZH, 14_000, 160, mode=N.PLAYOUT_PLIES)
    assert len(pos) > (1 << 20)
    gs, go = ev.eval_vgroups(pos, off, N.GROUP_CHAIN)
    ss, so = ev.eval_vpositions(pos)
    assert np.array_equal(gs, ss) and np.array_equal(go, so)
    idx = np.r_[0:3000, (1 << 20) - 3000:(1 << 20) + 3000]
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert np.array_equal(gs[idx], ops) and np.array_equal(go[idx], opo)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(pos[:5000]).to(dev)
    d_off = torch.tensor([0, 3000, 2000, 5000], dtype=torch.int32, device=dev)
    p = torch.zeros(5000, dtype=torch.int32, device=dev)
    ev.eval_vgroups_device(d.data_ptr(), d_off.data_ptr(), 3, 5000, N.GROUP_CHAIN, p.data_ptr(), p.data_ptr(), None)
    with pytest.raises(F.FnnueError) as e:
        ev.check()
    assert e.value.name == "FNNUE_E_ARG"
    with pytest.raises(F.FnnueError) as e:
        ev.eval_groups(np.zeros((1, 36), np.uint8), np.array([0, 1], np.uint32))
    assert e.value.name == "FNNUE_E_ARCH"
    chess = F.Evaluator(F.Net.from_bytes(F.synthesize_net(1, 128)), 0)
    try:
        with pytest.raises(F.FnnueError) as e:
            chess.eval_vgroups(pos[:10], np.array([0, 10], np.uint32))
        assert e.value.name == "FNNUE_E_ARCH"
    finally:
        chess.close()
