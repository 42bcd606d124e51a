"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle,
bit-exact (integer arithmetic: no tolerance).  Run on an MI355X with -m gpu."""
import json
import os

import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from oracle.oracle import OracleNet
from tests.conftest import ROOT, net_bytes
from tests.positions import FENS

pytestmark = pytest.mark.gpu

GAMES = json.load(open(os.path.join(ROOT, "tests", "golden", "wcc_games.json")))["games"]


@pytest.fixture(scope="module")
def ev_cache():
    cache = {}

    def get(seed=1, hd=1024, flags=0):
        key = (seed, hd, flags)
        if key not in cache:
            data = net_bytes(seed, hd, flags)
            cache[key] = (F.Evaluator(F.Net.from_bytes(data), 0), OracleNet(data))
        return cache[key]

    yield get
    for ev, _ in cache.values():
        ev.close()


def assert_same(ev, on, pos):
    ps, po = ev.eval_positions(pos)
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert rc == 0
    bad = np.nonzero((ps != ops) | (po != opo))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}: gpu {ps[bad[:3]]},{po[bad[:3]]} " \
                          f"oracle {ops[bad[:3]]},{opo[bad[:3]]}"


def test_mfma_layout_selftest():
    F.selftest_mfma(0)


def test_fens_big_net(ev_cache):
    ev, on = ev_cache()
    pos = np.stack([F.pos_from_fen(f) for f in FENS])
    assert_same(ev, on, pos)


def test_random_playouts_big_net(ev_cache):
    ev, on = ev_cache()
    assert_same(ev, on, F.random_playouts(1, 20000, threads=8))


# later-SF widths: 1536, 2560, 3072 run the same kernels
WIDE = [(8, 1536, N.SYNTH_LEB128), (9, 2560, 0), (10, 3072, N.SYNTH_WRAP)]


@pytest.mark.parametrize("seed,hd,flags", [(7, 128, 0), (4, 256, N.SYNTH_FC1_PAD), (2, 512, N.SYNTH_LEB128),
                                           (3, 1024, N.SYNTH_WRAP), (6, 2048, 0)] + WIDE)
def test_other_nets(ev_cache, seed, hd, flags):
    ev, on = ev_cache(seed, hd, flags)
    assert_same(ev, on, F.random_playouts(seed + 100, 3000, threads=8))


@pytest.mark.parametrize("impl", [N.FT_SLICED, N.FT_GATHER, N.FT_AUTO])
@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 63, 65, 1000, 2049, 4097, N.FT_GATHER_MAX, N.FT_GATHER_MAX + 1])
def test_ragged_batch_sizes(ev_cache, n, impl):
    """Every size through each feature-transformer choice (FNNUE_FT_AUTO, the
    default, gathers up to FNNUE_FT_GATHER_MAX positions and runs sliced above)."""
    ev, on = ev_cache()
    ev.set_ft_impl(impl)
    try:
        assert_same(ev, on, F.random_playouts(50 + n, n, threads=4))
    finally:
        ev.set_ft_impl(N.FT_AUTO)


@pytest.mark.parametrize("seed,hd,flags", [(1, 1024, 0), (7, 128, 0), (3, 1024, N.SYNTH_WRAP), (6, 2048, 0),
                                           WIDE[2]])
def test_ft_impls_agree(ev_cache, seed, hd, flags):
    """LDS-stationary (sliced) and per-position gather feature transformers."""
    ev, on = ev_cache(seed, hd, flags)
    pos = F.random_playouts(seed + 7, 50000, threads=8)
    a = ev.eval_positions(pos)
    ev.set_ft_impl(N.FT_GATHER)
    b = ev.eval_positions(pos)
    ev.set_ft_impl(N.FT_AUTO)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    idx = np.arange(0, len(pos), 7)
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert np.array_equal(a[0][idx], ops) and np.array_equal(a[1][idx], opo)


def test_chunk_boundary_wide_net(ev_cache):
    """HD = 3072 runs in chunks of 698368 positions (chunk * hd < 2^31, one
    buffer resource): a batch crossing the boundary, positions and CHAIN
    groups, is exact on both sides of it."""
    ev, on = ev_cache(*WIDE[2])
    chunk = min(1 << 20, (0x7FFFFFFF // 3072) & ~1023)
    pos = F.random_playouts(31, chunk + 3000, threads=8)
    ps, po = ev.eval_positions(pos)
    idx = np.r_[0:2000, chunk - 2000:chunk + 3000]
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert np.array_equal(ps[idx], ops) and np.array_equal(po[idx], opo)
    gpos, off = F.random_playouts(32, 9000, mode=N.PLAYOUT_PLIES, threads=8)
    assert off[-1] > chunk
    gs, go = ev.eval_groups(gpos, off, N.GROUP_CHAIN)
    # chunks are cut at fixed positions: the game straddling position `chunk`
    # restarts with a refresh there
    idx = np.r_[0:2000, chunk - 2000:chunk + 2000, len(gpos) - 2000:len(gpos)]
    ops, opo, rc = on.eval_packed(gpos[idx], threads=8)
    assert np.array_equal(gs[idx], ops) and np.array_equal(go[idx], opo)


def test_gather_groups_across_chunks(ev_cache):
    """The per-group gather kernel walks only the groups overlapping its
    chunk (a binary search over the offsets): CHAIN groups across the HD-3072
    chunk boundary, with empty groups mixed in (repeated offsets), equal the
    segment path everywhere and the oracle around the boundary."""
    ev, on = ev_cache(*WIDE[2])
    chunk = min(1 << 20, (0x7FFFFFFF // 3072) & ~1023)
    gpos, off = F.random_playouts(33, 9000, mode=N.PLAYOUT_PLIES, threads=8)
    assert off[-1] > chunk
    off = np.sort(np.concatenate([off, off[::97], off[::1000]])).astype(np.uint32)
    res = []
    for impl in (N.FT_SLICED, N.FT_GATHER):
        ev.set_ft_impl(impl)
        res.append(ev.eval_groups(gpos, off, N.GROUP_CHAIN))
    ev.set_ft_impl(N.FT_AUTO)
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    idx = np.r_[0:1000, chunk - 2000:chunk + 2000, len(gpos) - 1000:len(gpos)]
    ops, opo, rc = on.eval_packed(gpos[idx], threads=8)
    assert np.array_equal(res[1][0][idx], ops) and np.array_equal(res[1][1][idx], opo)


def test_same_king_block_everywhere(ev_cache):
    """Degenerate plan: every item in one king block / one n bin (one huge bin,
    many units for a single tile)."""
    ev, on = ev_cache()
    start = F.pos_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1")
    pos = np.repeat(start[None, :], 10000, axis=0)
    assert_same(ev, on, pos)


def test_empty_batch(ev_cache):
    ev, _ = ev_cache()
    ps, po = ev.eval_positions(np.zeros((0, 36), dtype=np.uint8))
    assert len(ps) == 0 and len(po) == 0


def test_invalid_position_fails_whole_batch(ev_cache):
    ev, _ = ev_cache()
    pos = F.random_playouts(5, 10, threads=2)
    pos[3, :32] = 0  # no kings
    with pytest.raises(F.FnnueError) as e:
        ev.eval_positions(pos)
    assert e.value.name == "FNNUE_E_POSITION"
    assert "index 3" in str(e.value)  # latched on the device, named by the host
    pos = F.random_playouts(5, 10, threads=2)
    pos[4, 0] = (pos[4, 0] & 0xF0) | 7  # invalid piece code 7 on a1
    with pytest.raises(F.FnnueError) as e:
        ev.eval_positions(pos)
    assert e.value.name == "FNNUE_E_POSITION"
    # the ctx stays usable after the failed batch
    ev2, on = ev_cache()
    assert_same(ev2, on, F.random_playouts(6, 10, threads=2))


def test_device_latched_invalid_position(ev_cache):
    """Device-pointer path: validity is checked on the GPU and latched."""
    import torch
    ev, _ = ev_cache()
    pos = F.random_playouts(5, 64, threads=2)
    pos[10, 32] = 2  # stm out of range
    d = torch.from_numpy(pos).cuda()
    ps = torch.zeros(64, dtype=torch.int32, device="cuda")
    po = torch.zeros(64, dtype=torch.int32, device="cuda")
    ev.eval_positions_device(d.data_ptr(), 64, ps.data_ptr(), po.data_ptr(), torch.cuda.current_stream().cuda_stream)
    with pytest.raises(F.FnnueError) as e:
        ev.check()
    assert e.value.name == "FNNUE_E_POSITION"
    ev.check()  # cleared


def test_games_chain_incremental(ev_cache):
    """CHAIN groups (incremental add/sub along each game) == oracle from scratch."""
    ev, on = ev_cache()
    pos = [F.game_positions(g["position"], g["moves"]) for g in GAMES]
    off = np.concatenate([[0], np.cumsum([len(p) for p in pos])]).astype(np.uint32)
    allpos = np.concatenate(pos)
    ps, po = ev.eval_groups(allpos, off, N.GROUP_CHAIN)
    ops, opo, rc = on.eval_packed(allpos, threads=8)
    assert rc == 0
    assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_random_games_chain_and_small_net(ev_cache):
    for seed, hd in ((1, 1024), (7, 128)):
        ev, on = ev_cache(seed, hd, 0)
        pos, off = F.random_playouts(2, 300, mode=N.PLAYOUT_PLIES, threads=8)
        ps, po = ev.eval_groups(pos, off, N.GROUP_CHAIN)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert np.array_equal(ps, ops) and np.array_equal(po, opo)


@pytest.mark.parametrize("big,small", [(1024, 128), (2048, 256), (1536, 128)])
def test_dual_groups_big_and_small_net(ev_cache, big, small):
    """fnnue_eval_groups_dual_device (BASELINE config 3's big + small net over
    one plan, the small net on the small context's stream): identical to two
    separate grouped calls and to the oracle, CHAIN and STAR, and across a
    chunk boundary (> 2^20 positions)."""
    eb, ob = ev_cache(1, big, 0)
    es, os_ = ev_cache(7, small, 0)
    pos, off = F.random_playouts(2, 300, mode=N.PLAYOUT_PLIES, threads=8)
    kids = [F.game_children(g["position"], g["moves"]) for g in GAMES[:4]]
    cpos = np.concatenate([k[0] for k in kids])
    coff = np.concatenate([[0]] + [k[1][1:] + sum(len(x[0]) for x in kids[:i]) for i, k in enumerate(kids)])
    for p, o, mode in ((pos, off, N.GROUP_CHAIN), (cpos, coff.astype(np.uint32), N.GROUP_STAR)):
        ps, po, ps2, po2 = eb.eval_groups_dual(es, p, o, mode)
        a, b = eb.eval_groups(p, o, mode)
        c, d = es.eval_groups(p, o, mode)
        assert np.array_equal(ps, a) and np.array_equal(po, b), mode
        assert np.array_equal(ps2, c) and np.array_equal(po2, d), mode
        for on, x, y in ((ob, ps, po), (os_, ps2, po2)):
            ops, opo, rc = on.eval_packed(p, threads=8)
            assert rc == 0 and np.array_equal(x, ops) and np.array_equal(y, opo), mode
    if big == 1024:
        pos, off = F.random_playouts(11, 14_000, max_plies=160, mode=N.PLAYOUT_PLIES, threads=16)
        assert len(pos) > (1 << 20)
        ps, po, ps2, po2 = eb.eval_groups_dual(es, pos, off, N.GROUP_CHAIN)
        a, b = eb.eval_groups(pos, off, N.GROUP_CHAIN)
        c, d = es.eval_groups(pos, off, N.GROUP_CHAIN)
        assert np.array_equal(ps, a) and np.array_equal(po, b) and np.array_equal(ps2, c) and np.array_equal(po2, d)
        idx = np.r_[0:2000, (1 << 20) - 2000:(1 << 20) + 2000]
        ops, opo, rc = os_.eval_packed(pos[idx], threads=8)
        assert np.array_equal(ps2[idx], ops) and np.array_equal(po2[idx], opo)


def test_dual_groups_rejects_mismatched_contexts(ev_cache):
    eb, _ = ev_cache(1, 1024, 0)
    pos, off = F.random_playouts(2, 10, mode=N.PLAYOUT_PLIES, threads=2)
    with pytest.raises(F.FnnueError) as e:
        eb.eval_groups_dual(eb, pos, off)
    assert e.value.name == "FNNUE_E_ARG"
    zh = F.Evaluator(F.Net.from_bytes_variant(F.synthesize_variant_net(5, 256, N.VARIANT_CRAZYHOUSE),
                                              N.VARIANT_CRAZYHOUSE), 0)
    try:
        with pytest.raises(F.FnnueError) as e:
            eb.eval_groups_dual(zh, pos, off)
        assert e.value.name == "FNNUE_E_ARCH"
    finally:
        zh.close()


def test_children_star(ev_cache):
    ev, on = ev_cache()
    for g in GAMES[:3]:
        pos, off = F.game_children(g["position"], g["moves"])
        ps, po = ev.eval_groups(pos, off, N.GROUP_STAR)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_wrap_net_chain(ev_cache):
    """int16 wraparound: incremental (mod 2^16) must still equal refresh."""
    ev, on = ev_cache(3, 1024, N.SYNTH_WRAP)
    pos, off = F.random_playouts(8, 100, mode=N.PLAYOUT_PLIES, threads=8)
    ps, po = ev.eval_groups(pos, off, N.GROUP_CHAIN)
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_full_size_properties(ev_cache):
    """BASELINE config 2 size (1M positions): scratch == CHAIN-of-singletons
    == STAR re-evaluation, plus a sampled oracle check."""
    ev, on = ev_cache()
    pos = F.random_playouts(1, 1_000_000, threads=16)
    ps, po = ev.eval_positions(pos)
    idx = np.random.default_rng(0).choice(len(pos), 20000, replace=False)
    ops, opo, rc = on.eval_packed(pos[idx], threads=16)
    assert np.array_equal(ps[idx], ops) and np.array_equal(po[idx], opo)
    # groups of 2 in STAR mode: second = first re-derived incrementally
    pairs = np.repeat(pos[:200_000], 2, axis=0)
    off = np.arange(0, len(pairs) + 1, 2, dtype=np.uint32)
    ps2, po2 = ev.eval_groups(pairs, off, N.GROUP_STAR)
    assert np.array_equal(ps2[1::2], ps[:200_000]) and np.array_equal(po2[1::2], po[:200_000])


def test_groups_longer_than_a_span_chunk(ev_cache):
    """Groups longer than the 4096-position span chunk (one CHAIN over a whole
    random game corpus, a single group holding every position of the call,
    mixed with small and empty groups) give the from-scratch
    results: grouping never changes a result, and the span table of a long
    group is filled by one workgroup per chunk."""
    ev, on = ev_cache()
    pos, off = F.random_playouts(21, 4000, mode=N.PLAYOUT_PLIES, threads=8)
    ps, po = ev.eval_positions(pos)
    n = len(pos)
    cuts = [0, 4095, 4095, 4096 * 3 + 17, 4096 * 3 + 18, 4096 * 5, 4096 * 5 + 4097, n - 3, n]
    for o in (np.array([0, n], np.uint32), np.array(cuts, np.uint32)):
        for mode in (N.GROUP_CHAIN, N.GROUP_STAR):
            gs, go = ev.eval_groups(pos, o, mode)
            assert np.array_equal(gs, ps) and np.array_equal(go, po), (len(o), mode)
    idx = np.arange(0, n, 97)
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert np.array_equal(ps[idx], ops) and np.array_equal(po[idx], opo)


def test_image_broadcast_path(ev_cache):
    """ctx from a device image (what bench.py broadcasts over RCCL) == ctx from the net."""
    import torch
    ev, _ = ev_cache()
    img = F.Net.from_bytes(net_bytes(1, 1024, 0)).image()
    buf = torch.from_numpy(img).cuda()
    ev2 = F.Evaluator(None, 0, image_ptr=buf.data_ptr(), image_bytes=img.size, hd=1024)
    pos = F.random_playouts(12, 500, threads=4)
    a, b = ev.eval_positions(pos), ev2.eval_positions(pos)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    ev2.close()


@pytest.mark.parametrize("seed,hd,flags", [(1, 1024, 0), (7, 128, 0), (6, 2048, 0), (3, 1024, N.SYNTH_WRAP)] + WIDE)
def test_group_impls_agree(ev_cache, seed, hd, flags):
    """Incremental groups: LDS-tile segments (sliced, default) == per-group
    gather kernel == oracle, for CHAIN games and STAR children."""
    ev, on = ev_cache(seed, hd, flags)
    for mode, pm, count in ((N.GROUP_CHAIN, N.PLAYOUT_PLIES, 400), (N.GROUP_STAR, N.PLAYOUT_CHILDREN, 40)):
        pos, off = F.random_playouts(seed + 20, count, mode=pm, threads=8)
        res = []
        for impl in (N.FT_SLICED, N.FT_GATHER):
            ev.set_ft_impl(impl)
            res.append(ev.eval_groups(pos, off, mode))
        ev.set_ft_impl(N.FT_AUTO)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        for ps, po in res:
            assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_groups_of_unrelated_positions(ev_cache):
    """Groups need not be games: big diffs and king jumps refresh."""
    ev, on = ev_cache()
    pos = F.random_playouts(5, 3000, threads=8)
    off = np.array([0, 1, 7, 500, 501, 2999, 3000], dtype=np.uint32)
    for mode in (N.GROUP_CHAIN, N.GROUP_STAR):
        ps, po = ev.eval_groups(pos, off, mode)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert np.array_equal(ps, ops) and np.array_equal(po, opo)


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 511, 513, 1025, 2047, 2048, 2049, 4097, 8193])
def test_groups_ragged_sizes(ev_cache, n):
    """Batch sizes around the segment plan's 256-position scan blocks (refresh
    counts per block, block scan, local scans) and either side of the
    one-workgroup plan's limit (2048 positions): CHAIN plies and STAR
    children, the last group cut short."""
    ev, on = ev_cache()
    for mode, pm, count in ((N.GROUP_CHAIN, N.PLAYOUT_PLIES, 130), (N.GROUP_STAR, N.PLAYOUT_CHILDREN, 4)):
        pos, off = F.random_playouts(31, count, mode=pm, threads=8)
        assert len(pos) >= n
        pos = pos[:n]
        off = np.concatenate([off[off < n], [n]]).astype(np.uint32)
        ps, po = ev.eval_groups(pos, off, mode)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert rc == 0
        assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_groups_with_invalid_position(ev_cache):
    """An invalid position fails the batch (host API) and never feeds a delta."""
    ev, on = ev_cache()
    pos, off = F.random_playouts(9, 30, mode=N.PLAYOUT_PLIES, threads=8)
    bad = pos.copy()
    bad[off[3] + 2, :32] = 0  # no kings
    with pytest.raises(F.FnnueError) as e:
        ev.eval_groups(bad, off, N.GROUP_CHAIN)
    assert e.value.name == "FNNUE_E_POSITION"
    ps, po = ev.eval_groups(pos, off, N.GROUP_CHAIN)  # ctx still usable
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_groups_device_latched_invalid(ev_cache):
    """Device entry point: invalid positions inside CHAIN/STAR groups give 0/0,
    the rest stay exact (refresh after the hole), error latched."""
    import torch
    ev, on = ev_cache()
    for mode, pm in ((N.GROUP_CHAIN, N.PLAYOUT_PLIES), (N.GROUP_STAR, N.PLAYOUT_CHILDREN)):
        pos, off = F.random_playouts(10, 20, mode=pm, threads=8)
        holes = [int(off[2]) + 1, int(off[5]), int(off[7]) + 3]
        bad = pos.copy()
        for h in holes:
            bad[h, :32] = 0
        dev = torch.device("cuda", 0)
        d_pos = torch.from_numpy(bad).to(dev)
        d_off = torch.from_numpy(off.astype(np.int32)).to(dev)
        d_ps = torch.full((len(pos),), 77, dtype=torch.int32, device=dev)
        d_po = torch.full((len(pos),), 77, dtype=torch.int32, device=dev)
        ev.eval_groups_device(d_pos.data_ptr(), d_off.data_ptr(), len(off) - 1, len(pos), mode, d_ps.data_ptr(),
                              d_po.data_ptr(), None)
        with pytest.raises(F.FnnueError):
            ev.check()
        ps, po = d_ps.cpu().numpy(), d_po.cpu().numpy()
        ops, opo, rc = on.eval_packed(pos, threads=8)
        ok = np.ones(len(pos), dtype=bool)
        ok[holes] = False
        assert np.all(ps[~ok] == 0) and np.all(po[~ok] == 0)
        assert np.array_equal(ps[ok], ops[ok]) and np.array_equal(po[ok], opo[ok])


def test_device_groups_offsets_checked_on_device(ev_cache):
    """fnnue_eval_groups_device never reads the offsets on the host (any size):
    malformed offsets latch FNNUE_E_ARG, stay in bounds, and the ctx stays usable;
    arbitrary (valid) groupings give the oracle's results."""
    import torch
    ev, on = ev_cache()
    pos, off = F.random_playouts(31, 40, mode=F.PLAYOUT_PLIES, threads=2)
    n = len(pos)
    d = torch.from_numpy(pos).cuda()
    ps = torch.zeros(n, dtype=torch.int32, device="cuda")
    po = torch.zeros(n, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for bad in ([0, 50, 20, n], [0, 10, n - 1], [5, 10, n], [0, n + 7]):
        d_off = torch.tensor(bad, dtype=torch.int32, device="cuda")
        for mode in (F.GROUP_CHAIN, F.GROUP_STAR):
            ev.eval_groups_device(d.data_ptr(), d_off.data_ptr(), len(bad) - 1, n, mode, ps.data_ptr(),
                                  po.data_ptr(), stream)
            with pytest.raises(F.FnnueError) as e:
                ev.check()
            assert e.value.name == "FNNUE_E_ARG"
    ops, opo, rc = on.eval_packed(pos, threads=4)
    assert rc == 0
    # valid but arbitrary groupings: STAR "children" that are other plies, CHAIN cut mid-game
    rng = np.random.default_rng(3)
    cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n, 57)])).astype(np.uint32)
    for mode in (F.GROUP_CHAIN, F.GROUP_STAR):
        d_off = torch.from_numpy(cuts.view(np.int32)).cuda()
        ev.eval_groups_device(d.data_ptr(), d_off.data_ptr(), len(cuts) - 1, n, mode, ps.data_ptr(), po.data_ptr(),
                              stream)
        ev.check()
        assert np.array_equal(ps.cpu().numpy(), ops) and np.array_equal(po.cpu().numpy(), opo)


def test_segments_units_split_inside_king_block(ev_cache):
    """Many segments in ONE king block (the kings' start squares): far more than
    2 x kSegUnitPlies (20480) plies of work there, so plan_scan cuts the king
    block's length bins into several units mid-bin (sliced_common.h
    build_units).  CHAIN over 5000 random games and STAR over the children of
    150 games, both against the oracle."""
    ev, on = ev_cache()
    for mode, pm, count in ((N.GROUP_CHAIN, N.PLAYOUT_PLIES, 5000), (N.GROUP_STAR, N.PLAYOUT_CHILDREN, 150)):
        pos, off = F.random_playouts(77, count, mode=pm, threads=8)
        board = np.zeros((len(pos), 64), np.uint8)
        board[:, 0::2] = pos[:, :32] & 15
        board[:, 1::2] = pos[:, :32] >> 4
        assert int((board[:, 4] == 6).sum()) > 2 * 20480  # white king on e1: one king block
        ps, po = ev.eval_groups(pos, off, mode)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert rc == 0
        assert np.array_equal(ps, ops) and np.array_equal(po, opo)


def test_eval_groups_rejects_bad_offsets(ev_cache):
    """Host API: offsets must end at the number of positions given (no read past
    the input) and there must be at least one offset."""
    ev, _ = ev_cache()
    pos, off = F.random_playouts(3, 5, mode=N.PLAYOUT_PLIES, threads=2)
    bad = off.copy()
    bad[-1] += 1
    with pytest.raises(ValueError):
        ev.eval_groups(pos, bad, N.GROUP_CHAIN)
    with pytest.raises(ValueError):
        ev.eval_groups(pos, np.zeros(0, np.uint32), N.GROUP_CHAIN)
    import ctypes as C
    ps = np.zeros(len(pos), np.int32)
    po = np.zeros(len(pos), np.int32)
    rc = N.lib.fnnue_eval_groups(ev.handle, N.ptr(pos), len(pos) - 1, N.ptr(off), len(off) - 1, N.GROUP_CHAIN,
                                 N.ptr(ps), N.ptr(po))
    assert rc == -1 and b"npos" in N.lib.fnnue_last_error()


def test_device_calls_on_two_streams(ev_cache):
    """Two *_device calls on different streams with no sync in between: the
    library orders the shared workspace, both results exact."""
    import torch
    ev, on = ev_cache()
    a = F.random_playouts(41, 200_000, threads=8)
    b = F.random_playouts(42, 200_000, threads=8)
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    out = [torch.zeros(len(a), dtype=torch.int32, device=dev) for _ in range(4)]
    torch.cuda.synchronize()
    ev.eval_positions_device(da.data_ptr(), len(a), out[0].data_ptr(), out[1].data_ptr(), s1.cuda_stream)
    ev.eval_positions_device(db.data_ptr(), len(b), out[2].data_ptr(), out[3].data_ptr(), s2.cuda_stream)
    torch.cuda.synchronize()
    ev.check()
    for pos, ps, po in ((a, out[0], out[1]), (b, out[2], out[3])):
        idx = np.arange(0, len(pos), 13)
        ops, opo, rc = on.eval_packed(pos[idx], threads=8)
        assert np.array_equal(ps.cpu().numpy()[idx], ops) and np.array_equal(po.cpu().numpy()[idx], opo)


def test_device_calls_own_stream_then_other_stream(ev_cache):
    """Calls on the context's own stream record no workspace event; a following
    call on another stream (no sync in between) records it on the own stream
    first and waits for it, and a call on the own stream after that waits for
    the other stream's event: own -> other -> own -> own, all results exact."""
    import torch
    ev, on = ev_cache()
    batches = [F.random_playouts(51 + k, 150_000, threads=8) for k in range(4)]
    dev = torch.device("cuda", 0)
    s2 = torch.cuda.Stream(dev)
    ds = [torch.from_numpy(b).to(dev) for b in batches]
    outs = [torch.zeros(len(b), dtype=torch.int32, device=dev) for b in batches for _ in range(2)]
    torch.cuda.synchronize()
    for k, stream in enumerate((None, s2.cuda_stream, None, None)):
        ev.eval_positions_device(ds[k].data_ptr(), len(batches[k]), outs[2 * k].data_ptr(), outs[2 * k + 1].data_ptr(),
                                 stream)
    ev.check()
    torch.cuda.synchronize()
    for k, pos in enumerate(batches):
        idx = np.arange(k, len(pos), 11)
        ops, opo, rc = on.eval_packed(pos[idx], threads=8)
        assert rc == 0
        assert np.array_equal(outs[2 * k].cpu().numpy()[idx], ops)
        assert np.array_equal(outs[2 * k + 1].cpu().numpy()[idx], opo)


def test_device_call_after_its_stream_was_destroyed(ev_cache):
    """A *_device call on a temporary stream, the stream destroyed right after,
    then calls on the context's own stream and on another stream: the library
    never touches the destroyed stream again (the workspace event is recorded
    on each call's own stream), results exact."""
    import torch
    ev, on = ev_cache()
    pos = F.random_playouts(43, 50_000, threads=8)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(pos).to(dev)
    outs = [torch.zeros(len(pos), dtype=torch.int32, device=dev) for _ in range(6)]
    torch.cuda.synchronize()
    tmp = torch.cuda.Stream(dev)
    ev.eval_positions_device(d.data_ptr(), len(pos), outs[0].data_ptr(), outs[1].data_ptr(), tmp.cuda_stream)
    tmp.synchronize()
    del tmp  # torch destroys the stream (or returns it to its pool)
    ev.eval_positions_device(d.data_ptr(), len(pos), outs[2].data_ptr(), outs[3].data_ptr(), None)
    ev.check()
    s2 = torch.cuda.Stream(dev)
    ev.eval_positions_device(d.data_ptr(), len(pos), outs[4].data_ptr(), outs[5].data_ptr(), s2.cuda_stream)
    ev.check()  # waits for the last call's stream too, without draining the device
    idx = np.arange(0, len(pos), 7)
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert rc == 0
    for k in (0, 2, 4):
        assert np.array_equal(outs[k].cpu().numpy()[idx], ops) and np.array_equal(outs[k + 1].cpu().numpy()[idx], opo)


def test_device_groups_above_one_workspace(ev_cache):
    """A grouped *_device call above one workspace (> 2^20 positions): cut into
    chunks at fixed positions on the device, the offsets never read on the
    host.  STAR (every ply + children of 560 games, ~1.4M) and CHAIN (every
    ply of 20k games, ~1.6M) against the oracle, for both FT
    implementations; groups cut by a chunk boundary included; malformed
    offsets still latch FNNUE_E_ARG at this size."""
    import torch
    ev, on = ev_cache()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    for mode, pm, count, seed in ((N.GROUP_STAR, N.PLAYOUT_CHILDREN, 560, 51), (N.GROUP_CHAIN, N.PLAYOUT_PLIES, 20_000, 52)):
        pos, off = F.random_playouts(seed, count, mode=pm, threads=8)
        n = len(pos)
        assert n > (1 << 20)
        # a group straddles the first chunk boundary
        g = int(np.searchsorted(off, 1 << 20, side="right")) - 1
        assert off[g] < (1 << 20) < off[g + 1]
        d = torch.from_numpy(pos).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert rc == 0
        for impl in (N.FT_SLICED, N.FT_GATHER):
            ev.set_ft_impl(impl)
            try:
                ps = torch.full((n,), 7, dtype=torch.int32, device=dev)
                po = torch.full((n,), 7, dtype=torch.int32, device=dev)
                ev.eval_groups_device(d.data_ptr(), d_off.data_ptr(), len(off) - 1, n, mode, ps.data_ptr(),
                                      po.data_ptr(), stream)
                ev.check()
                assert np.array_equal(ps.cpu().numpy(), ops) and np.array_equal(po.cpu().numpy(), opo), (mode, impl)
                bad = off.copy()
                bad[len(bad) // 2] = bad[len(bad) // 2 + 1] + 1  # not non-decreasing, past the first chunk
                d_bad = torch.from_numpy(bad.view(np.int32)).to(dev)
                ev.eval_groups_device(d.data_ptr(), d_bad.data_ptr(), len(bad) - 1, n, mode, ps.data_ptr(),
                                      po.data_ptr(), stream)
                with pytest.raises(F.FnnueError) as e:
                    ev.check()
                assert e.value.name == "FNNUE_E_ARG"
            finally:
                ev.set_ft_impl(N.FT_AUTO)


@pytest.mark.parametrize("seed,hd,flags", [(1, 1024, 0), (7, 128, 0), (6, 2048, 0), (8, 1536, N.SYNTH_LEB128)])
def test_swar_rows_match_packed_rows(ev_cache, seed, hd, flags):
    """ft_slices with SWAR row sums (32-bit words, enabled from the accumulator
    bound) == packed int16 row sums == oracle; a net whose bound forbids SWAR
    refuses it."""
    ev, on = ev_cache(seed, hd, flags)
    on_swar, bound = ev.swar()
    assert on_swar and bound < 32768
    pos = F.random_playouts(seed + 60, 40000, threads=8)
    a = ev.eval_positions(pos)
    ev.set_swar(False)
    try:
        b = ev.eval_positions(pos)
    finally:
        ev.set_swar(True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    idx = np.arange(0, len(pos), 5)
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert np.array_equal(a[0][idx], ops) and np.array_equal(a[1][idx], opo)
    evw, _ = ev_cache(3, 1024, N.SYNTH_WRAP)
    assert evw.swar()[0] is False
    with pytest.raises(F.FnnueError) as e:
        evw.set_swar(True)
    assert e.value.name == "FNNUE_E_ARCH"


def edge_net(seed: int, hd: int, mag: tuple[int, int]) -> bytes:
    """A synthetic net whose FT columns each keep one sign over every row with
    |w| in [mag[0], mag[1]] and a zero bias: full-board accumulators reach
    31-32 times mag, close to the doubled-column SWAR limit (2^14).  The first
    half's odd columns stay small (|w| <= 12) so that half the transform pairs
    do not saturate and the evaluation still depends on the position."""
    data = bytearray(net_bytes(seed, hd, 0))
    desc_len = int(np.frombuffer(data, np.uint32, 1, 8)[0])
    o = 12 + desc_len + 4
    rng = np.random.default_rng(seed)
    sign = np.where(rng.random(hd) < 0.5, -1, 1)
    w = rng.integers(mag[0], mag[1] + 1, size=(22528, hd)) * sign
    small = np.arange(hd)[1:hd // 2:2]
    w[:, small] = rng.integers(-12, 13, size=(22528, small.size))
    data[o:o + 2 * hd] = bytes(2 * hd)
    data[o + 2 * hd:o + 2 * hd + 2 * 22528 * hd] = w.astype(np.int16).tobytes()
    return bytes(data)


def test_swar_exact_at_the_doubled_column_limit():
    """Second-half columns are summed doubled: a net whose
    accumulators come within ~15 % of 2^14 still runs SWAR rows and stays
    bit-exact against packed rows and the oracle (a wrap would turn a
    saturated 127 into 0); a net just past the limit falls back to packed
    rows."""
    data = edge_net(21, 256, (400, 500))
    net = F.Net.from_bytes(data)
    assert 31 * 400 * 2 < net.accumulator_bound() < 32768
    ev, on = F.Evaluator(net, 0), OracleNet(data)
    try:
        assert ev.swar()[0]
        pos = F.random_playouts(21, 20000, 0, 40, threads=8)  # early plies: 28-32 pieces
        a = ev.eval_positions(pos)
        ev.set_swar(False)
        b = ev.eval_positions(pos)
        ev.set_swar(True)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert rc == 0 and np.array_equal(a[0], ops) and np.array_equal(a[1], opo)
        gpos, off = F.random_playouts(22, 200, 0, 60, mode=N.PLAYOUT_PLIES, threads=8)
        gs, go = ev.eval_groups(gpos, off, N.GROUP_CHAIN)
        ops, opo, rc = on.eval_packed(gpos, threads=8)
        assert rc == 0 and np.array_equal(gs, ops) and np.array_equal(go, opo)
    finally:
        ev.close()
    over = F.Net.from_bytes(edge_net(21, 256, (520, 540)))
    assert over.accumulator_bound() >= 32768
    evo = F.Evaluator(over, 0)
    try:
        assert evo.swar()[0] is False
    finally:
        evo.close()


@pytest.mark.skipif(not os.environ.get("FNNUE_NET"), reason="set FNNUE_NET=<path to a real .nnue> to run")
def test_real_net_file_matches_oracle():
    """Opt-in: a real Stockfish net (e.g. nn-ad9b42354671.nnue, [ref] build.rs:7)
    if one is ever placed on the box.  Loading checks its identity (SHA-256
    prefix = name) and the structure-hash chain; then GPU == oracle over 200k
    config-2 random-playout positions (from scratch) and 2,000 games' plies
    (incremental CHAIN).  A match of both loaders on a real file pins the
    recalled architecture constants."""
    path = os.environ["FNNUE_NET"]
    data = open(path, "rb").read()
    net = F.Net.load(path)
    ev = F.Evaluator(net, 0)
    on = OracleNet(data)
    try:
        pos = F.random_playouts(1, 200_000, 0, 160, threads=8)
        ps, po = ev.eval_positions(pos)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert rc == 0 and np.array_equal(ps, ops) and np.array_equal(po, opo)
        gpos, off = F.random_playouts(2, 2000, 0, 160, mode=N.PLAYOUT_PLIES, threads=8)
        gs, go = ev.eval_groups(gpos, off, N.GROUP_CHAIN)
        ops, opo, rc = on.eval_packed(gpos, threads=8)
        assert rc == 0 and np.array_equal(gs, ops) and np.array_equal(go, opo)
        print(json.dumps({"real_net": os.path.basename(path), "sha256": net.sha256(), "hd": net.info()[0],
                          "positions": len(pos), "plies": len(gpos), "mismatches": 0}))
    finally:
        ev.close()


def test_timing_modes(ev_cache):
    """fnnue_ctx_set_timing: FNNUE_TIMING_ALL times plan / FT kernel / stacks of
    every chunk; FNNUE_TIMING_FT records only the two events around the FT
    kernel (plan and stack read 0); off records nothing.  Results unchanged."""
    import torch
    ev, on = ev_cache()
    pos = F.random_playouts(61, 100_000, threads=8)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(pos).to(dev)
    ps, po = (torch.zeros(len(pos), dtype=torch.int32, device=dev) for _ in range(2))
    torch.cuda.synchronize()
    for mode in ("all", "ft", "off"):
        ev.set_timing(mode != "off", ft_only=mode == "ft")
        for _ in range(3):
            ev.eval_positions_device(d.data_ptr(), len(pos), ps.data_ptr(), po.data_ptr(), None)
        ev.check()
        n, plan, ft, stack = ev.timing_phases()
        if mode == "off":
            assert n == 0 and plan == ft == stack == 0
        else:
            assert n == 3 and ft > 0
            assert (plan > 0 and stack > 0) if mode == "all" else (plan == 0 and stack == 0)
    ev.set_timing(False)
    idx = np.arange(0, len(pos), 17)
    ops, opo, rc = on.eval_packed(pos[idx], threads=8)
    assert rc == 0 and np.array_equal(ps.cpu().numpy()[idx], ops) and np.array_equal(po.cpu().numpy()[idx], opo)
