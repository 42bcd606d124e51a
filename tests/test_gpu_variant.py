"""GPU parity of the Fairy-Stockfish variant path (BASELINE config 5) against
the CPU restatement oracle/variant_oracle.c, bit-exact.  PARITY UNPINNED
against Fairy-Stockfish itself (see tests/test_variant.py)."""
import numpy as np
import pytest

import fishnet_amd as F
from fishnet_amd import _native as N
from oracle.oracle import VariantOracleNet

pytestmark = pytest.mark.gpu

CZH, ATOMIC = F.VARIANT_CRAZYHOUSE, F.VARIANT_ATOMIC


@pytest.fixture(scope="module")
def vcache():
    cache = {}

    def get(variant, hd=512, seed=3, flags=0):
        key = (variant, hd, seed, flags)
        if key not in cache:
            data = F.synthesize_variant_net(seed, hd, variant, flags)
            cache[key] = (F.Evaluator(F.Net.from_bytes_variant(data, variant), 0), VariantOracleNet(data, variant))
        return cache[key]

    yield get
    for ev, _ in cache.values():
        ev.close()


def same(ev, on, pos):
    ps, po = ev.eval_vpositions(pos)
    ops, opo, rc = on.eval_packed(pos, threads=8)
    assert rc == 0
    bad = np.nonzero((ps != ops) | (po != opo))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("variant", [CZH, ATOMIC])
@pytest.mark.parametrize("hd", [256, 512, 1024])
def test_variant_positions_match_oracle(vcache, variant, hd):
    ev, on = vcache(variant, hd)
    same(ev, on, F.random_vpositions(11 + hd, variant, 30000, 160))


@pytest.mark.parametrize("variant", [CZH, ATOMIC])
def test_variant_swar_and_packed_rows_agree(vcache, variant):
    ev, on = vcache(variant)
    assert ev.swar()[0]
    pos = F.random_vpositions(21, variant, 20000, 160)
    a = ev.eval_vpositions(pos)
    ev.set_swar(False)
    try:
        b = ev.eval_vpositions(pos)
    finally:
        ev.set_swar(True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_variant_fen_positions_and_ragged_sizes(vcache):
    ev, on = vcache(CZH)
    fens = ["rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1",
            "r1bqkb1r/ppp2ppp/2n2n2/4p3/4P3/5N2/PPP2PPP/RNBQKB1R[Pp] w KQkq - 0 1",
            "r1bqkb1r/ppp2ppp/2n2n2/4p3/4P3/5N2/PPP2PPP/RNBQ~KB1R[QQ] b - - 0 1",
            "4k3/8/8/8/8/8/8/4K3[QQRRBBNNPPPPPPPqqrrbbnnppppppp] w - - 0 1"]  # 30 pieces in hand
    same(ev, on, np.stack([F.vpos_from_fen(CZH, f) for f in fens]))
    for n in (1, 17, 1000, 4097):
        same(ev, on, F.random_vpositions(40 + n, CZH, n, 160))


def test_variant_invalid_position_and_wrong_entry_point(vcache):
    ev, _ = vcache(CZH)
    pos = F.random_vpositions(5, CZH, 10, 50)
    pos[4, 33] = 17  # 17 pawns in hand
    with pytest.raises(F.FnnueError) as e:
        ev.eval_vpositions(pos)
    assert e.value.name == "FNNUE_E_POSITION"
    eva, _ = vcache(ATOMIC)
    pos = F.random_vpositions(6, ATOMIC, 10, 50)
    pos[2, 35] = 1  # a knight in hand: atomic has no pockets
    with pytest.raises(F.FnnueError):
        eva.eval_vpositions(pos)
    with pytest.raises(F.FnnueError) as e:  # chess entry point on a variant context
        ev.eval_positions(F.random_playouts(1, 4, threads=2))
    assert e.value.name == "FNNUE_E_ARCH"


def test_atomic_game_over_records(vcache):
    """An atomic position with one king exploded is the game's end, not an
    error: (0, 0) on both entry points and in groups, the rest evaluated as
    usual; a position with no king at all still fails, naming its index
    (ADVICE r03)."""
    ev, on = vcache(ATOMIC)
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    moves = "g1f3 e7e6 f3g5 f8e7 g5f7"  # Nxf7 explodes the black king on e8
    assert F.game_end(start, moves, variant=ATOMIC) == F.END_NO_MOVES | F.END_EXTINCT
    pos = F.game_vpositions(ATOMIC, start, moves)
    ps, po = ev.eval_vpositions(pos)
    assert ps[-1] == 0 and po[-1] == 0 and np.any(po[:-1])
    ops, opo, rc = on.eval_packed(pos)
    assert rc == 0 and np.array_equal(ps, ops) and np.array_equal(po, opo)
    gs, go = ev.eval_vgroups(pos, np.array([0, len(pos)], np.uint32))
    assert np.array_equal(gs, ps) and np.array_equal(go, po)
    bad = np.concatenate([pos, pos[-1:]])
    bad[-1, :32] &= np.where((bad[-1, :32] & 15) == 6, 0xF0, 0xFF).astype(np.uint8)  # drop the white king too
    bad[-1, :32] &= np.where((bad[-1, :32] >> 4) == 6, 0x0F, 0xFF).astype(np.uint8)
    with pytest.raises(F.FnnueError) as e:
        ev.eval_vpositions(bad)
    assert e.value.name == "FNNUE_E_POSITION" and f"index {len(pos)}" in str(e.value)


def test_variant_full_batch(vcache):
    """1M crazyhouse positions in one call (the config-2 batch size), sampled
    against the oracle, and the device entry point agrees with the host one."""
    import torch
    ev, on = vcache(CZH)
    pos = F.random_vpositions(77, CZH, 1_000_000, 160)
    ps, po = ev.eval_vpositions(pos)
    idx = np.random.default_rng(1).choice(len(pos), 20000, replace=False)
    ops, opo, rc = on.eval_packed(pos[idx], threads=16)
    assert rc == 0 and np.array_equal(ps[idx], ops) and np.array_equal(po[idx], opo)
    dev = torch.device("cuda", 0)
    d_pos = torch.from_numpy(pos).to(dev)
    d_ps = torch.zeros(len(pos), dtype=torch.int32, device=dev)
    d_po = torch.zeros(len(pos), dtype=torch.int32, device=dev)
    ev.eval_vpositions_device(d_pos.data_ptr(), len(pos), d_ps.data_ptr(), d_po.data_ptr(),
                              torch.cuda.current_stream().cuda_stream)
    ev.check()
    assert np.array_equal(d_ps.cpu().numpy(), ps) and np.array_equal(d_po.cpu().numpy(), po)


def test_variant_multi_device(vcache):
    """fnnue_multi with a variant net (RCCL broadcast of the variant image)."""
    data = F.synthesize_variant_net(3, 512, CZH)
    m = F.MultiEvaluator(F.Net.from_bytes_variant(data, CZH), [0])
    try:
        pos = F.random_vpositions(12, CZH, 5000, 160)
        ps, po = m.ctx(0).eval_vpositions(pos)
        ops, opo, rc = VariantOracleNet(data, CZH).eval_packed(pos, threads=8)
        assert np.array_equal(ps, ops) and np.array_equal(po, opo)
        mps, mpo = m.eval_vpositions(pos)  # fnnue_multi_eval_vpositions (host buffers, sharded)
        assert np.array_equal(mps, ops) and np.array_equal(mpo, opo)
        import torch
        dev = torch.device("cuda", 0)
        d_pos = torch.from_numpy(pos).to(dev)
        d_ps = torch.zeros(len(pos), dtype=torch.int32, device=dev)
        d_po = torch.zeros(len(pos), dtype=torch.int32, device=dev)
        m.eval_vpositions_device([d_pos.data_ptr()], [len(pos)], [d_ps.data_ptr()], [d_po.data_ptr()])
        m.sync()
        assert np.array_equal(d_ps.cpu().numpy(), ops) and np.array_equal(d_po.cpu().numpy(), opo)
    finally:
        m.close()


def test_variant_golden_vectors_on_device():
    """The device path against the committed variant fixture (the same
    vectors tests/test_variant.py checks the restatement against)."""
    import hashlib
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_variant_evals.json")))
    for e in g["nets"]:
        v = e["variant"]
        ev = F.Evaluator(F.Net.from_bytes_variant(F.synthesize_variant_net(e["seed"], e["hd"], v), v), 0)
        try:
            pos = np.stack([F.vpos_from_fen(v, f) for f in e["fens"]])
            ps, po = ev.eval_vpositions(pos)
            assert ps.tolist() == e["psqt"] and po.tolist() == e["positional"]
            walks = F.random_vpositions(e["walks_seed"], v, e["walks_count"], e["walks_max_plies"])
            wps, wpo = ev.eval_vpositions(walks)
            digest = hashlib.sha256(wps.astype("<i4").tobytes() + wpo.astype("<i4").tobytes()).hexdigest()
            assert digest == e["walks_sha256"]
        finally:
            ev.close()
