"""Multi-GPU sharding: the partitioner (host), the fnnue_multi ABI's argument
checks (no GPU needed), a world_size-2 gloo run of the per-rank sharding of
grouped batches, and (-m gpu) the one-process multi-device path at ndev = 1
against the oracle (one MI355X per box; ndev > 1 runs in the driver's
8-GPU bench)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import fishnet_amd as F
from fishnet_amd import _native as N
from tests.conftest import ROOT, net_bytes


def test_partition_groups_balanced():
    rng = np.random.default_rng(5)
    for trial in range(20):
        sizes = rng.integers(0, 300, size=int(rng.integers(1, 2000)))
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
        total, big = int(off[-1]), int(sizes.max())
        for parts in (1, 2, 3, 4, 7, 8, 64):
            cut = F.partition_groups(off, parts)
            assert cut[0] == 0 and cut[-1] == len(sizes)
            assert np.all(np.diff(cut.astype(np.int64)) >= 0)
            for k in range(1, parts):  # each boundary within half a group of the ideal split
                assert abs(int(off[cut[k]]) - total * k // parts) <= big
            shares = np.diff(off[cut].astype(np.int64))
            assert shares.sum() == total


def test_partition_groups_edge_cases():
    off = np.array([0, 5, 5, 5, 12], dtype=np.uint32)  # empty groups
    assert list(F.partition_groups(off, 1)) == [0, 4]
    cut = F.partition_groups(off, 8)  # more parts than groups: empty parts
    assert cut[0] == 0 and cut[-1] == 4 and np.all(np.diff(cut.astype(int)) >= 0)
    assert list(F.partition_groups(np.zeros(1, np.uint32), 3)) == [0, 0, 0, 0]
    for bad in (np.array([1, 5], np.uint32), np.array([0, 5, 3], np.uint32)):
        with pytest.raises(F.FnnueError) as e:
            F.partition_groups(bad, 2)
        assert e.value.name == "FNNUE_E_ARG"
    cut = np.zeros(2, np.uint32)
    assert N.lib.fnnue_partition_groups(N.ptr(off), 4, 0, N.ptr(cut)) == -1


def test_multi_create_argument_checks():
    import ctypes as C
    net = F.Net.from_bytes(net_bytes(7, 128, 0))
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert N.lib.fnnue_multi_create(net.handle, devs, 0, C.byref(h)) == -1  # ndev < 1
    rc = N.lib.fnnue_multi_create(net.handle, devs, 2, C.byref(h))
    # no GPU here -> FNNUE_E_DEVICE; with one, the duplicate device -> FNNUE_E_ARG
    assert rc in (-1, -5) and not h.value
    assert N.lib.fnnue_multi_sync(None) == -1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import fishnet_amd as F
    from fishnet_amd import dist as D
    from oracle.oracle import OracleNet

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cpu = torch.device("cpu")
        pos, off = F.random_playouts(11, 40, mode=F.PLAYOUT_CHILDREN, threads=2)  # same batch on every rank
        g0, g1 = D.shard_groups(off, rank, world)
        lo, hi = int(off[g0]), int(off[g1])
        on = OracleNet(F.synthesize_net(7, 128, 0))  # each rank "evaluates" its shard (CPU stand-in)
        ps, po, rc = on.simd_eval_groups(pos[lo:hi], (off[g0:g1 + 1] - off[g0]).astype(np.uint32), F.GROUP_STAR,
                                         threads=1)
        assert rc == 0
        gps = D.gather_to_rank0(ps, cpu)
        gpo = D.gather_to_rank0(torch.from_numpy(po), cpu)
        q.put((rank, hi - lo, None if gps is None else (gps.tobytes(), gpo.tobytes())))
    finally:
        dist.destroy_process_group()


def test_two_rank_group_sharding_gloo():
    """Whole STAR groups split over 2 ranks by position count; the gathered
    results equal the whole batch evaluated in one piece."""
    from oracle.oracle import OracleNet
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pos, off = F.random_playouts(11, 40, mode=F.PLAYOUT_CHILDREN, threads=2)
    assert res[0][1] + res[1][1] == len(pos)
    assert abs(res[0][1] - res[1][1]) < 400  # balanced by positions (groups are <= ~60 positions)
    ps, po, rc = OracleNet(F.synthesize_net(7, 128, 0)).eval_packed(pos)
    gps, gpo = res[0][2]
    assert np.frombuffer(gps, np.int32).tolist() == ps.tolist()
    assert np.frombuffer(gpo, np.int32).tolist() == po.tolist()


@pytest.mark.gpu
def test_multi_single_device_matches_oracle():
    """fnnue_multi at ndev = 1 (RCCL communicator + broadcast of the image to
    itself): host and device entry points bit-exact against the oracle."""
    import torch
    from oracle.oracle import OracleNet
    data = net_bytes(1, 1024, 0)
    m = F.MultiEvaluator(F.Net.from_bytes(data), [0])
    on = OracleNet(data)
    try:
        pos = F.random_playouts(21, 30000, threads=8)
        ps, po = m.eval_positions(pos)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        assert rc == 0 and np.array_equal(ps, ops) and np.array_equal(po, opo)
        for mode, pm, count in ((F.GROUP_CHAIN, F.PLAYOUT_PLIES, 300), (F.GROUP_STAR, F.PLAYOUT_CHILDREN, 30)):
            gpos, off = F.random_playouts(22, count, mode=pm, threads=8)
            gs, go = m.eval_groups(gpos, off, mode)
            ops, opo, rc = on.eval_packed(gpos, threads=8)
            assert np.array_equal(gs, ops) and np.array_equal(go, opo)
        dev = torch.device("cuda", 0)
        d_pos = torch.from_numpy(pos).to(dev)
        d_ps = torch.zeros(len(pos), dtype=torch.int32, device=dev)
        d_po = torch.zeros(len(pos), dtype=torch.int32, device=dev)
        cur = [torch.cuda.current_stream(dev).cuda_stream]  # ordered after the zero fills above
        m.eval_positions_device([d_pos.data_ptr()], [len(pos)], [d_ps.data_ptr()], [d_po.data_ptr()], cur)
        m.sync()
        assert np.array_equal(d_ps.cpu().numpy(), ps) and np.array_equal(d_po.cpu().numpy(), po)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        d_g = torch.from_numpy(gpos).to(dev)
        d_gs = torch.zeros(len(gpos), dtype=torch.int32, device=dev)
        d_go = torch.zeros(len(gpos), dtype=torch.int32, device=dev)
        m.eval_groups_device([d_g.data_ptr()], [d_off.data_ptr()], [len(off) - 1], [len(gpos)], F.GROUP_STAR,
                             [d_gs.data_ptr()], [d_go.data_ptr()], cur)
        m.sync()
        assert np.array_equal(d_gs.cpu().numpy(), gs) and np.array_equal(d_go.cpu().numpy(), go)
        assert m.ctx(0).device == 0
    finally:
        m.close()
