"""Full-size parity runs, on by default in `-m gpu`.

* test_full_size_parity — north star "bit-exact NNUE evals for >= 1e8
  positions per run": BASELINE config 4's workload (every ply of random games
  plus all their legal 1-ply children, >= 1e8 positions) evaluated on one
  MI355X by both device paths (incremental STAR groups and from-scratch
  sliced), and EVERY result compared with the CPU oracle.  The expansion
  mirrors [ref] src/queue.rs:571-606 (every ply of every game) plus the
  children of SURVEY.md §8d config 4.
* test_config3_full_size — BASELINE config 3 at its full size: 10,000
  random-playout games (seed 2), every ply through the incremental CHAIN
  path with the big (HD 1024) and the small (HD 128) net, every ply of both
  compared with the oracle.

The multi-GPU entry points at full per-GPU size (ndev = 1 here; the 2/8-GPU
runs use exactly these calls with more devices):
* test_config4_shard_multi_groups_device — a config-4 shard (>= 12.5M
  positions = 1e8 / 8 GPUs, STAR) through fnnue_multi_eval_groups_device:
  above one workspace, so the device cuts it into chunks with no host sync.
* test_config3_multi_groups — config 3 (10k games, CHAIN) through
  fnnue_multi_eval_groups with the HD 1024 and HD 128 nets.
* test_config5_multi_vpositions_device — 1M crazyhouse and 1M atomic
  positions through fnnue_multi_eval_vpositions_device.

FNNUE_FULL=<positions> overrides the config-4 size (default 1e8).  JSON
records go to gpurun_out/<name>.json (one line each also on stdout).
Host cost on the GPU box (16 threads): ~10 s generation, ~20 s oracle.
"""
import json
import os
import time

import numpy as np
import pytest

import fishnet_amd as F
from oracle.oracle import OracleNet
from tests.conftest import ROOT, net_bytes

pytestmark = pytest.mark.gpu

TARGET = int(os.environ.get("FNNUE_FULL", "100000000"))


def _threads() -> int:
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


def _record(name: str, rec: dict) -> None:
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", name), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec), flush=True)


@pytest.mark.timeout(900)
def test_full_size_parity():
    import torch

    threads = _threads()
    t0 = time.time()
    pos_parts, off_parts, total, seed, base = [], [np.zeros(1, np.int64)], 0, 3, 0
    while total < TARGET:  # config 4: seed 3, games of U[0,160] plies + all legal children
        p, o = F.random_playouts(seed, 4000, 0, 160, mode=F.PLAYOUT_CHILDREN, threads=threads)
        pos_parts.append(p)
        off_parts.append(o[1:].astype(np.int64) + base)
        base += len(p)
        total += len(p)
        seed += 7919
    pos = np.concatenate(pos_parts)
    off = np.concatenate(off_parts)
    del pos_parts
    t_gen = time.time() - t0
    n, ng = len(pos), len(off) - 1
    print(f"generated {n} positions in {ng} STAR groups in {t_gen:.1f} s", flush=True)
    assert n >= TARGET and n < 2 ** 31

    data = net_bytes(1, 1024, 0)
    ev = F.Evaluator(F.Net.from_bytes(data), 0)
    dev = torch.device("cuda", 0)
    d_pos = torch.from_numpy(pos).to(dev)
    d_off = torch.from_numpy(off.astype(np.uint32).view(np.int32)).to(dev)
    d_ps = torch.empty(n, dtype=torch.int32, device=dev)
    d_po = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    times = {}
    results = {}
    for name in ("groups", "positions"):
        d_ps.fill_(-1)
        d_po.fill_(-1)
        torch.cuda.synchronize()
        t = time.perf_counter()
        if name == "groups":
            ev.eval_groups_device(d_pos.data_ptr(), d_off.data_ptr(), ng, n, F.GROUP_STAR,
                                  d_ps.data_ptr(), d_po.data_ptr(), stream)
        else:
            ev.eval_positions_device(d_pos.data_ptr(), n, d_ps.data_ptr(), d_po.data_ptr(), stream)
        torch.cuda.synchronize()
        times[name] = time.perf_counter() - t
        ev.check()
        results[name] = (d_ps.cpu().numpy(), d_po.cpu().numpy())
        print(f"gpu {name}: {n / times[name] / 1e6:.1f}M positions/s (one call, host-timed)", flush=True)
    ev.close()
    del d_pos, d_off, d_ps, d_po

    gps, gpo = results["groups"]
    sps, spo = results["positions"]
    paths_agree = int(((gps != sps) | (gpo != spo)).sum())

    on = OracleNet(data)
    mism = 0
    t = time.perf_counter()
    step = 10_000_000
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        ops, opo, rc = on.eval_packed(pos[lo:hi], threads=threads)
        assert rc == 0
        mism += int(((ops != gps[lo:hi]) | (opo != gpo[lo:hi])).sum())
        print(f"oracle {hi}/{n} mismatches so far {mism} ({time.perf_counter() - t:.0f} s)", flush=True)
    t_oracle = time.perf_counter() - t

    _record("full_parity.json", {
        "test": "tests/test_gpu_full.py::test_full_size_parity",
        "workload": "BASELINE config 4: random games (seed 3, L~U[0,160]) + all legal 1-ply children, "
                    "synthetic SFNNv5 net HD 1024",
        "positions": n, "groups": ng, "gen_s": round(t_gen, 1),
        "gpu_s": {k: round(v, 3) for k, v in times.items()},
        "gpu_positions_per_s": {k: round(n / v) for k, v in times.items()},
        "oracle_s": round(t_oracle, 1), "oracle_threads": threads,
        "mismatches_vs_oracle": mism, "groups_vs_positions_mismatches": paths_agree})
    assert paths_agree == 0
    assert mism == 0


@pytest.mark.timeout(600)
def test_config3_full_size():
    """10k random games (seed 2, L~U[0,160]), every ply, big HD-1024 + small
    HD-128 net through the shipped config-3 entry point
    fnnue_eval_groups_dual_device (one plan, the small net on its own units),
    CHAIN; every ply of both nets against the oracle."""
    threads = _threads()
    pos, off = F.random_playouts(2, 10_000, 0, 160, mode=F.PLAYOUT_PLIES, threads=threads)
    n, ng = len(pos), len(off) - 1
    rec = {"test": "tests/test_gpu_full.py::test_config3_full_size",
           "workload": "BASELINE config 3: 10,000 random-playout games (seed 2, L~U[0,160]), every ply, "
                       "incremental CHAIN; big (HD 1024) + small (HD 128) synthetic nets, one dual call",
           "positions": n, "games": ng, "nets": {}}
    big_data, small_data = net_bytes(1, 1024, 0), net_bytes(1001, 128, 0)
    big = F.Evaluator(F.Net.from_bytes(big_data), 0)
    small = F.Evaluator(F.Net.from_bytes(small_data), 0)
    t = time.perf_counter()
    ps, po, ps2, po2 = big.eval_groups_dual(small, pos, off, F.GROUP_CHAIN)
    t_gpu = time.perf_counter() - t
    big.close()
    small.close()
    bad = 0
    for hd, data, (gp, go) in ((1024, big_data, (ps, po)), (128, small_data, (ps2, po2))):
        ops, opo, rc = OracleNet(data).eval_packed(pos, threads=threads)
        assert rc == 0
        m = int(((gp != ops) | (go != opo)).sum())
        bad += m
        rec["nets"][f"hd{hd}"] = {"mismatches_vs_oracle": m}
    rec["gpu_dual_host_api_s"] = round(t_gpu, 3)
    _record("config3_full.json", rec)
    assert n > 700_000
    assert bad == 0


def _multi_groups_device(m, pos, off, mode):
    import torch
    dev = torch.device("cuda", 0)
    n = len(pos)
    d_pos = torch.from_numpy(pos).to(dev)
    d_off = torch.from_numpy(off.astype(np.uint32).view(np.int32)).to(dev)
    d_ps = torch.full((n,), -1, dtype=torch.int32, device=dev)
    d_po = torch.full((n,), -1, dtype=torch.int32, device=dev)
    cur = [torch.cuda.current_stream(dev).cuda_stream]
    t = time.perf_counter()
    m.eval_groups_device([d_pos.data_ptr()], [d_off.data_ptr()], [len(off) - 1], [n], mode, [d_ps.data_ptr()],
                         [d_po.data_ptr()], cur)
    t_enq = time.perf_counter() - t
    m.sync()
    t_all = time.perf_counter() - t
    return d_ps.cpu().numpy(), d_po.cpu().numpy(), t_enq, t_all


@pytest.mark.timeout(600)
def test_config4_shard_multi_groups_device():
    """BASELINE config 4 per GPU: 1e8 / 8 = 12.5M positions (random games of
    seed 3 + all legal 1-ply children, STAR) through
    fnnue_multi_eval_groups_device at ndev = 1; every result vs the oracle."""
    threads = _threads()
    want = int(os.environ.get("FNNUE_CONFIG4_SHARD", "12500000"))
    parts, offs, base, seed, total = [], [np.zeros(1, np.int64)], 0, 3, 0
    while total < want:
        p, o = F.random_playouts(seed, 2000, 0, 160, mode=F.PLAYOUT_CHILDREN, threads=threads)
        parts.append(p)
        offs.append(o[1:].astype(np.int64) + base)
        base += len(p)
        total += len(p)
        seed += 7919
    pos, off = np.concatenate(parts), np.concatenate(offs)
    del parts
    n = len(pos)
    data = net_bytes(1, 1024, 0)
    m = F.MultiEvaluator(F.Net.from_bytes(data), [0])
    try:
        ps, po, t_enq, t_all = _multi_groups_device(m, pos, off, F.GROUP_STAR)
    finally:
        m.close()
    on = OracleNet(data)
    mism = 0
    for lo in range(0, n, 5_000_000):
        hi = min(n, lo + 5_000_000)
        ops, opo, rc = on.eval_packed(pos[lo:hi], threads=threads)
        assert rc == 0
        mism += int(((ops != ps[lo:hi]) | (opo != po[lo:hi])).sum())
    _record("config4_shard_multi.json", {
        "test": "tests/test_gpu_full.py::test_config4_shard_multi_groups_device",
        "baseline_config": "config 4: 100M 1-ply children positions over 8 GPUs -> one GPU's shard",
        "entry_point": "fnnue_multi_eval_groups_device (ndev = 1, STAR)",
        "positions": n, "groups": len(off) - 1, "chunks": -(-n // (1 << 20)),
        "enqueue_ms": round(t_enq * 1e3, 3), "call_to_sync_s": round(t_all, 3),
        "mismatches_vs_oracle": mism})
    assert n >= want
    assert mism == 0


@pytest.mark.timeout(600)
def test_config3_multi_groups():
    """BASELINE config 3: 10k games (seed 2), every ply, CHAIN, big HD 1024 +
    small HD 128 net, through fnnue_multi_eval_groups (host buffers)."""
    threads = _threads()
    pos, off = F.random_playouts(2, 10_000, 0, 160, mode=F.PLAYOUT_PLIES, threads=threads)
    rec = {"test": "tests/test_gpu_full.py::test_config3_multi_groups",
           "baseline_config": "config 3: 10k-game corpus, incremental along move sequences, big + small net",
           "entry_point": "fnnue_multi_eval_groups (ndev = 1, CHAIN)", "positions": len(pos),
           "games": len(off) - 1, "nets": {}}
    bad = 0
    for hd, seed in ((1024, 1), (128, 1001)):
        data = net_bytes(seed, hd, 0)
        m = F.MultiEvaluator(F.Net.from_bytes(data), [0])
        try:
            ps, po = m.eval_groups(pos, off, F.GROUP_CHAIN)
        finally:
            m.close()
        ops, opo, rc = OracleNet(data).eval_packed(pos, threads=threads)
        assert rc == 0
        k = int(((ps != ops) | (po != opo)).sum())
        bad += k
        rec["nets"][f"hd{hd}"] = {"mismatches_vs_oracle": k}
    _record("config3_multi.json", rec)
    assert len(pos) > 700_000
    assert bad == 0


@pytest.mark.timeout(600)
def test_config5_multi_vpositions_device():
    """BASELINE config 5: 1M crazyhouse and 1M atomic random-walk positions
    through fnnue_multi_eval_vpositions_device (HD 1024 synthetic variant
    nets), every result vs the variant oracle (parity unpinned: DESIGN §3)."""
    import torch
    from oracle.oracle import VariantOracleNet
    threads = _threads()
    dev = torch.device("cuda", 0)
    rec = {"test": "tests/test_gpu_full.py::test_config5_multi_vpositions_device",
           "baseline_config": "config 5: Fairy-Stockfish variant NNUE (crazyhouse / atomic) batched eval",
           "entry_point": "fnnue_multi_eval_vpositions_device (ndev = 1)", "variants": {}}
    bad = 0
    for name, variant, seed in (("crazyhouse", F.VARIANT_CRAZYHOUSE, 5), ("atomic", F.VARIANT_ATOMIC, 6)):
        data = F.synthesize_variant_net(seed, 1024, variant)
        pos = F.random_vpositions(seed, variant, 1_000_000, 160)
        m = F.MultiEvaluator(F.Net.from_bytes_variant(data, variant), [0])
        try:
            d_pos = torch.from_numpy(pos).to(dev)
            d_ps = torch.full((len(pos),), -1, dtype=torch.int32, device=dev)
            d_po = torch.full((len(pos),), -1, dtype=torch.int32, device=dev)
            m.eval_vpositions_device([d_pos.data_ptr()], [len(pos)], [d_ps.data_ptr()], [d_po.data_ptr()],
                                     [torch.cuda.current_stream(dev).cuda_stream])
            m.sync()
            ps, po = d_ps.cpu().numpy(), d_po.cpu().numpy()
        finally:
            m.close()
        ops, opo, rc = VariantOracleNet(data, variant).eval_packed(pos, threads=threads)
        assert rc == 0
        k = int(((ps != ops) | (po != opo)).sum())
        bad += k
        rec["variants"][name] = {"positions": len(pos), "mismatches_vs_oracle": k}
    _record("config5_multi.json", rec)
    assert bad == 0
