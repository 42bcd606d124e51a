#!/usr/bin/env python3
"""Throughput bench: batched NNUE static evaluation on MI355X.

Metric (BASELINE.json): NNUE positions evaluated/sec + % HBM roofline, bit-exact.

Default workload (N=1 headline) = BASELINE config 2 (configs[1]): 1,000,000
random-playout positions per GPU (splitmix64 seed 1, L ~ U[0,160] random legal
plies), synthetic SFNNv5 net with HD = 1024 (same shapes and file format as
nn-ad9b42354671.nnue, which is not available offline), accumulators from
scratch.  A step = one fnnue_eval_*_device call over the HBM-resident batch.
For N > 1 every rank evaluates its own shard (weak scaling; positions are
independent, no data-path collective); the net image is RCCL-broadcast from
rank 0 once at start-up.

Other workloads (not the headline line; the other BASELINE configs, measured for DESIGN.md):
  --workload games     config 3: random-playout games, every ply, incremental (CHAIN)
  --workload children  config 4: every ply of random games plus all legal children (STAR)
  --small-net 128      also evaluate every position with a small net each step (config 3's big + small)

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md "Chip-level parameters")
VALU_PEAK = 256 * 4 * 2.4e9 / 4  # VOP3-class wave64 instructions/s: 1024 SIMDs, 4 cycles each at 2.4 GHz
METRIC = "NNUE positions evaluated/sec (1–8 MI355X) + % HBM roofline, bit-exact"
PSQT_BUCKETS = 8


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["positions", "games", "children"], default="positions")
    ap.add_argument("--positions", type=int, default=1_000_000, help="positions per GPU (positions workload)")
    ap.add_argument("--games", type=int, default=10_000, help="games per GPU (games / children workloads)")
    ap.add_argument("--hd", type=int, default=1024)
    ap.add_argument("--small-net", type=int, default=0, metavar="HD",
                    help="also evaluate every position with a second (small) net of this width each step "
                         "(BASELINE config 3: big + small net; later Stockfish's small net is HD 128)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-api", action="store_true", help="skip timing the host-buffer entry points")
    ap.add_argument("--threads", type=int, default=0, help="host threads (0 = min(16, cpu_count))")
    ap.add_argument("--ft-impl", choices=["sliced", "gather"], default="sliced",
                    help="feature-transformer kernel for independent positions")
    return ap.parse_args()


def boards_of(pos: np.ndarray) -> np.ndarray:
    b = np.zeros((len(pos), 64), dtype=np.uint8)
    b[:, 0::2] = pos[:, :32] & 15
    b[:, 1::2] = pos[:, :32] >> 4
    return b


def rows_scratch(board: np.ndarray) -> np.ndarray:
    """Feature rows per position, both perspectives, from scratch (2n)."""
    return 2 * (board != 0).sum(axis=1)


def rows_incremental(board: np.ndarray, base: np.ndarray, has_base: np.ndarray) -> np.ndarray:
    """Rows touched per position when derived from `base` (upstream update_accumulator):
    per perspective, removed + added feature rows, or n rows on a refresh (no
    base, or that perspective's own king moved); never more than a refresh."""
    n = (board != 0).sum(axis=1)
    changed = board != base
    delta = ((base != 0) & changed).sum(axis=1) + ((board != 0) & changed).sum(axis=1)
    rows = np.zeros(len(board), dtype=np.int64)
    for king in (6, 14):
        moved = (board == king).argmax(axis=1) != (base == king).argmax(axis=1)
        refresh = ~has_base | moved
        rows += np.where(refresh, n, np.minimum(n, delta))
    return rows


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    import fishnet_amd as F
    from fishnet_amd import dist as D

    rank, world, local = D.env_rank()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    threads = args.threads or min(16, os.cpu_count() or 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist_on = world > 1
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    # ---- net: synthesized on rank 0, device image broadcast over RCCL/xGMI ----
    t0 = time.time()
    image = F.Net.from_bytes(F.synthesize_net(args.seed, args.hd, 0)).image() if rank == 0 else None
    img = D.broadcast_image(image, dev) if dist_on else torch.from_numpy(image).to(dev)
    torch.cuda.synchronize()
    ev = F.Evaluator(None, local, image_ptr=img.data_ptr(), image_bytes=img.numel(), hd=args.hd)
    ev.set_ft_impl(F._native.FT_GATHER if args.ft_impl == "gather" else F._native.FT_SLICED)
    del img
    ev_small = None
    if args.small_net:
        image2 = (F.Net.from_bytes(F.synthesize_net(args.seed + 1000, args.small_net, 0)).image()
                  if rank == 0 else None)
        img2 = D.broadcast_image(image2, dev) if dist_on else torch.from_numpy(image2).to(dev)
        torch.cuda.synchronize()
        ev_small = F.Evaluator(None, local, image_ptr=img2.data_ptr(), image_bytes=img2.numel(), hd=args.small_net)
        del img2
    t_net = time.time() - t0

    # ---- inputs: this rank's shard, resident in HBM ----
    t0 = time.time()
    seed = D.shard_seed(args.seed, rank)
    off = None
    if args.workload == "positions":
        pos = F.random_playouts(seed, args.positions, 0, 160, threads=threads)
        board = boards_of(pos)
        rows = rows_scratch(board)
        workload = ("BASELINE config 2: random-playout positions (splitmix64, L~U[0,160]), from-scratch "
                    "accumulators, synthetic SFNNv5 net (HalfKAv2_hm, HD=%d)" % args.hd)
    else:
        mode = F.PLAYOUT_PLIES if args.workload == "games" else F.PLAYOUT_CHILDREN
        pos, off = F.random_playouts(seed + 1, args.games, 0, 160, mode=mode, threads=threads)
        board = boards_of(pos)
        starts = off[:-1].astype(np.int64)
        has_base = np.ones(len(pos), dtype=bool)
        has_base[starts] = False
        if args.workload == "games":
            base_idx = np.arange(len(pos)) - 1
        else:
            base_idx = starts[np.repeat(np.arange(len(starts)), np.diff(off))]
        base_idx[~has_base] = 0
        rows = rows_incremental(board, board[base_idx], has_base)
        workload = ("BASELINE config %s: %d random-playout games per GPU, %s, synthetic SFNNv5 net (HD=%d)"
                    % ("3" if args.workload == "games" else "4", args.games,
                       "every ply, incremental CHAIN" if args.workload == "games"
                       else "every ply + all legal 1-ply children, STAR", args.hd))
    if args.small_net:
        workload += (f"; every position also through a second synthetic net of HD {args.small_net} "
                     f"(big + small net, both evaluated each step)")
    t_gen = time.time() - t0
    npos = len(pos)
    pieces = (board != 0).sum(axis=1)
    d_pos = torch.from_numpy(pos).to(dev)
    d_off = torch.from_numpy(off.astype(np.int32)).to(dev) if off is not None else None
    d_psqt = torch.zeros(npos, dtype=torch.int32, device=dev)
    d_positional = torch.zeros(npos, dtype=torch.int32, device=dev)
    d_small = torch.zeros(2, npos, dtype=torch.int32, device=dev) if ev_small else None
    stream = torch.cuda.current_stream()

    def run(e, ps, po):
        if off is None:
            e.eval_positions_device(d_pos.data_ptr(), npos, ps, po, stream.cuda_stream)
        else:
            e.eval_groups_device(d_pos.data_ptr(), d_off.data_ptr(), len(off) - 1, npos,
                                 F.GROUP_CHAIN if args.workload == "games" else F.GROUP_STAR, ps, po,
                                 stream.cuda_stream)

    def step():
        run(ev, d_psqt.data_ptr(), d_positional.data_ptr())
        if ev_small:
            run(ev_small, d_small[0].data_ptr(), d_small[1].data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev.check()
    if ev_small:
        ev_small.check()
        ev_small.set_timing(True)

    ev.set_timing(True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    launches, ft_ms, stack_ms = ev.timing_read()
    ev.set_timing(False)
    ev.check()
    small = None
    if ev_small:
        l2, f2, s2 = ev_small.timing_read()
        ev_small.set_timing(False)
        ev_small.check()
        # parity of the small net on a bounded sample against the oracle (test infrastructure)
        from oracle.oracle import OracleNet
        on2 = OracleNet(F.synthesize_net(args.seed + 1000, args.small_net, 0))
        k = min(npos, 200_000)
        ps2, po2, rc2 = on2.simd_eval_packed(pos[:k], threads=threads)
        g2 = d_small[:, :k].cpu().numpy()
        small = {"hd": args.small_net, "ft_kernel_avg_ms": round(f2 / max(l2, 1), 4),
                 "stack_kernel_avg_ms": round(s2 / max(l2, 1), 4),
                 "parity_spot_check": {"checked": k, "mismatches": int(((g2[0] != ps2) | (g2[1] != po2)).sum())
                                       if rc2 == 0 else None}}
    if dist_on:
        elapsed_max = D.max_over_ranks(elapsed, dev)
        tot = torch.tensor([float(npos)], dtype=torch.float64, device=dev)
        dist.all_reduce(tot)
        total_positions = float(tot.item())
    else:
        elapsed_max, total_positions = elapsed, float(npos)
    value = total_positions * args.steps / elapsed_max

    # ---- roofline of the dominant kernel (feature transformer) ----
    # each feature row costs 2*HD bytes of FT weights + 4*PB bytes of PSQT
    # weights; + 36 B position in + 8 B results out.
    bytes_per_launch = float(rows.sum()) * (2 * args.hd + 4 * PSQT_BUCKETS) + npos * (36 + 8)
    ft_avg_ms = ft_ms / max(launches, 1)
    stack_avg_ms = stack_ms / max(launches, 1)
    achieved_gbs = bytes_per_launch / (ft_avg_ms * 1e-3) / 1e9

    # ---- results back to host (outside the timed region): parity spot check + CPU baseline ----
    psqt = d_psqt.cpu().numpy()
    positional = d_positional.cpu().numpy()
    cpu = None
    parity = None
    gathered = None
    if dist_on:
        # Evals gathered back to rank 0 over RCCL (north star: "evals are gathered
        # back"), outside the timed region: 8 B per position.
        g_ps = D.gather_to_rank0(psqt, dev)
        g_po = D.gather_to_rank0(positional, dev)
        if rank == 0:
            gathered = {"positions": int(g_ps.size), "equals_sum_of_shards": bool(g_ps.size == g_po.size
                                                                                  == int(total_positions))}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import OracleNet  # cpu_baseline leg: oracle/nnue_cpu_simd.c is the timed CPU port
        from oracle.oracle import lib as olib
        isa = "AVX-512 VNNI" if olib.cpu_simd_isa512() else "AVX2"
        on = OracleNet(F.synthesize_net(args.seed, args.hd, 0))
        done, mism, t0 = 0, 0, time.perf_counter()
        chunk = 100_000
        if off is not None:
            gmode = F.GROUP_CHAIN if args.workload == "games" else F.GROUP_STAR
            ng = len(off) - 1
            g_per = max(1, int(chunk * ng / npos))
        g = 0
        while True:
            if off is None:
                lo = done % npos
                hi = min(lo + chunk, npos)
                ps, po, rc = on.simd_eval_packed(pos[lo:hi], threads=threads)
            else:
                g0, g1 = g % ng, min(g % ng + g_per, ng)
                lo, hi = int(off[g0]), int(off[g1])
                ps, po, rc = on.simd_eval_groups(pos[lo:hi], (off[g0:g1 + 1] - off[g0]).astype(np.uint32), gmode,
                                                 threads=threads)
                g += g1 - g0
            assert rc == 0
            mism += int(((ps != psqt[lo:hi]) | (po != positional[lo:hi])).sum())
            done += hi - lo
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        cpu_el = time.perf_counter() - t0
        how = ("from-scratch refresh per position" if off is None else
               "incremental accumulators along the groups, refresh on own-king moves")
        cpu = {"value": done / cpu_el, "unit": "positions/s", "cores": threads, "kind": "port",
               "sample": f"{done} positions of the same workload ({how}; {cpu_el:.1f} s wall on {threads} "
                         f"threads; oracle/nnue_cpu_simd.c = Stockfish's {isa} NNUE code paths restated "
                         f"(register-tiled accumulators, maddubs/VPDPBUSD affine), -O3; bit-identical to the "
                         f"scalar oracle)"}
        parity = {"checked": min(done, npos), "mismatches": mism}

    # The host-buffer entry points (fnnue_eval_positions / _groups: host arrays in,
    # host arrays out, PCIe both ways, host-side validation) — reported beside
    # `value`, never as it (inputs resident in HBM is the contract).
    host_api = None
    if world == 1 and not args.no_host_api:
        ev.set_timing(False)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            if off is None:
                hp, hq = ev.eval_positions(pos)
            else:
                hp, hq = ev.eval_groups(pos, off, F.GROUP_CHAIN if args.workload == "games" else F.GROUP_STAR)
        host_el = time.perf_counter() - t0
        host_api = {"value": npos * reps / host_el, "unit": "positions/s",
                    "same_results": bool(np.array_equal(hp, psqt) and np.array_equal(hq, positional)),
                    "note": "host (pageable numpy) buffers through the C ABI: H2D 36 B + D2H 8 B per position "
                            "over PCIe around the same kernels (validity checked on the device)"}

    # roofline.traffic: PMC-measured bytes per launch of the same workload, from the
    # committed profile (tools/profile.sh + tools/traffic.py -> profiles/traffic.json).
    traffic, traffic_src, issue = None, None, None
    tkey = f"{args.workload}:{args.ft_impl if off is None else 'groups'}:hd{args.hd}"
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        entry = json.load(open(tpath)).get(tkey)
        if entry:
            traffic, traffic_src = entry["bytes_per_launch"], entry["source"]
            if entry.get("valu_insts_per_launch"):
                # The sliced FT moves ~2% of its algorithmic bytes through HBM; what bounds
                # it is vector-instruction issue: SQ_INSTS_VALU per launch
                # (committed PMC profile) over the live kernel time, against one
                # 64-bit-encoded (VOP3/VOP3P/SDWA) wave64 VALU instruction per 4 cycles
                # per SIMD at the 2.4 GHz spec clock (tools/diag/valu_bench.hip).
                rate = entry["valu_insts_per_launch"] / (ft_avg_ms * 1e-3)
                issue = {"unit": "VALU instr/s", "achieved": round(rate, -6), "peak": VALU_PEAK,
                         "frac": round(rate / VALU_PEAK, 4), "source": traffic_src}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "positions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16",
            "data": "synthetic",
            "config": {
                "workload": workload,
                "positions_per_gpu": npos,
                "mean_pieces": round(float(pieces.mean()), 3),
                "hd": args.hd if not args.small_net else f"{args.hd}+{args.small_net}",
                "parallelism": f"dp{world}",
                "ft_impl": args.ft_impl if off is None else "groups",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "issue": issue,
                "kernel": {("positions", "sliced"): "ft_slices_kernel + plan_* (LDS-stationary FT)",
                           ("positions", "gather"): "ft_scratch_kernel",
                           ("groups", "sliced"): "ft_segments_kernel + seg_* plan (incremental on LDS tiles)",
                           ("groups", "gather"): "ft_groups_kernel"}[("positions" if off is None else "groups",
                                                                     args.ft_impl)],
                "kernel_avg_ms": round(ft_avg_ms, 4),
                "stack_kernel_avg_ms": round(stack_avg_ms, 4),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
            },
            "cpu_baseline": cpu,
            "parity_spot_check": parity,
            "gathered": gathered,
            "host_api": host_api,
            "small_net": small,
            "setup_s": {"net": round(t_net, 2), "inputs": round(t_gen, 2)},
        }
        print(json.dumps(out), flush=True)
    ev.close()
    if ev_small:
        ev_small.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
