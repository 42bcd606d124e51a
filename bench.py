#!/usr/bin/env python3
"""Throughput bench: batched NNUE static evaluation on MI355X.

Metric (BASELINE.json): NNUE positions evaluated/sec + % HBM roofline, bit-exact.
Workload at N=1 = BASELINE config 2 (configs[1]): 1,000,000 random-playout
positions (splitmix64 seed 1, L ~ U[0,160] random legal plies), synthetic
SFNNv5 net with HD = 1024 (same shapes/format as nn-ad9b42354671.nnue, which
is not available offline), accumulators from scratch.  A step = one
fnnue_eval_positions_device call over the resident batch (feature
transformer kernel + layer-stack kernel).  For N > 1 every rank evaluates its
own 1M-position shard (weak scaling; positions are independent, no data-path
collective); the net image is RCCL-broadcast from rank 0 once at start-up.

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
METRIC = "NNUE positions evaluated/sec (1–8 MI355X) + % HBM roofline, bit-exact"


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--positions", type=int, default=1_000_000, help="positions per GPU")
    ap.add_argument("--hd", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--threads", type=int, default=0, help="host threads (0 = min(16, cpu_count))")
    ap.add_argument("--ft-impl", choices=["sliced", "gather"], default="sliced",
                    help="feature-transformer kernel: LDS-stationary tiles (default) or per-position gather")
    return ap.parse_args()


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
    dist_on = world > 1
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    # ---- net: synthesized on rank 0, device image broadcast over RCCL/xGMI ----
    t0 = time.time()
    image = F.Net.from_bytes(F.synthesize_net(args.seed, args.hd, 0)).image() if rank == 0 else None
    if dist_on:
        img = D.broadcast_image(image, torch.device("cuda", local))
    else:
        img = torch.from_numpy(image).cuda()
    torch.cuda.synchronize()
    ev = F.Evaluator(None, local, image_ptr=img.data_ptr(), image_bytes=img.numel(), hd=args.hd)
    ev.set_ft_impl(F._native.FT_GATHER if args.ft_impl == "gather" else F._native.FT_SLICED)
    del img
    t_net = time.time() - t0

    # ---- inputs: this rank's shard of random-playout positions, resident in HBM ----
    t0 = time.time()
    pos = F.random_playouts(D.shard_seed(args.seed, rank), args.positions, 0, 160, threads=threads)
    t_gen = time.time() - t0
    board = np.zeros((len(pos), 64), dtype=np.uint8)
    board[:, 0::2] = pos[:, :32] & 15
    board[:, 1::2] = pos[:, :32] >> 4
    pieces = (board != 0).sum(axis=1)
    mean_n = float(pieces.mean())
    d_pos = torch.from_numpy(pos).cuda()
    d_psqt = torch.zeros(len(pos), dtype=torch.int32, device="cuda")
    d_positional = torch.zeros(len(pos), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        ev.eval_positions_device(d_pos.data_ptr(), len(pos), d_psqt.data_ptr(), d_positional.data_ptr(),
                                 stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev.check()

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

    elapsed_max = D.max_over_ranks(elapsed, torch.device("cuda", local)) if dist_on else elapsed
    total_positions = args.positions * world * args.steps
    value = total_positions / elapsed_max

    # ---- roofline of the dominant kernel (feature transformer) ----
    # algorithmic bytes/position = n * (2*HD*2 + 4*PB*2) + 36 in + 8 out.
    per_pos = pieces.astype(np.float64) * (2 * args.hd * 2 + 2 * 4 * 8) + 36 + 8
    bytes_per_launch = float(per_pos.sum())
    ft_avg_ms = ft_ms / max(launches, 1)
    stack_avg_ms = stack_ms / max(launches, 1)
    achieved_gbs = bytes_per_launch / (ft_avg_ms * 1e-3) / 1e9

    # ---- results back to host (outside the timed region): spot parity + CPU baseline ----
    psqt = d_psqt.cpu().numpy()
    positional = d_positional.cpu().numpy()
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import OracleNet  # cpu_baseline leg: the oracle is the timed CPU port
        on = OracleNet(F.synthesize_net(args.seed, args.hd, 0))
        done, t0 = 0, time.perf_counter()
        chunk = 100_000
        mism = 0
        while True:
            lo = done % len(pos)
            hi = min(lo + chunk, len(pos))
            ps, po, rc = on.eval_packed(pos[lo:hi], threads=threads)
            assert rc == 0
            mism += int(((ps != psqt[lo:hi]) | (po != positional[lo:hi])).sum())
            done += hi - lo
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        cpu_el = time.perf_counter() - t0
        cpu = {"value": done / cpu_el, "unit": "positions/s", "cores": threads, "kind": "port",
               "sample": f"{done} positions of the same workload (first {min(done, len(pos))} of the batch, "
                         f"{cpu_el:.1f} s wall on {threads} threads, scalar C oracle -O3 -march=x86-64-v3)"}
        parity = {"checked": min(done, len(pos)), "mismatches": mism}

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
                "workload": "BASELINE config 2: random-playout positions (splitmix64, L~U[0,160]), "
                            "from-scratch accumulators, synthetic SFNNv5 net (HalfKAv2_hm, HD=%d)" % args.hd,
                "positions_per_gpu": args.positions,
                "mean_pieces": round(mean_n, 3),
                "hd": args.hd,
                "parallelism": f"dp{world}",
                "ft_impl": args.ft_impl,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": None,
                "kernel": "feature transformer (%s)" % ("ft_slices_kernel + plan_*" if args.ft_impl == "sliced"
                                                         else "ft_scratch_kernel"),
                "kernel_avg_ms": round(ft_avg_ms, 4),
                "stack_kernel_avg_ms": round(stack_avg_ms, 4),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
            },
            "cpu_baseline": cpu,
            "parity_spot_check": parity,
            "setup_s": {"net": round(t_net, 2), "playouts": round(t_gen, 2)},
        }
        print(json.dumps(out), flush=True)
    ev.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
