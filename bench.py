#!/usr/bin/env python3
"""Throughput bench: batched NNUE static evaluation on MI355X.

Metric (BASELINE.json): NNUE positions evaluated/sec + % HBM roofline, bit-exact.

Default workload (N=1 headline) = BASELINE config 2 (configs[1]): 1,000,000
random-playout positions per GPU (splitmix64 seed 1, L ~ U[0,160] random legal
plies), synthetic SFNNv5 net with HD = 1024 (same shapes and file format as
nn-ad9b42354671.nnue, which is not available offline), accumulators from
scratch.  A step = one evaluation call over the HBM-resident batch of every
GPU.  Weak scaling: every GPU evaluates its own 1M-position shard; positions
are independent, so there is no data-path collective.

N > 1, two launch forms, both measuring N GPUs (n_gpus = N is asserted):
  * torchrun --nproc-per-node N bench.py --gpus N   one process per GPU; the
    net image is RCCL-broadcast from rank 0 (torch.distributed "nccl"); the
    timed region is closed by a barrier, the max over ranks is taken; results
    are then gathered to rank 0 over RCCL (gather_ms, outside `value`).
  * python bench.py --gpus N                         one process driving N
    GPUs through the C ABI's fnnue_multi (ncclCommInitAll + ncclBroadcast of
    the image inside libfnnue.so, one stream per device).

Other workloads (the other BASELINE configs, measured for DESIGN.md):
  --workload games     config 3: random-playout games, every ply, incremental (CHAIN)
  --workload children  config 4: every ply of random games plus all legal children (STAR)
  --small-net 128      also evaluate every position with a small net each step (config 3's big + small)
  --workload crazyhouse / atomic
                       config 5: Fairy-Stockfish HalfKAv2-variants nets (synthetic), 1M random-walk
                       variant positions per GPU (pockets / explosions), from scratch
  --workload crazyhouse-games / atomic-games
                       config 5 along games: every ply of 10k random legal variant games per GPU
                       (drops, pockets, explosions), incremental CHAIN (fnnue_eval_vgroups_device)
  --workload backend   the drop-in itself: lichess-shaped acquired analysis batches (FEN + UCI moves,
                       40-160 plies, some chess960 / crazyhouse / atomic) through fnnue_backend_go at
                       --go-batches per call (host text in, responses out: the component fishnet calls)

roofline: the binding resource of the dominant kernel (ft_slices for config
2, ft_segments for configs 3/4) from the committed PMC profile of this tree
(profiles/counters.json, tools/profile_round.sh + tools/roofline.py): VALU
issue, LDS-array busy and bytes past L2, each over the kernel's live time
measured here with HIP events on its launch stream; `frac` = the largest.
"""
from __future__ import annotations

import argparse
import contextlib
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md "Chip-level parameters")
CLOCK_HZ = 2.4e9  # spec peak engine clock
CUS, SIMDS = 256, 1024
VALU_PEAK = SIMDS * CLOCK_HZ / 4  # 64-bit-encoded wave64 VALU instructions/s (4 cycles each per SIMD)
LDS_PEAK = CUS * CLOCK_HZ  # LDS-array busy cycles/s over all CUs
I8_MFMA_PEAK = 5.0e15  # dense int8 MFMA (2x the ~2.5 PF dense BF16 rate per clock)
MFMA_PEAK = SIMDS * CLOCK_HZ  # matrix-core busy cycles/s over all SIMDs (SQ_VALU_MFMA_BUSY_CYCLES counts cycles)
METRIC = "NNUE positions evaluated/sec (1–8 MI355X) + % HBM roofline, bit-exact"
PSQT_BUCKETS = 8
MAIN_KERNEL = {("positions", "sliced"): "ft_slices_kernel", ("positions", "gather"): "ft_scratch_kernel",
               ("groups", "sliced"): "ft_segments_kernel", ("groups", "gather"): "ft_groups_kernel"}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000,
                    help="timed steps (1000: ~1.5 s of config 2, long enough for an SMI sampler to see the GPU busy)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed steps for this many seconds before the warm-up steps (the GPU's clock ramp out of "
                         "the host-only setup; 0: none)")
    ap.add_argument("--workload", choices=["positions", "games", "children", "crazyhouse", "atomic", "crazyhouse-games",
                                           "atomic-games", "backend"], default="positions")
    ap.add_argument("--go-batches", default="1,64,1024,16384",
                    help="backend workload: acquired batches per fnnue_backend_go call (comma list; the value is the "
                         "largest)")
    ap.add_argument("--go-seconds", type=float, default=1.5, help="backend workload: timed wall per batch count")
    ap.add_argument("--go-calls", type=int, default=0, help="backend workload: exactly this many timed calls per count")
    ap.add_argument("--positions", type=int, default=1_000_000, help="positions per GPU (positions / variant workloads)")
    ap.add_argument("--games", type=int, default=None,
                    help="games per GPU (games: 10,000 = config 3; children: 5,000 ~ 12.5M positions per GPU = "
                         "config 4's 1e8 positions over 8 GPUs)")
    ap.add_argument("--hd", type=int, default=1024)
    ap.add_argument("--small-net", type=int, default=0, metavar="HD",
                    help="also evaluate every position with a second (small) net of this width each step "
                         "(BASELINE config 3: big + small net; later Stockfish's small net is HD 128)")
    ap.add_argument("--no-dual", action="store_true",
                    help="with --small-net on groups: two evaluation calls per step instead of one "
                         "fnnue_eval_groups_dual_device call (A/B)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="default run: skip the extra config-3 and engine-actor lines appended after the headline")
    ap.add_argument("--no-host-api", action="store_true", help="skip timing the host-buffer entry points")
    ap.add_argument("--kernel-events", choices=["ft", "all"], default="ft",
                    help="HIP events in the timed steps: around the FT main kernel only (default), or around every "
                         "phase (plan / FT / stacks; each event record costs the stream a few microseconds)")
    ap.add_argument("--threads", type=int, default=0, help="host threads (0 = every core this process may use)")
    ap.add_argument("--ft-impl", choices=["sliced", "gather"], default="sliced",
                    help="feature-transformer kernel for independent positions")
    ap.add_argument("--launch", choices=["auto", "devices", "ranks"], default="auto",
                    help="devices: drive the GPUs through fnnue_multi from this process even at --gpus 1; "
                         "ranks: the torchrun path (RCCL broadcast, max over ranks, gather) even at WORLD_SIZE 1 "
                         "(auto: torchrun ranks if WORLD_SIZE > 1, else fnnue_multi for --gpus > 1)")
    return ap.parse_args()


def host_cpus() -> dict:
    """The host cores this process may use ([ref] src/configure.rs:196-206:
    Cores::All = available_parallelism, i.e. the affinity set / cgroup quota)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = total
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    share = os.environ.get("OMP_NUM_THREADS")
    # The GPU box exports OMP_NUM_THREADS = its CPU share per GPU (16); a box
    # whose affinity set shows the whole machine is capped to that share.
    if share and share.isdigit() and 0 < int(share) < usable:
        usable = int(share)
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "os_cpu_count": total, "affinity": aff, "cgroup_quota": quota,
            "omp_num_threads": share, "model": model}


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


def tree_hash() -> str:
    spec = importlib.util.spec_from_file_location("roofline_tool", os.path.join(ROOT, "tools", "roofline.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.tree_hash()


def resource_fractions(c: dict, t_s: float) -> dict:
    """Fractions of VALU issue, LDS-array busy and HBM for one launch of a
    kernel whose per-launch counters are `c`, running t_s seconds."""
    fr = {}
    if c.get("SQ_INSTS_VALU"):
        fr["valu"] = {"achieved": c["SQ_INSTS_VALU"] / t_s, "peak": VALU_PEAK, "unit": "VALU wave-instr/s"}
    if c.get("SQ_LDS_IDX_ACTIVE"):
        fr["lds"] = {"achieved": c["SQ_LDS_IDX_ACTIVE"] / t_s, "peak": LDS_PEAK, "unit": "LDS-busy CU-cycles/s"}
    if c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        fr["mfma"] = {"achieved": c["SQ_VALU_MFMA_BUSY_CYCLES"] / t_s, "peak": MFMA_PEAK,
                      "unit": "MFMA-busy SIMD-cycles/s"}
    if c.get("FETCH_SIZE") is not None and c.get("WRITE_SIZE") is not None:
        b = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        fr["hbm"] = {"achieved": b / t_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s", "bytes": b}
    for v in fr.values():
        v["frac"] = round(v["achieved"] / v["peak"], 4)
        v["achieved"] = round(v["achieved"], 1) if v["unit"] == "GB/s" else float(f"{v['achieved']:.4g}")
    return fr


class Shard:
    """One GPU's HBM-resident inputs and outputs."""

    def __init__(self, torch, dev, pos, off, small):
        self.dev = dev
        self.n = len(pos)
        self.pos = torch.from_numpy(pos).to(dev)
        self.off = torch.from_numpy(off.astype(np.uint32).view(np.int32)).to(dev) if off is not None else None
        self.ng = len(off) - 1 if off is not None else 0
        self.psqt = torch.zeros(self.n, dtype=torch.int32, device=dev)
        self.positional = torch.zeros(self.n, dtype=torch.int32, device=dev)
        self.small = torch.zeros(2, self.n, dtype=torch.int32, device=dev) if small else None


@contextlib.contextmanager
def stdout_to_stderr():
    """RCCL prints a version banner on stdout when a communicator is created;
    the bench's stdout is its one JSON line, so fd 1 points at stderr meanwhile."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def variant_of(F, workload):
    return {"crazyhouse": F.VARIANT_CRAZYHOUSE, "atomic": F.VARIANT_ATOMIC}.get(workload.replace("-games", ""))


def make_inputs(F, args, seed, threads):
    off = None
    variant = variant_of(F, args.workload)
    if variant is not None and args.workload.endswith("-games"):
        pos, off = F.random_vgames(seed + 1, variant, args.games, 160, threads=threads)
    elif variant is not None:
        pos = F.random_vpositions(seed, variant, args.positions, 160)
    elif args.workload == "positions":
        pos = F.random_playouts(seed, args.positions, 0, 160, threads=threads)
    else:
        mode = F.PLAYOUT_PLIES if args.workload == "games" else F.PLAYOUT_CHILDREN
        pos, off = F.random_playouts(seed + 1, args.games, 0, 160, mode=mode, threads=threads)
    return pos, off


def chess960_fen(rng) -> str:
    """A Chess960 start position (Shredder-FEN castling letters)."""
    back = [""] * 8
    back[int(rng.choice([0, 2, 4, 6]))] = "b"
    back[int(rng.choice([1, 3, 5, 7]))] = "b"
    for pc in ("q", "n", "n"):
        free = [i for i in range(8) if not back[i]]
        back[int(rng.choice(free))] = pc
    free = [i for i in range(8) if not back[i]]
    for i, pc in zip(free, "rkr"):
        back[i] = pc
    rooks = [chr(ord("a") + i) for i in free[::2]]
    castle = "".join(r.upper() for r in rooks[::-1]) + "".join(rooks[::-1])
    return f"{''.join(back)}/pppppppp/8/8/8/8/PPPPPPPP/{''.join(back).upper()} w {castle} - 0 1"


def lichess_batches(F, seed: int, count: int, c960: float = 0.05, variants: float = 0.04):
    """Acquired analysis batches shaped like lichess work ([ref] src/api.rs:293-309,
    src/stats.rs:136-138: ~60 positions per batch): a root FEN and 40-160
    random legal UCI moves; standard chess, a share of Chess960 starts and of
    crazyhouse / atomic games (seeded)."""
    from fishnet_amd import backend as B
    rng = np.random.default_rng(seed)
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    bodies = []
    for i in range(count):
        plies = int(rng.integers(40, 161))
        u = float(rng.random())
        if u < variants:
            zh = u < variants / 2
            fen = start.replace(" w", "[] w") if zh else start
            name = "crazyhouse" if zh else "atomic"
            mv = F.random_vgame(seed * 1_000_003 + i, F.VARIANT_CRAZYHOUSE if zh else F.VARIANT_ATOMIC, fen, plies)
            bodies.append(B.AcquireResponseBody(f"b{i}", fen, mv, variant=name))
        elif u < variants + c960:
            fen = chess960_fen(rng)
            bodies.append(B.AcquireResponseBody(f"b{i}", fen, F.random_game(seed * 1_000_003 + i, fen, plies),
                                                variant="chess960"))
        else:
            bodies.append(B.AcquireResponseBody(f"b{i}", start, F.random_game(seed * 1_000_003 + i, start, plies)))
    return bodies


def backend_roofline(sizes) -> dict | None:
    """The actor's device work at each batch count from the committed profile
    of this tree (profiles/counters.json, workloads "backend:<k>",
    tools/profile_round.sh): the kernel with the most device time per call
    (its chess instance when the nets share a kernel), its average duration in
    the kernel trace and its binding resource.  The actor has no live kernel
    events, so these times are the profiled run's."""
    cpath = os.path.join(ROOT, "profiles", "counters.json")
    if not os.path.exists(cpath):
        return None
    db = json.load(open(cpath))
    tree_ok = db.get("tree") == tree_hash()
    per = {}
    for k in sizes:
        ks = db.get("workloads", {}).get(f"backend:{k}")
        if not ks:
            continue
        focus = {n: r for n, r in ks.items() if r.get("fractions") and r.get("avg_ns")}
        if not focus:
            continue
        total = {n: r["avg_ns"] * (r.get("calls") or 1) for n, r in focus.items()}
        dom = max(total, key=total.get)
        r = focus[dom]
        fr = r["fractions"]
        per[str(k)] = {"kernel": dom, "instance": r.get("instance"), "avg_ms": round(r["avg_ns"] / 1e6, 4),
                       "bound": r.get("bound"), "frac": round(fr[r["bound"]], 4),
                       "fractions": {n: round(v, 4) for n, v in fr.items()},
                       "waves_per_cu": round(r.get("wave_states", {}).get("mean_waves_per_cu", 0), 2),
                       "others": {n: {"avg_ms": round(x["avg_ns"] / 1e6, 4), "bound": x.get("bound"),
                                      "frac": round(x["fractions"][x["bound"]], 4)}
                                  for n, x in focus.items() if n != dom}}
    if not per:
        return None
    top = per[max(per, key=int)]
    return {"bound": top["bound"], "frac": top["frac"], "kernel": top["kernel"], "per_batches": per,
            "counters": {"source": db.get("source"), "tree_matches": tree_ok},
            "note": "binding resource (largest of VALU-issue / LDS-busy / bytes-past-L2 fractions) of the kernel with "
                    "the most device time per call, counters per dispatch over its kernel-trace duration in the "
                    "profiled run of this tree (profiles/counters.json backend:<k>)"}


def backend_line(args) -> dict:
    """The drop-in as fishnet would call it: fnnue_backend_go over acquired
    analysis batches (host text in, PositionResponses out, one call = one
    step), at several batch counts per call; the CPU baseline expands and
    evaluates the same chess batches on every usable core."""
    import ctypes as C

    import torch

    import fishnet_amd as F
    from fishnet_amd import _native as N
    from fishnet_amd import backend as B

    if args.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--workload backend runs one actor on one GPU (the reference runs one engine per worker)")
    cpus = host_cpus()
    threads = args.threads or cpus["usable"]
    sizes = sorted({int(x) for x in args.go_batches.split(",") if x.strip()})
    t0 = time.time()
    chess_net = F.synthesize_net(args.seed, args.hd, 0)
    zh_net = F.synthesize_variant_net(args.seed + 5, 512, F.VARIANT_CRAZYHOUSE)
    at_net = F.synthesize_variant_net(args.seed + 6, 512, F.VARIANT_ATOMIC)
    stub, actor = B.channel(F.Net.from_bytes(chess_net), 0,
                            crazyhouse=F.Net.from_bytes_variant(zh_net, F.VARIANT_CRAZYHOUSE),
                            atomic=F.Net.from_bytes_variant(at_net, F.VARIANT_ATOMIC))
    t_net = time.time() - t0
    t0 = time.time()
    bodies = lichess_batches(F, args.seed, max(sizes))
    arr, keep = B._acquired(bodies)
    plies = np.array([B.batch_size(b) for b in bodies], dtype=np.int64)
    cap = int(plies.sum())
    out = (B._Response * cap)()
    off = np.zeros(len(bodies) + 1, dtype=np.uint32)
    rc = np.zeros(len(bodies), dtype=np.int32)
    t_gen = time.time() - t0
    h = actor._h
    # the compact form of the answer (fnnue_backend_go_compact): 16 B per position + 24 B per batch
    cout = (B._Compact * cap)()
    bout = (B._BatchCompact * len(bodies))()
    off_c = np.zeros(len(bodies) + 1, dtype=np.uint32)
    rc_c = np.zeros(len(bodies), dtype=np.int32)

    def go(k):
        N.check(N.lib.fnnue_backend_go(h, arr, k, out, cap, N.ptr(off), N.ptr(rc)))

    def go_compact(k):
        N.check(N.lib.fnnue_backend_go_compact(h, arr, k, cout, cap, bout, N.ptr(off_c), N.ptr(rc_c), 0))

    def timed(fn, k, reps):
        times, phases = [], []
        for _ in range(reps):
            tp = time.perf_counter()
            fn(k)
            times.append(time.perf_counter() - tp)
            phases.append(B.last_stats(actor))
        t = np.array(times)
        ph = {key: round(float(np.mean([p[key] for p in phases])), 4)
              for key in ("prep_ms", "device_ms", "fill_ms", "total_ms")}
        ph["stream_syncs_per_go"] = float(np.mean([p["stream_syncs"] for p in phases]))
        ph["host_threads"] = phases[-1]["host_threads"]
        ph["host_share"] = round((ph["prep_ms"] + ph["fill_ms"]) / max(ph["total_ms"], 1e-9), 3)
        return t, ph

    rows = []
    for k in sizes:
        npk = int(plies[:k].sum())
        for _ in range(max(args.warmup, 1)):
            go(k)
            go_compact(k)
        # reps from one probe call: about --go-seconds of wall per batch count and form
        tp = time.perf_counter()
        go(k)
        probe = time.perf_counter() - tp
        reps = int(min(2000, max(args.steps if args.steps < 1000 else 3, args.go_seconds / max(probe, 1e-6))))
        if args.go_calls:
            reps = args.go_calls
        t, ph = timed(go, k, reps)
        tc, phc = timed(go_compact, k, reps)
        assert not rc[:k].any() and not rc_c[:k].any(), "a synthetic batch failed"
        rows.append({"batches_per_go": k, "positions_per_go": npk, "calls": reps,
                     "ms_per_go_mean": round(float(t.mean()) * 1e3, 4),
                     "ms_per_go_median": round(float(np.median(t)) * 1e3, 4),
                     "ms_per_go_min": round(float(t.min()) * 1e3, 4),
                     "positions_per_s": npk / float(t.mean()), "actor_phases_ms": ph,
                     "compact": {"ms_per_go_mean": round(float(tc.mean()) * 1e3, 4),
                                 "ms_per_go_median": round(float(np.median(tc)) * 1e3, 4),
                                 "ms_per_go_min": round(float(tc.min()) * 1e3, 4),
                                 "positions_per_s": npk / float(tc.mean()), "actor_phases_ms": phc}})
    top = rows[-1]
    kmax = top["batches_per_go"]
    # the compact answer of the largest call carries the same results as the full records
    nres = int(off[kmax])
    compact_same = bool(np.array_equal(off[:kmax + 1], off_c[:kmax + 1]) and all(
        (cout[i].psqt, cout[i].positional) == (out[i].psqt, out[i].positional) for i in range(0, nres, 97)) and all(
        cout[i].score == out[i].score for i in range(0, nres, 97)))
    # results of the last (largest) call: parity spot check + CPU baseline on the chess batches
    got_ps = np.array([out[i].psqt for i in range(int(off[kmax]))], dtype=np.int32)
    got_po = np.array([out[i].positional for i in range(int(off[kmax]))], dtype=np.int32)
    cpu = parity = None
    if not args.no_cpu_baseline:
        from oracle.oracle import OracleNet  # cpu_baseline leg (test infrastructure)
        from oracle.oracle import lib as olib
        chess = [i for i in range(kmax) if bodies[i].variant in ("standard", "chess960")]
        games = [(bodies[i].position, bodies[i].moves) for i in chess]
        text, fo, mo = F.pack_games(games)
        oo = np.concatenate([[0], np.cumsum(plies[chess])]).astype(np.uint32)
        on = OracleNet(chess_net)
        done, t_cpu = 0, time.perf_counter()
        first = None
        while True:
            ps, po, crc = on.simd_eval_games(text, fo, mo, oo, threads=threads)
            assert crc == 0
            first = first or (ps, po)
            done += int(oo[-1])
            if time.perf_counter() - t_cpu >= args.cpu_seconds:
                break
        cpu_el = time.perf_counter() - t_cpu
        isa = "AVX-512 VNNI" if olib.cpu_simd_isa512() else "AVX2"
        cpu = {"value": done / cpu_el, "unit": "positions/s", "cores": threads, "kind": "port",
               "cpu": {k: cpus[k] for k in ("model", "os_cpu_count", "affinity", "cgroup_quota", "omp_num_threads")},
               "sample": f"the {len(chess)} chess batches ({int(oo[-1])} plies) of the largest call, repeated for "
                         f"{cpu_el:.1f} s on {threads} threads: FEN parse + UCI replay + every ply evaluated along "
                         f"the game (oracle/nnue_cpu_simd.c cpu_simd_eval_games, Stockfish's {isa} NNUE code paths "
                         f"restated; variant batches excluded: no Fairy-Stockfish SIMD code exists offline)"}
        idx = np.concatenate([np.arange(off[i], off[i + 1]) for i in chess]) if chess else np.zeros(0, np.int64)
        parity = {"checked": int(len(idx)),
                  "mismatches": int(((got_ps[idx] != first[0]) | (got_po[idx] != first[1])).sum())}
    actor.close()
    nvar = sum(1 for b in bodies[:kmax] if b.variant in ("crazyhouse", "atomic"))
    n960 = sum(1 for b in bodies[:kmax] if b.variant == "chess960")
    line = {
        "metric": METRIC, "value": top["positions_per_s"], "unit": "positions/s", "n_gpus": 1,
        "steps": top["calls"], "warmup": args.warmup, "ms_per_step": top["ms_per_go_mean"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16", "data": "synthetic",
        "config": {"workload": f"fnnue_backend_go over lichess-shaped acquired analysis batches (root FEN + 40-160 "
                               f"random legal UCI moves; {n960} chess960, {nvar} crazyhouse/atomic of {kmax}); "
                               f"host text in, one PositionResponse per ply out, synthetic nets (chess HD {args.hd}, "
                               f"variants HD 512)",
                   "batches_per_go": kmax, "positions_per_go": top["positions_per_go"], "parallelism": "dp1"},
        "backend": rows,
        "compact_same_results": compact_same,
        "roofline": backend_roofline(sizes),
        "cpu_baseline": cpu, "parity_spot_check": parity,
        "setup_s": {"net": round(t_net, 2), "inputs": round(t_gen, 2)},
    }
    del keep
    return line


def run(args) -> dict | None:
    """One workload (args.workload) measured; rank 0 returns the JSON line."""
    if args.games is None:
        args.games = 5_000 if args.workload == "children" else 10_000
    import torch
    import torch.distributed as dist

    import fishnet_amd as F
    from fishnet_amd import dist as D

    rank, world, local = D.env_rank()
    if world > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch N ranks for N GPUs")
    if args.launch == "ranks" and "MASTER_PORT" not in os.environ:
        raise SystemExit("--launch ranks needs a torchrun environment (MASTER_ADDR / MASTER_PORT)")
    launch = "ranks" if world > 1 or args.launch == "ranks" else (
        "devices" if args.gpus > 1 or args.launch == "devices" else "single")
    ndev_here = args.gpus if launch == "devices" else 1
    have = F.device_count()
    need = (local + 1) if launch != "devices" else args.gpus
    if have < need:
        raise SystemExit(f"bench needs {need} visible GPU(s) for --gpus {args.gpus}, found {have}")
    devices = list(range(args.gpus)) if launch == "devices" else [local]
    cpus = host_cpus()
    threads = args.threads or cpus["usable"]
    torch.cuda.set_device(devices[0])
    dist_on = launch == "ranks"
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with stdout_to_stderr():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    variant = variant_of(F, args.workload)
    if variant is not None and args.small_net:
        raise SystemExit("--small-net applies to the chess workloads")
    vgames = args.workload.endswith("-games")
    groups = args.workload in ("games", "children") or vgames
    gmode = None if not groups else (F.GROUP_STAR if args.workload == "children" else F.GROUP_CHAIN)

    # ---- net: rank 0 / device 0 holds it, RCCL broadcasts it over xGMI ----
    t0 = time.time()
    multi = multi_small = None
    nets = [(args.seed, args.hd)] + ([(args.seed + 1000, args.small_net)] if args.small_net else [])
    evs = []  # per net: list of per-device contexts
    for seed, hd in nets:
        if variant is not None:
            # variant nets: every rank / device builds its context from the net
            # file (fnnue_multi RCCL-broadcasts the image for the devices launch)
            vnet = F.Net.from_bytes_variant(F.synthesize_variant_net(seed, hd, variant), variant)
            if launch == "devices":
                with stdout_to_stderr():
                    multi = F.MultiEvaluator(vnet, devices)
                evs.append([multi.ctx(i) for i in range(len(devices))])
            else:
                evs.append([F.Evaluator(vnet, local)])
            continue
        if launch == "devices":
            with stdout_to_stderr():
                m = F.MultiEvaluator(F.Net.from_bytes(F.synthesize_net(seed, hd, 0)), devices)
            if multi is None:
                multi = m
            else:
                multi_small = m
            evs.append([m.ctx(i) for i in range(len(devices))])
        else:
            dev = torch.device("cuda", local)
            image = F.Net.from_bytes(F.synthesize_net(seed, hd, 0)).image() if rank == 0 else None
            with stdout_to_stderr():
                img = D.broadcast_image(image, dev) if dist_on else torch.from_numpy(image).to(dev)
            torch.cuda.synchronize()
            evs.append([F.Evaluator(None, local, image_ptr=img.data_ptr(), image_bytes=img.numel(), hd=hd)])
            del img
    for e in evs[0] if variant is None else []:
        e.set_ft_impl(F._native.FT_GATHER if args.ft_impl == "gather" else F._native.FT_SLICED)
    t_net = time.time() - t0

    # ---- inputs: one shard per GPU, resident in HBM ----
    t0 = time.time()
    shards, host0 = [], None
    for i, d in enumerate(devices):
        g = rank if dist_on else i
        pos, off = make_inputs(F, args, D.shard_seed(args.seed, g), threads)
        if host0 is None:
            host0 = (pos, off)
        shards.append(Shard(torch, torch.device("cuda", d), pos, off, args.small_net))
    pos, off = host0
    board = boards_of(pos)
    if variant is not None and vgames:
        hand = pos[:, 33:43].astype(np.int64)
        starts = off[:-1].astype(np.int64)
        has_base = np.ones(len(pos), dtype=bool)
        has_base[starts] = False
        base_idx = np.arange(len(pos)) - 1
        base_idx[~has_base] = 0
        # board rows as for chess, plus each pocket change as a hand row, both perspectives
        rows = rows_incremental(board, board[base_idx], has_base) + np.where(
            has_base, 2 * np.abs(hand - hand[base_idx]).sum(axis=1), 2 * hand.sum(axis=1))
        vname = args.workload.replace("-games", "")
        workload = ("BASELINE config 5 along games: every ply of %d random legal %s games per GPU (L~U[0,160], %s), "
                    "incremental CHAIN accumulators, synthetic Fairy-Stockfish HalfKAv2-variants net (HD=%d)"
                    % (args.games, vname, "drops, captures to the pocket" if vname == "crazyhouse" else "explosions",
                       args.hd))
    elif variant is not None:
        hand = pos[:, 33:43].astype(np.int64).sum(axis=1)
        rows = rows_scratch(board) + 2 * hand
        workload = ("BASELINE config 5: %s random-walk positions (pseudo-legal moves, %s; L~U[0,160]), "
                    "from-scratch accumulators, synthetic Fairy-Stockfish HalfKAv2-variants net (HD=%d)"
                    % (args.workload, "drops and captures to hand" if args.workload == "crazyhouse"
                       else "explosions", args.hd))
    elif not groups:
        rows = rows_scratch(board)
        workload = ("BASELINE config 2: random-playout positions (splitmix64, L~U[0,160]), from-scratch "
                    "accumulators, synthetic SFNNv5 net (HalfKAv2_hm, HD=%d)" % args.hd)
    else:
        starts = off[:-1].astype(np.int64)
        has_base = np.ones(len(pos), dtype=bool)
        has_base[starts] = False
        base_idx = (np.arange(len(pos)) - 1 if args.workload == "games"
                    else starts[np.repeat(np.arange(len(starts)), np.diff(off))])
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
    npos = shards[0].n
    pieces = (board != 0).sum(axis=1)

    def run_net(k):
        outs = [(s.psqt, s.positional) if k == 0 else (s.small[0], s.small[1]) for s in shards]
        if variant is not None and vgames and launch == "devices":
            multi.eval_vgroups_device([s.pos.data_ptr() for s in shards], [s.off.data_ptr() for s in shards],
                                      [s.ng for s in shards], [s.n for s in shards], gmode,
                                      [o[0].data_ptr() for o in outs], [o[1].data_ptr() for o in outs], streams)
        elif variant is not None and vgames:
            s, e = shards[0], evs[k][0]
            e.eval_vgroups_device(s.pos.data_ptr(), s.off.data_ptr(), s.ng, s.n, gmode, outs[0][0].data_ptr(),
                                  outs[0][1].data_ptr(), torch.cuda.current_stream().cuda_stream)
        elif variant is not None and launch == "devices":
            multi.eval_vpositions_device([s.pos.data_ptr() for s in shards], [s.n for s in shards],
                                         [o[0].data_ptr() for o in outs], [o[1].data_ptr() for o in outs],
                                         streams)
        elif variant is not None:
            s, e = shards[0], evs[k][0]
            e.eval_vpositions_device(s.pos.data_ptr(), s.n, outs[0][0].data_ptr(), outs[0][1].data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
        elif launch == "devices":
            m = multi if k == 0 else multi_small
            if not groups:
                m.eval_positions_device([s.pos.data_ptr() for s in shards], [s.n for s in shards],
                                        [o[0].data_ptr() for o in outs], [o[1].data_ptr() for o in outs], streams)
            else:
                m.eval_groups_device([s.pos.data_ptr() for s in shards], [s.off.data_ptr() for s in shards],
                                     [s.ng for s in shards], [s.n for s in shards], gmode,
                                     [o[0].data_ptr() for o in outs], [o[1].data_ptr() for o in outs], streams)
        else:
            s, e = shards[0], evs[k][0]
            stream = torch.cuda.current_stream().cuda_stream
            if not groups:
                e.eval_positions_device(s.pos.data_ptr(), s.n, outs[0][0].data_ptr(), outs[0][1].data_ptr(), stream)
            else:
                e.eval_groups_device(s.pos.data_ptr(), s.off.data_ptr(), s.ng, s.n, gmode, outs[0][0].data_ptr(),
                                     outs[0][1].data_ptr(), stream)

    # every device's work on torch's current stream of that device (after the
    # input copies); one process launch: no host sync between devices
    streams = [torch.cuda.current_stream(torch.device("cuda", d)).cuda_stream for d in devices]

    # Big + small net over groups on one GPU: one call, one plan
    # (fnnue_eval_groups_dual_device; the small net's FT and stacks overlap
    # the big net's stacks on the small context's stream).
    dual = bool(args.small_net) and groups and launch == "single" and variant is None and not args.no_dual

    def step():
        if dual:
            s, e = shards[0], evs[0][0]
            e.eval_groups_dual_device(evs[1][0], s.pos.data_ptr(), s.off.data_ptr(), s.ng, s.n, gmode,
                                      s.psqt.data_ptr(), s.positional.data_ptr(), s.small[0].data_ptr(),
                                      s.small[1].data_ptr(), torch.cuda.current_stream().cuda_stream)
            return
        for k in range(len(evs)):
            run_net(k)

    def sync_all():
        for d in devices:
            torch.cuda.synchronize(d)

    def check_all():
        for ctxs in evs:
            for e in ctxs:
                e.check()

    # FNNUE_STEP_EVENTS=1 (diagnostic runs only, never the driver's): every
    # step on a stream of torch's own (the evaluator then runs on it, so a
    # torch event pair brackets each step's GPU work)
    diag_stream = torch.cuda.Stream() if os.environ.get("FNNUE_STEP_EVENTS") and launch == "single" else None
    if diag_stream is not None:
        torch.cuda.set_stream(diag_stream)
        streams = [diag_stream.cuda_stream]
    # Clock settle (untimed, before the W warm-up steps): the GPU leaves its
    # idle clock over ~25 steps of sustained work after the host-only setup
    # phase (profiles/r05/driver_gap: a 20-step window after 5 warm-up steps
    # averaged that ramp, 1.58 -> 1.41 ms per step).  The steps are run, in
    # full, until `settle_s` of wall time has passed; the timed steps then see
    # the steady state a serving process runs at.  Reported as "settle".
    settle_steps, ts = 0, time.perf_counter()
    while args.settle_s > 0 and time.perf_counter() - ts < args.settle_s and settle_steps < 10_000:
        step()
        settle_steps += 1
        if settle_steps % 8 == 0:
            sync_all()
    sync_all()
    settle = {"steps": settle_steps, "s": round(time.perf_counter() - ts, 3)}
    for _ in range(args.warmup):
        step()
    sync_all()
    check_all()
    # The timed steps record HIP events only around the FT main kernel (the
    # roofline's kernel): every event record between two kernels costs the
    # stream a few microseconds.  Plan and stack kernel times come from a
    # short untimed pass with events around every phase afterwards.
    ft_only = args.kernel_events == "ft"
    for ctxs in evs:
        ctxs[0].set_timing(True, ft_only=ft_only)
    if dist_on:
        dist.barrier()
    sync_all()
    # (per-step GPU times of a short run against a long one: warm-up, clock or box?)
    step_events = [] if diag_stream is not None else None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if step_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        step()
        if step_events is not None:
            ev[1].record()
            step_events.append(ev)
    sync_all()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = [round(a.elapsed_time(b), 4) for a, b in step_events] if step_events is not None else None
    launches, plan_ms, ft_ms, stack_ms = evs[0][0].timing_phases()
    small_t = evs[1][0].timing_phases() if len(evs) > 1 else None
    if ft_only:
        for ctxs in evs:
            ctxs[0].set_timing(True)
        for _ in range(min(args.steps, 50)):
            step()
        sync_all()
        pl, plan_ms, _, stack_ms = evs[0][0].timing_phases()
        plan_ms, stack_ms = plan_ms * launches / max(pl, 1), stack_ms * launches / max(pl, 1)
        if small_t is not None:
            spl, sp, _, ss = evs[1][0].timing_phases()
            small_t = (small_t[0], sp * small_t[0] / max(spl, 1), small_t[2], ss * small_t[0] / max(spl, 1))
    for ctxs in evs:
        ctxs[0].set_timing(False)
    # Two nets: each net's phases measured ALONE on the stream (one context per
    # pass, events around every phase).  With both contexts' calls on one
    # stream, the events of the second context's first phase are stamped
    # before the first context's last kernel ends (per-net phase
    # sums past the step), and the dual call overlaps the two nets; so the
    # per-net costs come from these passes, the two-net step from the timed
    # steps above.
    nets_alone = None
    if len(evs) > 1 and launch == "single":
        nets_alone = []
        m = max(5, min(args.steps, 50))
        for k in range(len(evs)):
            e = evs[k][0]
            e.set_timing(True)
            sync_all()
            ta = time.perf_counter()
            for _ in range(m):
                run_net(k)
            sync_all()
            wall = (time.perf_counter() - ta) * 1e3 / m
            _, pa, fa, sa = e.timing_phases()
            e.set_timing(False)
            nets_alone.append({"hd": args.hd if k == 0 else args.small_net, "step_ms": round(wall, 4),
                               "plan_ms": round(pa / m, 4), "ft_kernel_ms": round(fa / m, 4),
                               "stack_kernel_ms": round(sa / m, 4),
                               "phase_sum_ms": round((pa + fa + sa) / m, 4)})
        if not dual:
            # the per-net kernel times of this line: each net alone (a launch per step per net here)
            a0, a1 = nets_alone
            launches = max(launches, 1)
            plan_ms, ft_ms, stack_ms = (a0["plan_ms"] * launches, a0["ft_kernel_ms"] * launches,
                                        a0["stack_kernel_ms"] * launches)
            l1 = max(small_t[0], 1)
            small_t = (l1, a1["plan_ms"] * l1, a1["ft_kernel_ms"] * l1, a1["stack_kernel_ms"] * l1)
    check_all()
    if dist_on:
        elapsed_max = D.max_over_ranks(elapsed, torch.device("cuda", local))
        tot = torch.tensor([float(sum(s.n for s in shards))], dtype=torch.float64, device=shards[0].dev)
        dist.all_reduce(tot)
        total_positions = float(tot.item())
    else:
        elapsed_max, total_positions = elapsed, float(sum(s.n for s in shards))
    n_gpus = world if dist_on else len(devices)
    assert n_gpus == args.gpus, (n_gpus, args.gpus)
    value = total_positions * args.steps / elapsed_max

    # ---- live kernel times (HIP events on the launch stream, device 0) ----
    L = max(launches, 1)
    plan_avg, ft_avg, stack_avg = plan_ms / L, ft_ms / L, stack_ms / L
    bytes_per_launch = float(rows.sum()) * (2 * args.hd + 4 * PSQT_BUCKETS) + npos * (36 + 8)

    # ---- results of device 0 to the host (outside the timed region) ----
    psqt = shards[0].psqt.cpu().numpy()
    positional = shards[0].positional.cpu().numpy()
    gathered = None
    if dist_on:
        # evals gathered back to rank 0 over RCCL (north star "evals are gathered back"), timed on its own
        dev = torch.device("cuda", local)
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        g_ps = D.gather_to_rank0(shards[0].psqt, dev)
        g_po = D.gather_to_rank0(shards[0].positional, dev)
        gms = (time.perf_counter() - tg) * 1e3
        if rank == 0:
            gathered = {"positions": int(g_ps.size), "gather_ms": round(gms, 3),
                        "equals_sum_of_shards": bool(g_ps.size == g_po.size == int(total_positions)),
                        "how": "torch.distributed gather to rank 0 over RCCL"}
    else:
        # one process: every device's results D2H into disjoint slices of one
        # pinned host buffer per output (the per-rank gather of SURVEY §8e)
        sync_all()
        tg = time.perf_counter()
        h_ps = torch.empty(int(total_positions), dtype=torch.int32, pin_memory=True)
        h_po = torch.empty(int(total_positions), dtype=torch.int32, pin_memory=True)
        lo = 0
        for s in shards:
            h_ps[lo:lo + s.n].copy_(s.psqt, non_blocking=True)
            h_po[lo:lo + s.n].copy_(s.positional, non_blocking=True)
            lo += s.n
        sync_all()
        gms = (time.perf_counter() - tg) * 1e3
        gathered = {"positions": lo, "gather_ms": round(gms, 3),
                    "equals_sum_of_shards": bool(lo == int(total_positions)
                                                 and np.array_equal(h_ps[:npos].numpy(), psqt)),
                    "how": "one process: D2H of every device's shard into disjoint slices of pinned host buffers"}
    small = None
    if args.small_net and rank == 0:
        # parity of the small net on a bounded sample against the oracle (test infrastructure)
        from oracle.oracle import OracleNet
        on2 = OracleNet(F.synthesize_net(args.seed + 1000, args.small_net, 0))
        k = min(npos, 200_000)
        ps2, po2, rc2 = on2.simd_eval_packed(pos[:k], threads=threads)
        g2 = shards[0].small[:, :k].cpu().numpy()
        l2, p2, f2, s2 = small_t
        small = {"hd": args.small_net, "plan_avg_ms": round(p2 / max(l2, 1), 4),
                 "ft_kernel_avg_ms": round(f2 / max(l2, 1), 4), "stack_kernel_avg_ms": round(s2 / max(l2, 1), 4),
                 "parity_spot_check": {"checked": k, "mismatches": int(((g2[0] != ps2) | (g2[1] != po2)).sum())
                                       if rc2 == 0 else None}}

    cpu, parity = None, None
    # The CPU baseline at every N (rank 0 / device 0's shard, same host cores):
    # it doubles as the parity spot check of that shard.
    if rank == 0 and not args.no_cpu_baseline and variant is not None:
        from oracle.oracle import VariantOracleNet  # cpu_baseline leg: the scalar C restatement is the CPU port
        on = VariantOracleNet(F.synthesize_variant_net(args.seed, args.hd, variant), variant)
        done, mism, t0 = 0, 0, time.perf_counter()
        while True:
            lo = done % npos
            hi = min(lo + 20_000, npos)
            ps, po, rc = on.eval_packed(pos[lo:hi], threads=threads)
            assert rc == 0
            mism += int(((ps != psqt[lo:hi]) | (po != positional[lo:hi])).sum())
            done += hi - lo
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        cpu_el = time.perf_counter() - t0
        cpu = {"value": done / cpu_el, "unit": "positions/s", "cores": threads, "kind": "port",
               "cpu": {k: cpus[k] for k in ("model", "os_cpu_count", "affinity", "cgroup_quota", "omp_num_threads")},
               "sample": f"{done} positions of the same workload (from-scratch refresh per position; {cpu_el:.1f} s "
                         f"wall on {threads} threads; oracle/variant_oracle.c = scalar C restatement of "
                         f"Fairy-Stockfish's HalfKAv2-variants NNUE, -O3, no SIMD: Fairy-Stockfish itself is absent"
                         + ("; the GPU line is incremental along the games, the CPU port refreshes every ply"
                            if vgames else "") + ")"}
        parity = {"checked": min(done, npos), "mismatches": mism}
    elif rank == 0 and not args.no_cpu_baseline:
        from oracle.oracle import OracleNet  # cpu_baseline leg: oracle/nnue_cpu_simd.c is the timed CPU port
        from oracle.oracle import lib as olib
        isa = "AVX-512 VNNI" if olib.cpu_simd_isa512() else "AVX2"
        on = OracleNet(F.synthesize_net(args.seed, args.hd, 0))
        done, mism, t0 = 0, 0, time.perf_counter()
        chunk = 100_000
        if groups:
            ng = len(off) - 1
            g_per = max(1, int(chunk * ng / npos))
        g = 0
        while True:
            if not groups:
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
        how = ("from-scratch refresh per position" if not groups else
               "incremental accumulators along the groups, refresh on own-king moves")
        cpu = {"value": done / cpu_el, "unit": "positions/s", "cores": threads, "kind": "port",
               "cpu": {k: cpus[k] for k in ("model", "os_cpu_count", "affinity", "cgroup_quota", "omp_num_threads")},
               "sample": f"{done} positions of the same workload ({how}; {cpu_el:.1f} s wall on {threads} "
                         f"threads = every core this process may use; oracle/nnue_cpu_simd.c = Stockfish's {isa} "
                         f"NNUE code paths restated (register-tiled accumulators, maddubs/VPDPBUSD affine), -O3; "
                         f"bit-identical to the scalar oracle)"}
        parity = {"checked": min(done, npos), "mismatches": mism}
    elif rank == 0 and variant is not None:
        from oracle.oracle import VariantOracleNet
        on = VariantOracleNet(F.synthesize_variant_net(args.seed, args.hd, variant), variant)
        k = min(npos, 50_000)
        ops, opo, rc = on.eval_packed(pos[:k], threads=threads)
        parity = {"checked": k, "mismatches": int(((ops != psqt[:k]) | (opo != positional[:k])).sum())}
    elif rank == 0:
        # spot check of device 0's shard against the oracle (test infrastructure)
        from oracle.oracle import OracleNet
        on = OracleNet(F.synthesize_net(args.seed, args.hd, 0))
        k = min(npos, 100_000)
        ops, opo, rc = on.simd_eval_packed(pos[:k], threads=threads)
        parity = {"checked": k, "mismatches": int(((ops != psqt[:k]) | (opo != positional[:k])).sum())}

    # The host-buffer entry points (host arrays in and out over PCIe, validity
    # checked on the device) — reported beside `value`, never as it.
    host_api = None
    if not dist_on and not args.no_host_api:
        reps = 3
        hpos = pos if launch != "devices" else np.concatenate([pos] * len(devices))
        hoff = off
        if groups and launch == "devices":
            hoff = np.concatenate([off[:-1] + i * off[-1] for i in range(len(devices))] + [[off[-1] * len(devices)]])
        target = multi if launch == "devices" else evs[0][0]
        t0 = time.perf_counter()
        for _ in range(reps):
            if variant is not None and vgames:
                if launch == "devices":
                    hp, hq = evs[0][0].eval_vgroups(pos, off, gmode)  # device 0's shard
                else:
                    hp, hq = target.eval_vgroups(hpos, hoff, gmode)
            elif variant is not None:
                hp, hq = target.eval_vpositions(hpos)  # fnnue_multi_eval_vpositions for the devices launch
            else:
                hp, hq = target.eval_positions(hpos) if not groups else target.eval_groups(hpos, hoff, gmode)
        host_el = time.perf_counter() - t0
        host_api = {"value": len(hpos) * reps / host_el, "unit": "positions/s",
                    "same_results": bool(np.array_equal(hp[:npos], psqt) and np.array_equal(hq[:npos], positional)),
                    "note": f"host (pageable numpy) buffers through the C ABI: H2D {pos.shape[1]} B + D2H 8 B per position "
                            "over PCIe around the same kernels"
                            + (" (fnnue_multi: one host thread per GPU, results into disjoint slices)"
                               if launch == "devices" else "")}

    # ---- roofline: binding resource of the dominant kernel ----
    impl = "sliced" if args.ft_impl == "sliced" else "gather"
    main_k = MAIN_KERNEL[("groups" if groups else "positions", impl)]
    counters, src, tree_ok = None, None, None
    cpath = os.path.join(ROOT, "profiles", "counters.json")
    db = json.load(open(cpath)) if os.path.exists(cpath) else {}
    # counters are keyed by workload, "<workload>@<hd>" for widths other than 1024
    ckey = args.workload if args.hd == 1024 else f"{args.workload}@{args.hd}"
    if db:
        counters = db.get("workloads", {}).get(ckey)
        src = db.get("source")
        tree_ok = db.get("tree") == tree_hash()
    kernels = {}
    for name, t_ms in ((main_k, ft_avg), ("stack_kernel", stack_avg)):
        rec = {"live_avg_ms": round(t_ms, 4)}
        c = (counters or {}).get(name, {}).get("counters")
        if c and t_ms > 0:
            rec["fractions"] = resource_fractions(c, t_ms * 1e-3)
            rec["profiled_avg_ms"] = round((counters[name].get("avg_ns") or 0) / 1e6, 4)
        kernels[name] = rec
    # L1 (fc_0, 16 x HD int8 MACs per position) and fc_1 (32 x 32) on int8 MFMA in stack_kernel: achieved
    # int8 OP/s against the dense I8 matrix peak (2x BF16 per clock: ~5 POP/s, MI355X_MICROARCH.md Matrix cores)
    if stack_avg > 0:
        ops = 2.0 * npos * (16 * args.hd + 32 * 32)
        kernels["stack_kernel"]["mfma_int8"] = {
            "achieved_TOPs": round(ops / (stack_avg * 1e-3) / 1e12, 2), "peak_TOPs": I8_MFMA_PEAK / 1e12,
            "frac": round(ops / (stack_avg * 1e-3) / I8_MFMA_PEAK, 5),
            "note": "algorithmic int8 MACs x 2 of fc_0 + fc_1 per launch over its live time; "
                    "fractions.mfma (if profiled) is SQ_VALU_MFMA_BUSY_CYCLES over SIMD-cycles"}
    fr = kernels[main_k].get("fractions", {})
    roofline = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None}
    if fr:
        bound = max(fr, key=lambda k: fr[k]["frac"])
        b = fr[bound]
        roofline.update(bound=bound, achieved=b["achieved"], peak=b["peak"], unit=b["unit"], frac=b["frac"],
                        traffic=int(fr["hbm"]["bytes"]) if "hbm" in fr else None)
    roofline.update({
        "kernel": main_k, "kernel_avg_ms": round(ft_avg, 4), "plan_avg_ms": round(plan_avg, 4),
        "stack_kernel_avg_ms": round(stack_avg, 4), "kernels": kernels,
        "gather_equivalent_GBps": round(bytes_per_launch / (ft_avg * 1e-3) / 1e9, 1) if ft_avg > 0 else None,
        "algorithmic_bytes_per_launch": int(bytes_per_launch),
        "counters": {"source": src, "tree_matches": tree_ok},
        "live_times": ("overlapped: the big and the small net's kernels share the CUs on two streams (dual call); "
                       "counters were profiled per net alone, so these fractions are lower bounds of each kernel's "
                       "own rate (nets_alone: each net's phases alone)") if dual else (
            "the big net alone on the stream (its own pass; the timed steps run both nets)" if nets_alone
            else "kernel alone on the device"),
        "note": "frac = the largest of VALU-issue / LDS-busy / HBM fractions of the dominant kernel (counters per "
                "launch from the committed profile of this tree, over the live kernel time here; peaks at the "
                "2.4 GHz spec clock); gather_equivalent_GBps = SURVEY §8d algorithmic bytes (every feature row "
                "read from memory) over the same time: the sliced kernels read rows from LDS tiles, so it may "
                "exceed the 8 TB/s HBM peak"})

    if small is not None:
        # the small net's own feature-transformer roofline: its counters (profiled
        # alone at its width) over its live kernel time in this run
        sc = db.get("workloads", {}).get(f"{args.workload}@{args.small_net}", {}).get(main_k, {}).get("counters")
        sft = small["ft_kernel_avg_ms"]
        if sc and sft > 0:
            sfr = resource_fractions(sc, sft * 1e-3)
            sb = max(sfr, key=lambda k: sfr[k]["frac"])
            small["roofline"] = {"kernel": main_k, "bound": sb, "frac": sfr[sb]["frac"], "fractions": sfr,
                                 "counters": {"source": db.get("source"), "tree_matches": tree_ok,
                                              "key": f"{args.workload}@{args.small_net}"},
                                 "live_times": "overlapped with the big net's kernels (dual call)" if dual
                                 else "the small net alone on the stream (its own pass)"}
        small["how"] = ("one fnnue_eval_groups_dual_device call per step: one plan, the small net's FT + stacks on "
                        "the small context's stream beside the big net's FT and stacks" if dual else
                        "a second evaluation call per step on the small net's context")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "positions/s",
            "n_gpus": n_gpus,
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
                "parallelism": f"dp{n_gpus}",
                "launch": {"ranks": "torchrun: one process per GPU, RCCL broadcast of the net",
                           "devices": "one process, fnnue_multi over %d GPUs (RCCL broadcast inside the C ABI)"
                                      % n_gpus,
                           "single": "one process, one GPU"}[launch],
                "ft_impl": "groups" if groups else ("sliced (variant tiles)" if variant is not None else args.ft_impl),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity_spot_check": parity,
            "gathered": gathered,
            "host_api": host_api,
            "small_net": small,
            "setup_s": {"net": round(t_net, 2), "inputs": round(t_gen, 2)},
            "settle": settle,
        }
        if nets_alone is not None:
            out["nets_alone"] = nets_alone
        if step_ms is not None:
            out["step_ms"] = step_ms
    for ctxs in evs:
        for e in ctxs:
            e.close()
    for m in (multi, multi_small):
        if m is not None:
            m.close()
    if dist_on:
        dist.destroy_process_group()
    return out if rank == 0 else None


def move_work_line(args) -> dict:
    """The engine actor's move work (Work::Move, [ref] src/api.rs:160-165: the
    position after all moves, a one-ply search over its legal children) at 1
    and 8 move batches per go(): median latency over repeated calls; spot
    check: each answer's best child evaluated by the oracle (its psqt /
    positional negated) and its legal-children count."""
    import fishnet_amd as F
    from fishnet_amd import backend as B
    from oracle.oracle import OracleNet  # spot check only (test infrastructure)
    net = F.synthesize_net(args.seed, args.hd, 0)
    stub, actor = B.channel(F.Net.from_bytes(net), 0)
    on = OracleNet(net)
    rows, checked, bad = [], 0, 0
    try:
        pool = [b for b in lichess_batches(F, args.seed + 17, 64) if b.variant in ("standard", "chess960")]
        for nb in (1, 8):
            bodies = [B.AcquireResponseBody(f"m{i}", b.position, b.moves, work="move", variant=b.variant)
                      for i, b in enumerate(pool[:nb])]
            for _ in range(10):
                res = stub.go(bodies)
            ts, t_end = [], time.perf_counter() + 0.3
            while time.perf_counter() < t_end or len(ts) < 20:
                t = time.perf_counter()
                res = stub.go(bodies)
                ts.append((time.perf_counter() - t) * 1e3)
            for b, r in zip(bodies, res):
                (r,) = r
                _, goff = F.game_children(b.position, b.moves)  # the last group: the root and its children
                checked += 1
                ok = r.nodes == int(goff[-1]) - int(goff[-2]) - 1
                if ok and r.best_move and r.score.kind == "cp":
                    child = F.game_positions(b.position, b.moves + " " + r.best_move)[-1:]
                    ps, po, rc = on.eval_packed(child)
                    ok = rc == 0 and r.psqt == -int(ps[0]) and r.positional == -int(po[0])
                bad += 0 if ok else 1
            rows.append({"move_batches_per_go": nb, "children": int(sum(r[0].nodes for r in res)),
                         "calls": len(ts), "ms_per_go_median": round(float(np.median(ts)), 4)})
    finally:
        actor.close()
    return {"workload": "fnnue_backend_go over move batches (the position after 40-160 random legal moves, "
                        "standard and Chess960; best child by a one-ply search over the legal children)",
            "per_batches": rows, "parity_spot_check": {"checked": checked, "mismatches": bad}}


def extra_lines(args) -> dict:
    """The default run's extra workloads, measured after
    the headline and outside its timed steps: BASELINE config 3 with the big +
    small net through the dual call (20 steps), the engine actor at 1 / 64 /
    1024 acquired batches per go(), and its move work at 1 / 8 move batches;
    each with its own oracle spot check."""
    extra = {}
    t0 = time.time()
    a3 = argparse.Namespace(**vars(args))
    a3.workload, a3.games, a3.small_net, a3.no_dual = "games", 10_000, 128, False
    a3.steps, a3.warmup, a3.cpu_seconds, a3.no_host_api = 20, 3, 1.0, True
    o = run(a3)
    r = o["roofline"]
    extra["config3_big_small"] = {
        "workload": o["config"]["workload"], "value": o["value"], "unit": o["unit"], "steps": o["steps"],
        "ms_per_step": o["ms_per_step"], "dual_call": True,
        "roofline": {k: r.get(k) for k in ("kernel", "bound", "frac", "kernel_avg_ms", "plan_avg_ms",
                                           "stack_kernel_avg_ms", "live_times")},
        "small_net": {k: o["small_net"].get(k) for k in ("hd", "ft_kernel_avg_ms", "stack_kernel_avg_ms",
                                                         "parity_spot_check")},
        "nets_alone": o.get("nets_alone"), "parity_spot_check": o["parity_spot_check"],
        "cpu_baseline": {k: o["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind")}
        if o.get("cpu_baseline") else None}
    ab = argparse.Namespace(**vars(args))
    ab.workload, ab.go_batches, ab.go_seconds, ab.go_calls = "backend", "1,64,1024", 0.3, 0
    ab.steps, ab.warmup, ab.cpu_seconds = 1000, 3, 1.0
    o = backend_line(ab)
    extra["actor"] = {"workload": o["config"]["workload"], "per_batches": [
        {k: row[k] for k in ("batches_per_go", "positions_per_go", "calls", "ms_per_go_median", "ms_per_go_mean",
                             "positions_per_s", "actor_phases_ms", "compact")} for row in o["backend"]],
        "parity_spot_check": o["parity_spot_check"], "compact_same_results": o["compact_same_results"],
        "roofline": o.get("roofline"),
        "cpu_baseline": {k: o["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind")}
        if o.get("cpu_baseline") else None}
    extra["move_work"] = move_work_line(args)
    extra["seconds"] = round(time.time() - t0, 1)
    return extra


def main():
    args = parse_args()
    if args.workload == "backend":
        print(json.dumps(backend_line(args)), flush=True)
        return
    default_run = (args.workload == "positions" and args.gpus == 1 and not args.small_net and args.hd == 1024
                   and int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.launch == "auto")
    out = run(args)
    if out is None:
        return
    if default_run and not args.no_extra:
        out["extra"] = extra_lines(args)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
