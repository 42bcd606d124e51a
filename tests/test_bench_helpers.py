"""CPU tests of bench.py's algorithmic-byte accounting."""
import numpy as np

import bench
import fishnet_amd as F


def test_rows_scratch_counts_both_perspectives():
    pos = np.stack([F.pos_from_fen("4k3/8/8/8/8/8/8/4K3 w - - 0 1"),
                    F.pos_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1")])
    assert bench.rows_scratch(bench.boards_of(pos)).tolist() == [4, 64]


def test_rows_incremental_quiet_capture_king_move():
    fen = "4k3/8/8/3p4/4P3/8/8/4K3 w - - 0 1"
    pos = F.game_positions(fen, "e4d5 e8d7 e1e2")
    b = bench.boards_of(pos)
    has = np.array([False, True, True, True])
    rows = bench.rows_incremental(b, b[[0, 0, 1, 2]], has)
    # root: refresh 4 pieces x 2; capture: -P(e4) +P(d5) -p(d5) = 3 per perspective;
    # black king move: black refreshes (3 pieces), white -k +k = 2; white king move: 3 + 2
    assert rows.tolist() == [8, 6, 5, 5]


def test_default_arguments_match_the_driver_contract(monkeypatch):
    """No flags: one GPU, a run of minutes at most; the untimed settle phase
    runs before the W warm-up steps and is reported, not counted."""
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = bench.parse_args()
    assert (a.gpus, a.workload, a.positions, a.hd) == (1, "positions", 1_000_000, 1024)
    assert a.steps >= 1 and a.warmup >= 1 and 0 < a.settle_s <= 1.0
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5", "--settle-s", "0"])
    a = bench.parse_args()
    assert (a.steps, a.warmup, a.settle_s) == (20, 5, 0.0)


def test_resource_fractions_use_the_spec_peaks():
    """VALU issue, LDS-busy and bytes past L2 ((2 FETCH_SIZE + WRITE_SIZE) KiB,
    the gfx950 correction) of one launch over its time, against the 2.4 GHz
    spec peaks; the roofline's frac is the largest."""
    t = 1e-3
    c = {"SQ_INSTS_VALU": 0.5 * bench.VALU_PEAK * t, "SQ_LDS_IDX_ACTIVE": 0.25 * bench.LDS_PEAK * t,
         "FETCH_SIZE": 1e5, "WRITE_SIZE": 2e5}
    fr = bench.resource_fractions(c, t)
    assert fr["valu"]["frac"] == 0.5 and fr["lds"]["frac"] == 0.25
    assert fr["hbm"]["bytes"] == (2 * 1e5 + 2e5) * 1024
    assert abs(fr["hbm"]["frac"] - fr["hbm"]["bytes"] / t / 1e9 / bench.HBM_PEAK_GBS) < 1e-4
    assert max(fr, key=lambda k: fr[k]["frac"]) == "valu"
