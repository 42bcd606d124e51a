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
