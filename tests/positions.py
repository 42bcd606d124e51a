"""Shared position sets for the tests (FENs exercising castling, en passant,
promotion, Chess960 and every king bucket / piece-count bucket)."""

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
KIWIPETE = "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1"
POS3 = "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1"
POS4 = "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1"
POS5 = "rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8"
CHESS960 = "bqnb1rkr/pp3ppp/3ppn2/2p5/5P2/P2P4/NPP1P1PP/BQ1BNRKR w HFhf - 2 9"

FENS = [
    START, KIWIPETE, POS3, POS4, POS5, CHESS960,
    "4k3/8/8/8/8/8/8/4K3 w - - 0 1",          # bare kings: bucket 0
    "7k/8/8/8/8/8/8/K7 b - - 0 1",
    "k7/8/8/8/8/8/8/7K w - - 0 1",
    "8/8/8/3k4/8/8/8/R3K2R b KQ - 0 1",
    "rnbqkbnr/ppp1p1pp/8/3pPp2/8/8/PPPP1PPP/RNBQKBNR w KQkq f6 0 3",
    "8/P6k/8/8/8/8/6Kp/8 w - - 0 1",
    "r1bqk2r/pppp1ppp/2n2n2/2b1p3/2B1P3/3P1N2/PPP2PPP/RNBQK2R w KQkq - 1 5",
]

# perft known answers (published)
PERFT = [
    (START, [20, 400, 8902, 197281]),
    (KIWIPETE, [48, 2039, 97862]),
    (POS3, [14, 191, 2812, 43238]),
    (POS4, [6, 264, 9467]),
    (POS5, [44, 1486, 62379]),
]
