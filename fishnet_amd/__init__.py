"""fishnet_amd — MI355X-native batched NNUE static evaluator for fishnet's
analysis path (HIP/CDNA4 kernels behind the C ABI in include/fnnue.h)."""
from .nnue import (  # noqa: F401
    Evaluator, FnnueError, MultiEvaluator, Net, device_count, partition_groups, game_children, game_positions, perft, pos_from_fen,
    pack_games, random_game, random_playouts, selftest_mfma, synthesize_net,
)
from ._native import GROUP_CHAIN, GROUP_STAR, PLAYOUT_CHILDREN, PLAYOUT_FINAL, PLAYOUT_PLIES  # noqa: F401
