"""fishnet_amd — MI355X-native batched NNUE static evaluator for fishnet's
analysis path (HIP/CDNA4 kernels behind the C ABI in include/fnnue.h)."""
from .nnue import (  # noqa: F401
    Evaluator, FnnueError, MultiEvaluator, Net, device_count, partition_groups, game_children, game_positions, perft, pos_from_fen,
    pack_games, random_game, random_playouts, random_vpositions, selftest_mfma, synthesize_net,
    synthesize_variant_net, vpos_from_fen, game_vpositions, game_vchildren, vperft, random_vgame, random_vgames,
    game_end, END_NO_MOVES, END_CHECK, END_EXTINCT,
)
from ._native import (  # noqa: F401
    GROUP_CHAIN, GROUP_STAR, PLAYOUT_CHILDREN, PLAYOUT_FINAL, PLAYOUT_PLIES, VARIANT_ATOMIC, VARIANT_CRAZYHOUSE,
)
