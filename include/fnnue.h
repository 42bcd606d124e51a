/*
 * fnnue.h — C ABI of the MI355X batched NNUE evaluator (libfnnue.so).
 *
 * This is the drop-in boundary for fishnet's static-evaluation path.  The
 * reference has no FFI for NNUE: it drives a Stockfish child over UCI text
 * pipes.  Each entry point below names the reference interface it replaces.
 *
 *   [ref] = /root/reference (schlawg/fishnet).  Upstream = Stockfish 15.1
 *   (submodule Stockfish/, empty in the reference checkout).
 *
 * Conventions
 *  - Every function returns FNNUE_OK (0) or a negative FNNUE_E_* code and then
 *    sets a thread-local message readable with fnnue_last_error().  No aborts,
 *    no exits.  On error no output is guaranteed (the caller maps any error to
 *    fishnet's PositionFailed{batch_id}, [ref] src/ipc.rs:100-103,
 *    src/queue.rs:207-213: the whole batch is dropped, never partial results).
 *  - Host buffers are owned by the caller; device memory of a ctx is owned by
 *    the library.  *_device entry points take device pointers and a hipStream_t
 *    (as void*), enqueue work and return without synchronising.
 *  - A fnnue_net is immutable and may be shared across threads; a fnnue_ctx
 *    must not be used from two threads at once (one ctx per GPU — the analogue
 *    of one engine per worker, [ref] src/main.rs:158-170).  Calls on one ctx
 *    share its device workspace: *_device calls on different streams are
 *    ordered by the library (a call on a new stream waits for the previous
 *    call's stream), so they serialise rather than race.
 *  - Outputs per position are the two raw Stockfish NNUE terms, before
 *    optimism / material scaling (upstream evaluate_nnue.cpp evaluate()):
 *      psqt       = (psqtAcc[stm][bucket] - psqtAcc[~stm][bucket]) / 2
 *      positional = Network[bucket].propagate(transformed features)
 *    Stockfish's NNUE value is (psqt + positional) / 16 (OutputScale).
 */
#ifndef FNNUE_H
#define FNNUE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FNNUE_OK 0
#define FNNUE_E_ARG (-1)        /* bad argument (null pointer, size, mode)           */
#define FNNUE_E_IO (-2)         /* file could not be read / written                   */
#define FNNUE_E_FORMAT (-3)     /* .nnue version / hash / truncated / trailing bytes  */
#define FNNUE_E_ARCH (-4)       /* architecture not supported (HD)                     */
#define FNNUE_E_DEVICE (-5)     /* HIP runtime error or no such device                */
#define FNNUE_E_POSITION (-6)   /* invalid position in a batch (kings, pieces, stm)   */
#define FNNUE_E_OOM (-7)        /* host or device allocation failed                    */
#define FNNUE_E_MOVE (-8)       /* illegal or unparsable UCI move                      */
#define FNNUE_E_FEN (-9)        /* unparsable FEN                                      */
#define FNNUE_E_CAPACITY (-10)  /* output buffer too small                             */
#define FNNUE_E_TIMEOUT (-11)   /* fnnue_backend_go overran its time budget           */

typedef struct fnnue_net fnnue_net; /* parsed, validated, immutable host copy of a .nnue */
typedef struct fnnue_ctx fnnue_ctx; /* one GPU: device-resident net + workspaces          */

/* Packed position, 36 bytes.  sq[s>>1] holds square s (A1=0..H8=63) in its low
 * nibble for even s and high nibble for odd s, as a Stockfish Piece code
 * (W_PAWN=1..W_KING=6, B_PAWN=9..B_KING=14, 0 = empty; upstream types.h).
 * stm: 0 = white, 1 = black.  Castling rights, en-passant square and move
 * counters do not enter the NNUE features and are not stored. */
typedef struct {
  uint8_t sq[32];
  uint8_t stm;
  uint8_t pad[3];
} fnnue_pos;

/* Packed position of a Fairy-Stockfish variant (48 bytes): the board and side
 * to move as fnnue_pos, then the pieces in hand (crazyhouse pockets): hand[0..4]
 * = white P N B R Q, hand[5..9] = black P N B R Q, each <= 16; all zero for
 * variants without pockets. */
typedef struct {
  uint8_t sq[32];
  uint8_t stm;
  uint8_t hand[10];
  uint8_t pad[5];
} fnnue_vpos;

/* ---- errors ---- */
const char *fnnue_last_error(void);
/* ABI version: (major << 16) | minor. */
uint32_t fnnue_abi_version(void);

/* ---- net loading ----
 * Replaces `setoption name EvalFile value <path>` sent to the engine
 * ([ref] src/stockfish.rs:209-211; path from src/assets.rs:128-133, 449-453;
 * upstream evaluate_nnue.cpp load_eval/read_parameters).  Accepts plain and
 * COMPRESSED_LEB128 tensors, checks version 0x7AF32F20, the structure hash
 * chain and exact EOF. */
int fnnue_net_load(const char *path, fnnue_net **out);
int fnnue_net_load_mem(const void *buf, size_t len, fnnue_net **out);
/* Net identity ([ref] build.rs:7 pins nn-ad9b42354671.nnue; build.rs:100-112
 * deletes a corrupt download): fnnue_net_load / fnnue_net_load_variant compute
 * the SHA-256 of the file, and when its basename is nn-<12 lowercase hex>.nnue
 * (upstream's naming: the first 12 hex digits of the digest) a mismatch fails
 * with FNNUE_E_FORMAT.  digest: 32 bytes (also for nets loaded from memory). */
int fnnue_net_sha256(const fnnue_net *net, uint8_t *digest);
/* hd = TransformedFeatureDimensions (1024 for nn-ad9b42354671, [ref] build.rs:7). */
int fnnue_net_info(const fnnue_net *net, uint32_t *hd, uint32_t *file_hash, const char **desc);
void fnnue_net_free(fnnue_net *net);

/* Deterministic synthetic net in the exact .nnue file format (the pinned net is
 * not shipped with the reference checkout).  flags: FNNUE_SYNTH_*.  The buffer
 * is allocated by the library; release it with fnnue_buffer_free. */
#define FNNUE_SYNTH_LEB128 1u     /* write tensors COMPRESSED_LEB128                  */
#define FNNUE_SYNTH_WRAP 2u       /* large FT weights: int16 accumulators wrap around */
#define FNNUE_SYNTH_FC1_PAD 4u    /* non-zero fc_1 padding weights (inputs 30,31)      */
int fnnue_net_synthesize(uint64_t seed, uint32_t hd, uint32_t flags, void **buf, size_t *len);
void fnnue_buffer_free(void *buf);

/* ---- Fairy-Stockfish variant nets (BASELINE config 5) ----
 * The reference routes every variant to Fairy-Stockfish ([ref]
 * src/queue.rs:530-539, src/assets.rs:384-391) and runs it with its classical
 * eval (`Use NNUE false`, src/stockfish.rs:248-260); these entry points are the
 * NNUE evaluation of such positions with Fairy-Stockfish's variant feature set
 * ("HalfKAv2 variants", 8x8 boards, 64 own-king squares, no mirroring; pocket
 * features for crazyhouse) in front of the SF 15.1 layer stacks.  Recalled,
 * not read: parity unpinned.  Same file format; the feature
 * transformer hash is 0x5F234CB8 ^ 2*HD; widths 256, 512, 1024. */
#define FNNUE_VARIANT_CHESS 0
#define FNNUE_VARIANT_CRAZYHOUSE 1 /* 64 x (704 board + 160 hand) features */
#define FNNUE_VARIANT_ATOMIC 2     /* 64 x 704 board features (also kingofthehill, racingkings) */
int fnnue_net_load_variant(const char *path, int variant, fnnue_net **out);
int fnnue_net_load_variant_mem(const void *buf, size_t len, int variant, fnnue_net **out);
int fnnue_net_variant(const fnnue_net *net, int *variant);
int fnnue_net_synthesize_variant(uint64_t seed, uint32_t hd, int variant, uint32_t flags, void **buf, size_t *len);
/* FEN (crazyhouse holdings as "[PNbq]" after the placement or as a 9th
 * placement field; "~" promotion marks ignored) -> packed variant position. */
int fnnue_vpos_from_fen(int variant, const char *fen, fnnue_vpos *out);
/* Test inputs: `count` seeded pseudo-legal random walks from the start
 * position (captures go to the capturer's hand and drops come back out for
 * crazyhouse; captures explode for atomic, kings never removed), up to
 * max_plies each.  FNNUE_PLAYOUT_FINAL: the last position of each walk;
 * FNNUE_PLAYOUT_PLIES: every position as CHAIN groups (off[], n_groups + 1). */
int fnnue_random_vpositions(uint64_t seed, int variant, size_t count, uint32_t max_plies, int mode, fnnue_vpos *out,
                            size_t cap, uint32_t *off, size_t off_cap, size_t *n_out, size_t *n_groups);
/* Variant games (the expansion of IncomingBatch::from_acquired for the
 * variants the reference sends to Fairy-Stockfish, [ref] src/queue.rs:524-552,
 * :530-539): crazyhouse FENs with holdings / promoted marks and UCI moves with
 * drops ("P@e4"), atomic captures with explosions; every move checked for
 * legality in its variant (shakmaty's Uci::to_move).  Host replay: the root and
 * the position after every move (n_moves + 1 records). */
int fnnue_game_vpositions(int variant, const char *fen, const char *moves, fnnue_vpos *out, size_t cap,
                          size_t *n_out);
/* Same plus every legal 1-ply child (drops included) of each position, as STAR
 * groups (off has n_groups + 1 entries). */
int fnnue_game_vchildren(int variant, const char *fen, const char *moves, fnnue_vpos *out, size_t cap, uint32_t *off,
                         size_t off_cap, size_t *n_out, size_t *n_groups);
/* perft of the variant move generator (known answers pin it). */
int fnnue_vperft(int variant, const char *fen, int depth, uint64_t *nodes);
/* Up to `plies` uniformly random legal moves (drops included) from `fen`, as
 * space-separated UCI; stops when no move is left or a king exploded. */
int fnnue_random_vgame(uint64_t seed, int variant, const char *fen, uint32_t plies, char *moves, size_t cap,
                       size_t *len);
/* Test / bench inputs: every ply of `count` seeded random LEGAL games of the
 * variant from its start position (L ~ U[0, max_plies] plies, drops included),
 * as CHAIN groups; a game ends early with no legal move or an exploded king
 * (that position is the game's last: see fnnue_eval_vpositions on game-over
 * records).  Deterministic for (seed, index). */
int fnnue_random_vgames(uint64_t seed, int variant, size_t count, uint32_t max_plies, int threads, fnnue_vpos *out,
                        size_t cap, uint32_t *off, size_t off_cap, size_t *n_out, size_t *n_groups);
/* The batch expansion on the device, as fnnue_build_batch[_device] (same text
 * layout, modes FNNUE_PLAYOUT_PLIES / _CHILDREN, sizes reported on
 * FNNUE_E_CAPACITY), for variant games; records are those of the host replay.
 * ctx supplies the device and stream (any net). */
int fnnue_build_vbatch_device(fnnue_ctx *ctx, int variant, const char *d_text, const uint32_t *d_fen_off,
                              const uint32_t *d_moves_off, size_t ngames, int mode, fnnue_vpos *d_out, size_t cap,
                              uint32_t *d_off, size_t off_cap, size_t *n_out, size_t *n_groups, void *stream);
int fnnue_build_vbatch(fnnue_ctx *ctx, int variant, const char *text, size_t text_len, const uint32_t *fen_off,
                       const uint32_t *moves_off, size_t ngames, int mode, fnnue_vpos *out, size_t cap, uint32_t *off,
                       size_t off_cap, size_t *n_out, size_t *n_groups);
/* Evaluation of variant positions on a context created from a variant net
 * (fnnue_ctx_create / fnnue_multi_create): the LDS-stationary feature
 * transformer over the variant tiles, then the MFMA layer stacks.
 * Game-over records: an atomic position with exactly one king (the other
 * exploded — how atomic games end, and every child that captures next to the
 * enemy king) has no NNUE evaluation; its result is psqt = positional = 0 and
 * it is not an error (the game's result is the caller's: fnnue_game_end,
 * the backend's mate 0).  Any other position without one king per side fails
 * the call with FNNUE_E_POSITION, the message naming its index. */
int fnnue_eval_vpositions(fnnue_ctx *ctx, const fnnue_vpos *pos, size_t n, int32_t *psqt, int32_t *positional);
int fnnue_eval_vpositions_device(fnnue_ctx *ctx, const fnnue_vpos *d_pos, size_t n, int32_t *d_psqt,
                                 int32_t *d_positional, void *stream);
/* Grouped variant evaluation with accumulator reuse, as fnnue_eval_groups[_device]
 * (FNNUE_GROUP_CHAIN: a game's plies, e.g. fnnue_build_vbatch's output;
 * FNNUE_GROUP_STAR: a parent and its children): each accumulator is derived
 * from the previous ply's / the parent's by the changed board and pocket
 * features (a crazyhouse capture adds the captured piece's hand row, a drop
 * removes one), refreshed when the perspective's king moved or more than two
 * features left or entered (atomic explosions).  Results are identical to
 * fnnue_eval_vpositions on the same positions. */
int fnnue_eval_vgroups(fnnue_ctx *ctx, const fnnue_vpos *pos, size_t npos, const uint32_t *off, size_t ngroups,
                       int mode, int32_t *psqt, int32_t *positional);
int fnnue_eval_vgroups_device(fnnue_ctx *ctx, const fnnue_vpos *d_pos, const uint32_t *d_off, size_t ngroups,
                              size_t npos, int mode, int32_t *d_psqt, int32_t *d_positional, void *stream);

/* ---- device context ----
 * Replaces spawning + initialising an engine process ([ref] src/stockfish.rs:
 * 132-153 spawn, 203-233 init).  Uploads the net to `device` (HIP ordinal). */
int fnnue_device_count(int *count);
int fnnue_ctx_create(const fnnue_net *net, int device, fnnue_ctx **out);
/* Device image of a net: one contiguous buffer, so rank 0 can RCCL-broadcast it
 * over xGMI and the other ranks adopt it (copied into ctx-owned memory). */
int fnnue_net_image_size(const fnnue_net *net, size_t *bytes);
int fnnue_net_image_pack(const fnnue_net *net, void *host_buf, size_t bytes);
int fnnue_ctx_create_from_image(int device, uint32_t hd, const void *device_image, size_t bytes, fnnue_ctx **out);
/* Pointer to the ctx's own device image (for broadcasting from rank 0). */
int fnnue_ctx_image(fnnue_ctx *ctx, const void **device_image, size_t *bytes);
void fnnue_ctx_free(fnnue_ctx *ctx);

/* ---- several GPUs from one process ----
 * The reference runs one engine per core ([ref] src/main.rs:156-170,
 * src/configure.rs:196-206: Cores::All = available_parallelism).  A
 * fnnue_multi owns one context per listed device: the net is uploaded once to
 * devices[0] and RCCL-broadcast over xGMI (ncclCommInitAll, one communicator
 * per device, this process); batches are sharded with no data-path
 * collective — contiguous position ranges, or whole groups balanced by
 * position count (fnnue_partition_groups) — and each device's results land in
 * its disjoint slice of the caller's buffers.  Same results as one context. */
typedef struct fnnue_multi fnnue_multi;
int fnnue_multi_create(const fnnue_net *net, const int *devices, int ndev, fnnue_multi **out);
void fnnue_multi_free(fnnue_multi *m);
int fnnue_multi_size(const fnnue_multi *m, int *ndev);
/* The context of device i (borrowed; owned by m). */
int fnnue_multi_ctx(fnnue_multi *m, int i, fnnue_ctx **ctx);
/* Host buffers, synchronous: one host thread per device (H2D, eval, D2H). */
int fnnue_multi_eval_positions(fnnue_multi *m, const fnnue_pos *pos, size_t n, int32_t *psqt, int32_t *positional);
int fnnue_multi_eval_groups(fnnue_multi *m, const fnnue_pos *pos, size_t npos, const uint32_t *off, size_t ngroups,
                            int mode, int32_t *psqt, int32_t *positional);
/* Device buffers: arrays of one pointer / count per device (device i's
 * buffers live on device i); device i's work is enqueued on streams[i] (a
 * hipStream_t of device i, as void*) or, when `streams` or streams[i] is NULL,
 * on its context's own stream, so the caller can order it after the work that
 * wrote the inputs (or synchronise first).  Returns without synchronising the
 * host, at any batch size.  fnnue_multi_sync waits for every device's
 * context work and reports latched errors (as fnnue_ctx_check). */
int fnnue_multi_eval_positions_device(fnnue_multi *m, const fnnue_pos *const *d_pos, const size_t *n,
                                      int32_t *const *d_psqt, int32_t *const *d_positional, void *const *streams);
int fnnue_multi_eval_groups_device(fnnue_multi *m, const fnnue_pos *const *d_pos, const uint32_t *const *d_off,
                                   const size_t *ngroups, const size_t *npos, int mode, int32_t *const *d_psqt,
                                   int32_t *const *d_positional, void *const *streams);
int fnnue_multi_sync(fnnue_multi *m);
/* Fairy-Stockfish variant positions over every device of a multi built from a
 * variant net (BASELINE config 5 on 8 GPUs): contiguous shards, as
 * fnnue_multi_eval_positions[_device]. */
int fnnue_multi_eval_vpositions(fnnue_multi *m, const fnnue_vpos *pos, size_t n, int32_t *psqt, int32_t *positional);
int fnnue_multi_eval_vpositions_device(fnnue_multi *m, const fnnue_vpos *const *d_pos, const size_t *n,
                                       int32_t *const *d_psqt, int32_t *const *d_positional, void *const *streams);
/* Grouped variant positions on every device (fnnue_eval_vgroups_device per
 * device, one shard of whole games each), as fnnue_multi_eval_groups_device. */
int fnnue_multi_eval_vgroups_device(fnnue_multi *m, const fnnue_vpos *const *d_pos, const uint32_t *const *d_off,
                                    const size_t *ngroups, const size_t *npos, int mode, int32_t *const *d_psqt,
                                    int32_t *const *d_positional, void *const *streams);
/* Splits groups off[0..ngroups] into nparts contiguous runs of whole groups
 * with about equal position counts: part k = groups [cut[k], cut[k+1]),
 * cut has nparts + 1 entries.  Host only. */
int fnnue_partition_groups(const uint32_t *off, size_t ngroups, int nparts, uint32_t *cut);

/* ---- evaluation, host buffers (synchronous) ----
 * Copies in, runs the device path, copies out.  Position validity is checked
 * on the device; an invalid position fails the whole call with
 * FNNUE_E_POSITION (message: its index) and no outputs are guaranteed.
 * Static eval of independent positions, accumulators from scratch.  Replaces
 * one `position fen ... ` + eval round trip per position ([ref]
 * src/stockfish.rs:274-283 / StockfishStub::go :44-54) with one batched call. */
int fnnue_eval_positions(fnnue_ctx *ctx, const fnnue_pos *pos, size_t n, int32_t *psqt, int32_t *positional);

/* Grouped evaluation with accumulator reuse.  Group g is pos[off[g] .. off[g+1]).
 *  FNNUE_GROUP_CHAIN: a game's plies in order; each accumulator is derived
 *    from the previous ply's (incremental add/sub of changed features, refresh
 *    on own-king moves) — upstream update_accumulator along the StateInfo chain.
 *    Feed it the expansion of an analysis batch ([ref] src/queue.rs:571-600).
 *  FNNUE_GROUP_STAR: pos[off[g]] is a parent, the rest are its children; each
 *    child is derived from the parent's accumulator.
 * Results are identical to fnnue_eval_positions on the same positions. */
#define FNNUE_GROUP_CHAIN 0
#define FNNUE_GROUP_STAR 1
/* pos holds npos positions; off has ngroups + 1 entries, off[0] = 0,
 * non-decreasing, off[ngroups] = npos (else FNNUE_E_ARG, nothing read past
 * pos[npos - 1]). */
int fnnue_eval_groups(fnnue_ctx *ctx, const fnnue_pos *pos, size_t npos, const uint32_t *off, size_t ngroups,
                      int mode, int32_t *psqt, int32_t *positional);

/* ---- evaluation, device buffers (asynchronous on `stream`, a hipStream_t) ----
 * Inputs already resident in HBM; results written to device memory.  Position
 * validity errors are latched on the device: call fnnue_ctx_check() after
 * synchronising to turn them into FNNUE_E_POSITION. */
int fnnue_eval_positions_device(fnnue_ctx *ctx, const fnnue_pos *d_pos, size_t n, int32_t *d_psqt,
                                int32_t *d_positional, void *stream);
int fnnue_eval_groups_device(fnnue_ctx *ctx, const fnnue_pos *d_pos, const uint32_t *d_off, size_t ngroups,
                             size_t npos, int mode, int32_t *d_psqt, int32_t *d_positional, void *stream);
/* Big + small net over the same CHAIN / STAR batch (BASELINE config 3 "big +
 * small net"; later Stockfish's dual NNUE evaluates a small HalfKAv2_hm net
 * beside the big one on the same features): results identical to two
 * fnnue_eval_groups_device calls, but the plan (deltas, segments, feature
 * lists) is built once, in the big context's workspace, and the small net's
 * feature transformer and layer stacks run on the small context's stream
 * beside the big net's on `stream`.  Both contexts: chess nets on one device,
 * sliced feature transformer.  No host synchronisation. */
int fnnue_eval_groups_dual_device(fnnue_ctx *big, fnnue_ctx *small, const fnnue_pos *d_pos, const uint32_t *d_off,
                                  size_t ngroups, size_t npos, int mode, int32_t *d_psqt, int32_t *d_positional,
                                  int32_t *d_psqt_small, int32_t *d_positional_small, void *stream);
/* Synchronises the ctx's device and reports (and clears) latched errors. */
int fnnue_ctx_check(fnnue_ctx *ctx);

/* ---- batch building (host) ----
 * FEN -> packed position.  Accepts standard, X-FEN and Shredder-FEN castling. */
int fnnue_pos_from_fen(const char *fen, fnnue_pos *out);
/* Every position of a game: the root and the position after each move, i.e.
 * the expansion of IncomingBatch::from_acquired for an analysis batch
 * ([ref] src/queue.rs:543-600; moves checked for legality like
 * Uci::to_move, :545).  `moves` is space-separated UCI (standard or Chess960
 * castling).  Writes n_moves + 1 positions. */
int fnnue_game_positions(const char *fen, const char *moves, fnnue_pos *out, size_t cap, size_t *n_out);
/* Same, plus every legal 1-ply child of each position, as STAR groups:
 * out[off[g]] is ply g, followed by its children.  off has n_groups+1 entries. */
int fnnue_game_children(const char *fen, const char *moves, fnnue_pos *out, size_t cap, uint32_t *off,
                        size_t off_cap, size_t *n_out, size_t *n_groups);
/* Has the game ended on the board after `moves`?  *flags = FNNUE_END_*: no
 * legal move, the side to move's king attacked, its king exploded (atomic).
 * A position without a legal move is where the engine answers `score mate 0`
 * (checkmate / explosion) or `score cp 0` (stalemate) with `bestmove (none)`
 * ([ref] src/stockfish.rs:359-376).  variant: FNNUE_VARIANT_* (host replay). */
#define FNNUE_END_NO_MOVES 1
#define FNNUE_END_CHECK 2
#define FNNUE_END_EXTINCT 4
int fnnue_game_end(int variant, const char *fen, const char *moves, int *flags);
/* Seeded random playouts from the start position (splitmix64; L ~ U[min,max]
 * plies of uniformly random legal moves, stopping at mate, stalemate or the
 * 50-move rule).  Deterministic for a given (seed, index) regardless of threads.
 *  FNNUE_PLAYOUT_FINAL: out[i] = final position of playout i (n_out = count).
 *  FNNUE_PLAYOUT_PLIES: every ply of every playout as CHAIN groups.
 *  FNNUE_PLAYOUT_CHILDREN: every ply and its legal children as STAR groups.
 * For the grouped modes off[] receives group offsets (off_cap >= groups+1). */
#define FNNUE_PLAYOUT_FINAL 0
#define FNNUE_PLAYOUT_PLIES 1
#define FNNUE_PLAYOUT_CHILDREN 2
int fnnue_random_playouts(uint64_t seed, size_t count, uint32_t min_plies, uint32_t max_plies, int mode,
                          int threads, fnnue_pos *out, size_t cap, uint32_t *off, size_t off_cap, size_t *n_out,
                          size_t *n_groups);
/* perft node count (board-code self test against published known answers). */
int fnnue_perft(const char *fen, int depth, uint64_t *nodes);

/* ---- batch building on the device ----
 * The batch expansion of fnnue_game_positions / fnnue_game_children for a
 * whole batch at once, on the GPU (FEN parse, UCI replay with Chess960
 * castling / en passant / promotion, legal children): replaces the
 * per-game host loop of IncomingBatch::from_acquired ([ref] src/queue.rs:
 * 518-627; wire format src/api.rs:293-309) and produces the positions where
 * the evaluator reads them.  Results are record for record those of the host
 * builder.
 * d_text (device memory): game g's FEN in [fen_off[g], moves_off[g]) and its
 * space-separated UCI moves in [moves_off[g], fen_off[g + 1]); d_fen_off has
 * ngames + 1 entries, d_moves_off ngames (both device memory).
 *  FNNUE_PLAYOUT_PLIES: every ply of every game; group g = game g (CHAIN).
 *  FNNUE_PLAYOUT_CHILDREN: one STAR group per ply: the ply, then its legal
 *    children in generation order.
 * Synchronous on `stream` (sizes are read back).  *n_out / *n_groups are set
 * even when the call fails with FNNUE_E_CAPACITY (retry with bigger buffers);
 * FNNUE_E_FEN / FNNUE_E_MOVE name the first failing game and ply. */
int fnnue_build_batch_device(fnnue_ctx *ctx, const char *d_text, const uint32_t *d_fen_off,
                             const uint32_t *d_moves_off, size_t ngames, int mode, fnnue_pos *d_out, size_t cap,
                             uint32_t *d_off, size_t off_cap, size_t *n_out, size_t *n_groups, void *stream);
/* Same with host buffers (staged through the ctx's stream). */
int fnnue_build_batch(fnnue_ctx *ctx, const char *text, size_t text_len, const uint32_t *fen_off,
                      const uint32_t *moves_off, size_t ngames, int mode, fnnue_pos *out, size_t cap, uint32_t *off,
                      size_t off_cap, size_t *n_out, size_t *n_groups);
/* perft on the device (depth <= 3 per thread; shallower levels expanded on
 * the host): pins the device move generator on published counts. */
int fnnue_perft_device(fnnue_ctx *ctx, const char *fen, int depth, uint64_t *nodes);
/* A random legal game from `fen`: up to `plies` uniformly random legal moves
 * (splitmix64 seed), space-separated UCI (Chess960 notation when the position
 * needs it), NUL-terminated; *len = string length.  Test-input generator. */
int fnnue_random_game(uint64_t seed, const char *fen, uint32_t plies, char *moves, size_t cap, size_t *len);

/* ---- diagnostics ----
 * Runs the int8 MFMA operand-layout self test on `device`; 0 if the hardware
 * layout matches the kernels' assumption. */
int fnnue_selftest_mfma(int device);
/* Feature-transformer implementation for fnnue_eval_positions*:
 *  FNNUE_FT_SLICED: LDS-stationary weight tiles, positions planned and sorted
 *    on the device; for fnnue_eval_groups*, the incremental
 *    updates run on the same tiles (segments of positions that share the
 *    perspective's king square).
 *  FNNUE_FT_GATHER: one wave per position (groups: per group) gathering rows
 *    from L2/HBM.
 *  FNNUE_FT_AUTO (default): chess positions calls of at most
 *    FNNUE_FT_GATHER_MAX positions gather (the sliced plan and its tile loads
 *    are a fixed ~60-80 us that a small call does not amortise: move work's
 *    children, a few games' positions), larger ones and every grouped call
 *    run sliced.
 * All are bit-identical; the environment variable FNNUE_FT_IMPL=
 * gather|sliced|auto sets the default for new contexts. */
#define FNNUE_FT_SLICED 0
#define FNNUE_FT_GATHER 1
#define FNNUE_FT_AUTO 2
#define FNNUE_FT_GATHER_MAX 16384
int fnnue_ctx_set_ft_impl(fnnue_ctx *ctx, int impl);
/* SWAR row sums in the sliced feature transformer: pairs of int16 columns
 * summed as 32-bit words.  Exact whenever no reachable
 * accumulator's even column leaves int16 range; the library checks that from
 * the weights (fnnue_net_accumulator_bound < 32768) and turns SWAR on by
 * itself (FNNUE_SWAR=0 in the environment keeps it off).  Results are
 * identical either way; set_swar(1) fails with FNNUE_E_ARCH on a net whose
 * bound does not allow it. */
int fnnue_net_accumulator_bound(const fnnue_net *net, int32_t *bound);
int fnnue_ctx_swar(const fnnue_ctx *ctx, int *enabled, int32_t *bound);
int fnnue_ctx_set_swar(fnnue_ctx *ctx, int enable);

/* Kernel timing with HIP events on the launch stream: when enabled, every
 * chunk launched by a *_device call records events around the feature-
 * transformer kernel and the layer-stack kernel.  fnnue_ctx_timing_read
 * synchronises on the last event, returns the number of timed launches and the
 * summed kernel times (ms), and resets the accumulators.
 * enable: FNNUE_TIMING_OFF (0), FNNUE_TIMING_ALL (1, any other non-zero value:
 * four events per chunk, plan / FT kernel / stacks), FNNUE_TIMING_FT (2: only
 * the two events around the FT main kernel; plan and stack times read 0).  An
 * event record between two kernels costs the stream a few microseconds, so a
 * throughput measurement times with FNNUE_TIMING_FT. */
#define FNNUE_TIMING_OFF 0
#define FNNUE_TIMING_ALL 1
#define FNNUE_TIMING_FT 2
int fnnue_ctx_set_timing(fnnue_ctx *ctx, int enable);
int fnnue_ctx_timing_read(fnnue_ctx *ctx, uint32_t *launches, double *ft_ms, double *stack_ms);
/* Same, split into the FT plan kernels, the FT main kernel (ft_slices /
 * ft_segments / ft_scratch / ft_groups) and the layer stacks. */
int fnnue_ctx_timing_phases(fnnue_ctx *ctx, uint32_t *launches, double *plan_ms, double *ft_ms, double *stack_ms);

#ifdef __cplusplus
}
#endif
#endif /* FNNUE_H */
