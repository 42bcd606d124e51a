/* fnnue_backend.h — a batched static-evaluation backend with the shape of
 * fishnet's engine actor, above the evaluator ABI (fnnue.h).
 *
 * The reference sends every position of an acquired batch to a Stockfish
 * child over UCI, one position per round trip:
 *   stockfish::channel(exe, StockfishInit{nnue}, logger)
 *       -> (StockfishStub, StockfishActor)          [ref] src/stockfish.rs:23-38
 *   StockfishStub::go(Position)
 *       -> Result<PositionResponse, PositionFailed> [ref] src/stockfish.rs:44-54
 * with Position / PositionResponse / PositionFailed from src/ipc.rs:16-41,
 * 100-103, and the batch expanded by IncomingBatch::from_acquired
 * (src/queue.rs:518-627) from an AcquireResponseBody (src/api.rs:293-309).
 *
 * Here the same pair is a channel to one evaluator per net on one GPU: the
 * actor owns an fnnue_ctx per net (chess, and optionally the crazyhouse and
 * atomic Fairy-Stockfish variant nets); a go() hands it whole acquired
 * batches, which it answers on the calling thread, one call at a time (a
 * second caller waits, as on the reference's mpsc::channel(1)), returning
 * one response per position.
 * Each batch goes to the net of its variant (the reference picks the engine
 * by EngineFlavor, src/queue.rs:530-539, and the variant, src/assets.rs:
 * 384-391).  The expansion (FEN parse, UCI replay, every ply) runs on the
 * device (fnnue_build_batch_device / fnnue_build_vbatch_device), the plies are
 * evaluated incrementally along each game (CHAIN groups), and the two raw NNUE
 * terms become a Score::Cp.  A batch that fails (unparsable FEN, illegal move,
 * a variant this backend has no net for) gets its own nonzero code in
 * batch_rc — PositionFailed{batch_id} (queue.rs:207-213 drops that batch) —
 * while the other batches of the call complete.  A nonzero return of go()
 * itself (device failure) fails them all.
 *
 * Score (static evaluation; search is outside this path):
 *   v  = (psqt + positional) / 16            Stockfish's NNUE value (internal
 *                                             units, side to move, C division;
 *                                             upstream evaluate_nnue.cpp with
 *                                             adjusted = false — the "NNUE
 *                                             evaluation" the `eval` command
 *                                             prints)
 *   cp = v * 100 / normalize_to_pawn         UCI::value's normalisation (upstream
 *                                             uci.cpp; 361 in SF 15.1 as recalled,
 *                                             a parameter because it is unpinned)
 * Analysis work: one response per ply, depth 0, nodes 1, no pv / best move.
 * A position with no legal move (it can only be a game's last ply) is
 * answered as the engine answers it — `info depth 0 score mate 0` when the
 * side to move is checkmated (atomic: its king exploded), `score cp 0` when
 * stalemated, `bestmove (none)` (src/stockfish.rs:359-376, 418-425): score
 * Mate(0) / Cp(0), depth 0, nodes 0, no best move; psqt / positional still
 * carry the NNUE terms ((0, 0) for an exploded king).
 * Move work: the root after all moves; a one-ply search over its legal
 * children: a child that mates (checkmate, atomic explosion of the other
 * king) is chosen first (score Mate(1)), a stalemating child is worth 0, every
 * other child -v(child) from its NNUE evaluation; the first maximum is the
 * best move (depth 1, nodes = children).  A root with no legal move: no best
 * move, Mate(0) / Cp(0), depth 0, nodes 0.
 */
#ifndef FNNUE_BACKEND_H
#define FNNUE_BACKEND_H

#include "fnnue.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FNNUE_WORK_ANALYSIS 0 /* Work::Analysis (api.rs:130-143) */
#define FNNUE_WORK_MOVE 1     /* Work::Move (api.rs:144-151) */

#define FNNUE_SCORE_CP 0      /* Score::Cp (api.rs:383-388) */
#define FNNUE_SCORE_MATE 1    /* Score::Mate */

typedef struct fnnue_backend fnnue_backend;

/* StockfishInit (stockfish.rs): what the engine is configured with. */
typedef struct {
  int32_t normalize_to_pawn; /* cp = v * 100 / normalize_to_pawn; 0 -> 361 */
  uint32_t timeout_ms;       /* budget of one go(): 0 -> 60000, the worker's cap min(60 s, budget)
                                ([ref] src/main.rs:316); see fnnue_backend_go_timeout */
} fnnue_backend_init;

/* AcquireResponseBody (api.rs:293-309) of one batch. */
typedef struct {
  const char *batch_id;            /* Work::id (BatchId), copied into logs / errors */
  int work;                        /* FNNUE_WORK_* */
  int multipv;                     /* Work::Analysis multipv: 0 = None; >= 1 = Some(k): the response is the
                                      matrix form (AnalysisPart::Matrix, Work::matrix_wanted, api.rs:179-187)
                                      with its one line (static eval has no second PV) at depth 0 */
  const char *position;            /* root FEN (X-FEN / Shredder castling accepted) */
  const char *variant;             /* "standard", "chess960", "fromPosition", NULL / "" = standard;
                                      "crazyhouse", "atomic" (variant nets); anything else: FNNUE_E_ARCH */
  const char *moves;               /* space-separated UCI (Chess960 king-takes-rook accepted) */
  const uint32_t *skip_positions;  /* skipPositions: position ids answered as Skipped */
  size_t nskip;
} fnnue_acquired;

/* PositionResponse (ipc.rs:28-39) of one position (Skip::Skip when skipped). */
typedef struct {
  uint32_t position_id;  /* PositionId: 0 = root, k = after k moves */
  uint8_t skipped;       /* 1: Skip::Skip (AnalysisPart::Skipped) */
  uint8_t score_kind;    /* FNNUE_SCORE_* */
  uint8_t depth;
  uint8_t matrix;        /* 1: serialise as AnalysisPart::Matrix (multipv requested) */
  int64_t score;         /* centipawns (side to move) */
  int32_t psqt;          /* the raw NNUE terms the score came from */
  int32_t positional;
  uint64_t nodes;
  uint64_t time_ms;      /* wall time of the go() call until this position's piece was back on the host */
  uint32_t nps;          /* positions evaluated by then, per second */
  char best_move[8];     /* UCI, NUL-terminated; "" for analysis */
} fnnue_position_response;

/* The nets of one backend, by the batches they evaluate.  Any may be NULL
 * (not all); a batch whose variant has no net fails with FNNUE_E_ARCH. */
typedef struct {
  const fnnue_net *chess;      /* standard / chess960 / fromPosition: a HalfKAv2_hm net */
  const fnnue_net *crazyhouse; /* a FNNUE_VARIANT_CRAZYHOUSE net (fnnue_net_load_variant) */
  const fnnue_net *atomic;     /* a FNNUE_VARIANT_ATOMIC net */
} fnnue_backend_nets;

/* stockfish::channel: starts the actor (one evaluator per net on `device`, a
 * few host threads for the per-batch loops of large calls).  A net in the
 * wrong slot: FNNUE_E_ARCH.  init may be NULL (defaults).  The nets may be
 * freed after the call. */
int fnnue_backend_channel_nets(const fnnue_backend_nets *nets, int device, const fnnue_backend_init *init,
                               fnnue_backend **out);
/* The one-net form: the net goes to the slot of its variant. */
int fnnue_backend_channel(const fnnue_net *net, int device, const fnnue_backend_init *init, fnnue_backend **out);
/* Stops the actor (after the call in flight) and frees it.  Never waits for
 * the device: when a timed-out call's work is still running on the channel's
 * streams, its buffers are released later (by a later channel() or free()),
 * once the streams have drained. */
void fnnue_backend_free(fnnue_backend *b);

/* Number of responses batch `a` expands to (IncomingBatch::from_acquired):
 * analysis = moves + 1, move = 1.  Host only; FNNUE_E_ARG on a bad work type. */
int fnnue_backend_batch_size(const fnnue_acquired *a, size_t *n);

/* StockfishStub::go for whole batches.  Batch i's responses land in
 * out[off[i] .. off[i + 1]) (off: nbatches + 1 entries, filled here; cap =
 * capacity of out, FNNUE_E_CAPACITY when too small); batch_rc[i] = 0 or the
 * FNNUE_E_* code of its PositionFailed (its responses then are unspecified).
 * Thread-safe: concurrent callers queue on the capacity-1 channel. */
int fnnue_backend_go(fnnue_backend *b, const fnnue_acquired *batches, size_t nbatches, fnnue_position_response *out,
                     size_t cap, uint32_t *off, int32_t *batch_rc);

/* go() with its own budget (timeout_ms; 0 = the channel's init.timeout_ms).
 * The reference worker races each go against `min(60 s, budget) +
 * work.timeout()` and, when it runs out, drops the engine (the child is
 * killed) and fails the batch ([ref] src/main.rs:316, 343-351;
 * src/stockfish.rs:138).  Here every wait of the call is bounded by that
 * deadline; on expiry the call returns FNNUE_E_TIMEOUT at once, without
 * waiting for the device: batch_rc[i] = 0 for the batches whose responses were
 * written before the deadline (valid), FNNUE_E_TIMEOUT for the others.  The
 * channel is then broken — the device may still be working in its buffers —
 * and every later go() on it fails fast with FNNUE_E_TIMEOUT; free it and open
 * a new channel (the worker's drop-and-restart). */
int fnnue_backend_go_timeout(fnnue_backend *b, const fnnue_acquired *batches, size_t nbatches,
                             fnnue_position_response *out, size_t cap, uint32_t *off, int32_t *batch_rc,
                             uint32_t timeout_ms);

/* The compact form of a go()'s answer (16 B per position instead of 56, and
 * what is the same for all of a batch's positions once per batch): what a
 * caller that builds its own response objects needs — fishnet's actor builds
 * PositionResponse (ipc.rs:28-39) in Rust memory anyway, so the 56-byte C
 * record is an intermediate it need not pay for.  Same semantics as
 * fnnue_position_response field by field:
 *   nodes     = 0 when flags has FNNUE_COMPACT_SKIPPED or FNNUE_COMPACT_NO_MOVES,
 *               else 1 for an analysis position, fnnue_batch_compact.nodes for
 *               the answer of a move batch;
 *   best_move = fnnue_batch_compact.best_move (move work), else none;
 *   time_ms / nps = the batch's (every position of a batch gets its piece's).
 * score is 32-bit: exact for normalize_to_pawn >= 13 (|psqt + positional| <
 * 2^32), which the compact call requires. */
#define FNNUE_COMPACT_SKIPPED 1   /* Skip::Skip: nothing else set */
#define FNNUE_COMPACT_MATRIX 2    /* serialise as AnalysisPart::Matrix */
#define FNNUE_COMPACT_NO_MOVES 4  /* a position without a legal move: mate 0 / cp 0, nodes 0, depth 0 */
typedef struct {
  int32_t psqt;
  int32_t positional;
  int32_t score;         /* centipawns or mate (score_kind), side to move */
  uint8_t score_kind;    /* FNNUE_SCORE_* */
  uint8_t depth;
  uint8_t flags;         /* FNNUE_COMPACT_* */
  uint8_t reserved;
} fnnue_position_compact;

typedef struct {
  uint64_t time_ms;      /* wall time of the go() call until the batch's piece was back on the host */
  uint32_t nps;          /* positions evaluated by then, per second */
  uint32_t nodes;        /* move work: the legal children searched (0 for a root without one); analysis: 0 */
  char best_move[8];     /* move work: UCI, NUL-terminated; "" otherwise */
} fnnue_batch_compact;

/* go() answering in the compact form: batch i's positions in out[off[i] ..
 * off[i + 1]) (cap = capacity of out), its per-batch part in bout[i]; budget
 * and errors as fnnue_backend_go_timeout.  FNNUE_E_ARG when the channel's
 * normalize_to_pawn is below 13. */
int fnnue_backend_go_compact(fnnue_backend *b, const fnnue_acquired *batches, size_t nbatches,
                             fnnue_position_compact *out, size_t cap, fnnue_batch_compact *bout, uint32_t *off,
                             int32_t *batch_rc, uint32_t timeout_ms);

/* Where the last go() spent its time (diagnostics; the reference's engine
 * reports only time / nps per position).  Each net's games are cut into pieces
 * of about FNNUE_BACKEND_PIECE_PLIES plies (default 524288); a piece is one
 * host-to-device copy, the replay, the evaluation kernels and one device-to-
 * host copy of its results (plus the evaluator's error word), in order on the
 * net's stream; the host stages the next pieces and writes a piece's
 * responses while the device works on the later ones, in the order the
 * pieces come back (another net's may be written first), blocking only when
 * a single net is left. */
typedef struct {
  double prep_ms;         /* host: sizes, move-work roots, text staging, copies and kernels enqueued */
  double device_ms;       /* host waiting for the device (blocked, or polling the nets' pieces) */
  double fill_ms;         /* responses written (overlaps the device's later pieces) */
  double total_ms;
  uint64_t positions;     /* positions evaluated (analysis plies + move-work children) */
  uint32_t stream_syncs;  /* host blocking waits on an event, a stream or a copy */
  uint32_t rebuilds;      /* extra passes after a batch failed (per failed batch, its piece only) */
  uint32_t host_threads;  /* threads for the staging / fill loops (FNNUE_BACKEND_THREADS; default: the usable CPUs, at most 8) */
  uint32_t pieces;        /* pieces over all nets */
} fnnue_backend_stats;

int fnnue_backend_last_stats(fnnue_backend *b, fnnue_backend_stats *out);

/* The `analysis` array fishnet submits for one analysis batch
 * (CompletedBatch::into_analysis, queue.rs:715-727; AnalysisPart / Score
 * serialisation, api.rs:355-388): {"skipped":true} or {"score":{"cp":..},
 * "depth":..,"nodes":..,"time":..,"nps":..} per position, or for a MultiPV
 * batch the matrix form {"pv":[[[]]],"score":[[{"cp":..}]],"depth":0,...}
 * (Matrix::set(multipv 1, depth 0): one row, one column), as JSON.  Writes
 * at most cap bytes including the NUL; *len = the full length (without NUL);
 * FNNUE_E_CAPACITY when it did not fit. */
int fnnue_backend_analysis_json(const fnnue_position_response *r, size_t n, char *buf, size_t cap, size_t *len);

#ifdef __cplusplus
}
#endif
#endif
