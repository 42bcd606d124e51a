// backend.cpp — fnnue_backend (include/fnnue_backend.h): fishnet's engine
// actor shape over the evaluator.  The reference's pair
//   stockfish::channel -> (StockfishStub, StockfishActor)   [ref] src/stockfish.rs:23-61
// is a bounded mpsc channel (capacity 1) into an actor owning one engine
// process; StockfishStub::go sends a Position with a oneshot callback and
// maps any failure to PositionFailed{batch_id}.  Here the actor owns one
// fnnue_ctx per net (chess, and optionally the crazyhouse and atomic variant
// nets) and answers one message at a time on the caller's thread (a second
// caller waits: the capacity-1 channel); a message carries whole acquired batches
// (AcquireResponseBody, [ref] src/api.rs:293-309), expanded the way
// IncomingBatch::from_acquired does ([ref] src/queue.rs:518-627) — but on the
// device: the FEN/UCI text goes to HBM once, the builder replays every game
// there and the plies are evaluated incrementally along each game.
//
// One go(), per net: the host counts each batch's plies (it must: the
// response offsets are part of the answer) and cuts the games into pieces;
// per piece it stages the text, offsets (and, in the last piece, the
// move-work children) in a pinned image and sends it with one copy; the
// context's stream runs the replay (one wave per game), the CHAIN evaluation
// and the children's evaluation, and one copy brings back the builder's error
// word, the game-end flags and every (psqt, positional).  The nets' streams
// run side by side, and the host stages the next pieces and writes a piece's
// responses while the device works on the later ones.  Buffers are grow-only
// (device and pinned host), so a steady stream of calls allocates nothing.  A
// failed batch costs a second pass for its piece only.  Large calls spread the
// host work (text staging, response fill) over a few threads.
#include "../../include/fnnue_backend.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <emmintrin.h>
#include <sched.h>
#include <vector>

#include "board.h"
#include "builder.h"
#include "internal.h"
#include "text_scan.h"
#include "vboard.h"
#include "workers.h"

using namespace fnnue;
using namespace fnnue::detail;

namespace {

constexpr int32_t kNormalizeToPawnSf151 = 361;  // upstream uci.h NormalizeToPawnValue (SF 15.1, recalled)
constexpr int kKinds = 3;                       // net slots: kVariantChess, kVariantCrazyhouse, kVariantAtomic
constexpr uint32_t kDefaultTimeoutMs = 60000;
// Per-batch text bounds: far beyond any lichess batch (a FEN is < 100 bytes;
// the longest possible game, ~5,900 moves, < 64 KB of UCI), so that a piece's
// text fits its 32-bit offsets whatever the caller sends.
constexpr size_t kMaxFenBytes = 4096, kMaxMovesBytes = (size_t)1 << 22;
constexpr size_t kMaxPieceText = (size_t)1 << 30;  // a new piece before a piece's text passes this   // the worker's budget cap, min(60 s, budget) ([ref] src/main.rs:316)
using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// One message on the channel: StockfishMessage::Go with its answer.
struct Job {
  const fnnue_acquired* batches = nullptr;
  size_t nb = 0;
  fnnue_position_response* out = nullptr;    // the full records, or
  fnnue_position_compact* cout = nullptr;    // the compact form (fnnue_backend_go_compact) with
  fnnue_batch_compact* bout = nullptr;       // its per-batch part
  size_t cap = 0;
  uint32_t* off = nullptr;
  int32_t* rc = nullptr;
  uint32_t timeout_ms = 0;  // the call's budget (0: the channel's)
  int ret = 0;
  std::string err;  // fnnue_last_error of a failed call
};

// Grow-only device buffer.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int reserve(size_t want) {
    if (want <= bytes) return FNNUE_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    want = want + want / 4 + 256;
    if (hipMalloc(&p, want) != hipSuccess) return fail(FNNUE_E_OOM, "backend device buffer");
    bytes = want;
    return FNNUE_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* at(size_t off) const {
    return reinterpret_cast<T*>(static_cast<char*>(p) + off);
  }
};

// Grow-only pinned host buffer (the DMA engines read / write it directly, so
// the copies are asynchronous and need no staging through pageable memory).
struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int reserve(size_t want) {
    if (want <= bytes) return FNNUE_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    want = want + want / 4 + 4096;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return fail(FNNUE_E_OOM, "backend pinned buffer");
    bytes = want;
    return FNNUE_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* at(size_t off) const {
    return reinterpret_cast<T*>(static_cast<char*>(p) + off);
  }
};

size_t count_moves(const char* s) {
  size_t len = 0;
  return s ? scan_tokens(s, &len) : 0;
}

int64_t to_cp(int32_t psqt, int32_t positional, int32_t norm) {
  const int64_t v = ((int64_t)psqt + positional) / 16;  // OutputScale, C truncation
  return v * 100 / norm;
}

// A root with no legal move: the engine prints `info depth 0 score mate 0`
// (checkmated; atomic: its king exploded) or `score cp 0` (stalemate) and
// `bestmove (none)` ([ref] src/stockfish.rs:359-376, 418-425: Score::Mate(0)
// / Score::Cp(0), best_move None, nodes 0).
void terminal_response(fnnue_position_response& r, uint8_t fin) {
  r.score_kind = (fin & (kFinalCheck | kFinalExtinct)) ? FNNUE_SCORE_MATE : FNNUE_SCORE_CP;
  r.score = 0;
  r.depth = 0;
  r.nodes = 0;
  r.best_move[0] = 0;
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// A full response written in place as four stores — bytes 0-15 (position id,
// the four flag bytes, score), 16-31 (psqt, positional, nodes), 32-47 and
// 48-55 (time, nps, best move: the same for a whole piece of analysis plies)
// — instead of a memset and a store per field: the fill is bound by the
// stores into the caller's buffer.
static_assert(offsetof(fnnue_position_response, skipped) == 4 && offsetof(fnnue_position_response, score) == 8 &&
                  offsetof(fnnue_position_response, psqt) == 16 && offsetof(fnnue_position_response, nodes) == 24 &&
                  offsetof(fnnue_position_response, time_ms) == 32 && offsetof(fnnue_position_response, nps) == 40 &&
                  offsetof(fnnue_position_response, best_move) == 44 && sizeof(fnnue_position_response) == 56,
              "fnnue_position_response layout");
static_assert(sizeof(fnnue_position_compact) == 16 && sizeof(fnnue_batch_compact) == 24, "compact layouts");
struct ResponseTail {  // bytes 32-55 of an analysis response of one piece
  __m128i t32;
  uint64_t t48;
  ResponseTail(uint64_t ms, uint32_t nps) : t32(_mm_set_epi64x((long long)nps, (long long)ms)), t48(0) {}
};
inline uint64_t response_head(uint32_t id, uint8_t skipped, uint8_t kind, uint8_t depth, uint8_t matrix) {
  return id | (uint64_t)skipped << 32 | (uint64_t)kind << 40 | (uint64_t)depth << 48 | (uint64_t)matrix << 56;
}
inline void put_response(fnnue_position_response* r, uint64_t head, int64_t score, int32_t psqt, int32_t positional,
                         uint64_t nodes, const ResponseTail& tail) {
  char* d = reinterpret_cast<char*>(r);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(d), _mm_set_epi64x((long long)score, (long long)head));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(d + 16),
                   _mm_set_epi64x((long long)nodes, (long long)((uint64_t)(uint32_t)psqt | (uint64_t)(uint32_t)positional << 32)));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(d + 32), tail.t32);
  std::memcpy(d + 48, &tail.t48, 8);
}
inline void put_compact(fnnue_position_compact* r, int32_t psqt, int32_t positional, int32_t score, uint8_t kind,
                        uint8_t depth, uint8_t flags) {
  _mm_storeu_si128(reinterpret_cast<__m128i*>(r),
                   _mm_set_epi32((int)((uint32_t)kind | (uint32_t)depth << 8 | (uint32_t)flags << 16), score,
                                 positional, psqt));
}

// The net slot of a batch's variant (shakmaty Variant names, [ref]
// src/api.rs:304; logger.rs:194-201): standard chess (EngineFlavor::Official
// for analysis, queue.rs:530-539) and the two variants with a Fairy-Stockfish
// NNUE feature set here.  -1: a variant this backend does not evaluate
// (antichess, horde, kingOfTheHill, racingKings, threeCheck).
int kind_of(const char* v) {
  if (!v || !*v || !std::strcmp(v, "standard") || !std::strcmp(v, "chess960") || !std::strcmp(v, "fromPosition") ||
      !std::strcmp(v, "chess"))
    return kVariantChess;
  if (!std::strcmp(v, "crazyhouse")) return kVariantCrazyhouse;
  if (!std::strcmp(v, "atomic")) return kVariantAtomic;
  return -1;
}

// Host replay of a move batch's root (Work::Move: the position after all
// moves), with its legal children and their game-end flags.
struct MoveRoot {
  uint8_t fin = 0;                 // kFinal* of the root
  std::vector<std::string> uci;    // legal moves
  std::vector<uint8_t> kid_fin;    // kFinal* of each child
};

int chess_move_root(const fnnue_acquired& a, MoveRoot& R, std::vector<fnnue_pos>& kids) {
  Board b;
  std::string e;
  if (!board_from_fen(a.position ? a.position : "", b, &e)) return FNNUE_E_FEN;
  std::string tok;
  for (const char* p = a.moves ? a.moves : "";; ++p) {
    if (*p && *p != ' ' && *p != '\t' && *p != '\n' && *p != '\r') {
      tok += *p;
      continue;
    }
    if (!tok.empty()) {
      Move m;
      if (!parse_uci(b, tok.c_str(), m)) return FNNUE_E_MOVE;
      b.do_move(m);
      tok.clear();
    }
    if (!*p) break;
  }
  auto fin_of = [](const Board& x, bool any) {
    return (uint8_t)((any ? 0 : kFinalNoMoves) | (x.in_check() ? kFinalCheck : 0));
  };
  std::vector<Move> ms;
  b.legal_moves(ms);
  R.fin = fin_of(b, !ms.empty());
  kids.reserve(ms.size());
  for (const Move& m : ms) {
    Board k = b;
    k.do_move(m);
    kids.push_back(k.pack());
    R.uci.push_back(b.uci(m, b.chess960));
    R.kid_fin.push_back(fin_of(k, k.has_legal_move()));
  }
  return FNNUE_OK;
}

int variant_move_root(int variant, const fnnue_acquired& a, MoveRoot& R, std::vector<fnnue_vpos>& kids) {
  vb::VBoard b;
  const char* fen = a.position ? a.position : "";
  if (!vb::parse_fen(fen, 0, (uint32_t)std::strlen(fen), variant, b)) return FNNUE_E_FEN;
  const char* mv = a.moves ? a.moves : "";
  const uint32_t end = (uint32_t)std::strlen(mv);
  uint32_t p = 0, st;
  int len;
  while ((len = vb::next_token(mv, p, end, st)) > 0) {
    vb::VMove m;
    if (!vb::match_uci(b, mv + st, len, m)) return FNNUE_E_MOVE;
    vb::do_move(b, m);
  }
  R.fin = vb::final_state(b);
  vb::for_each_legal(b, [&](const vb::VMove& m) -> bool {
    vb::VBoard k = b;
    vb::do_move(k, m);
    kids.push_back(vb::pack(k));
    R.uci.push_back(vb::vuci(b, m));
    R.kid_fin.push_back(vb::final_state(k));
    return true;
  });
  return FNNUE_OK;
}

// One piece of a net's work: a run of its analysis games (the net's last piece
// also carries the move-work children), staged as one image
//   [text | fen_off | mv_off | ply_off | children | err (16 B) | fin | psqt | positional]
// at its own place in the net's buffers: the first five parts and the zeroed
// error words go up with one copy, the last four come back with one.  err
// words 0-2 are the builder's (code, game, ply), word 3 the evaluator's: the
// context's error word points there while the piece's evaluation is enqueued.
struct Piece {
  std::vector<size_t> games;  // analysis batches (job indices)
  bool kids = false;          // the net's move-work children ride in this piece
  uint32_t ng = 0, n = 0;     // games, plies
  size_t nk = 0;              // children
  size_t o_fen = 0, o_mv = 0, o_ply = 0, o_kids = 0, o_res = 0, o_fin = 0, o_ps = 0, o_po = 0, end = 0;
  size_t up0 = 0, down0 = 0, dev0 = 0, pos0 = 0;  // where the piece lives in the net's buffers
  bool pending = false;                           // evaluation enqueued, results not yet read
};

// One net's share of a go(): its analysis games cut into pieces of about
// piece_plies plies, and its move-work roots.  A piece's upload, replay,
// evaluation and download run on the context's stream, one piece after the
// other; the host stages the next pieces and writes a piece's responses while
// the device works on the later ones.  (The replay of the next piece on a
// stream of its own, beside this piece's evaluation, measured slower: its
// waves hold CU slots the evaluation's 1024-thread workgroups need.)
struct NetWork {
  std::vector<size_t> games;      // analysis batches (job indices)
  std::vector<size_t> roots;      // move batches whose roots have legal children
  std::vector<MoveRoot> mroots;   // their replayed roots
  std::vector<size_t> kid_first;  // first child of each root
  std::vector<uint8_t> kids;      // children records
  std::vector<size_t> terminal;   // move batches whose root has no legal move
  std::vector<MoveRoot> troots;
  std::vector<Piece> pieces;
  size_t nk = 0, rec = 0;
  size_t next = 0;                // first piece whose responses are not written yet
  std::vector<hipEvent_t> ev_done;  // per piece: results and error word on the host
  DevBuf dev, pos;
  PinnedBuf up, down, scratch;      // scratch: a failing piece's positions, read back by recover()
  void clear() {
    games.clear();
    roots.clear();
    mroots.clear();
    kid_first.clear();
    kids.clear();
    terminal.clear();
    troots.clear();
    pieces.clear();
    nk = 0;
    next = 0;
  }
  int events(size_t n) {
    while (ev_done.size() < n) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(FNNUE_E_DEVICE, "hipEventCreate");
      ev_done.push_back(e);
    }
    return FNNUE_OK;
  }
  void release() {
    dev.release();
    pos.release();
    up.release();
    down.release();
    scratch.release();
    for (hipEvent_t e : ev_done) (void)hipEventDestroy(e);
    ev_done.clear();
  }
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// CPUs this process may use: its affinity mask, capped by a cgroup v2 CPU
// quota (a container's share of a large host)
int usable_cpus() {
  int n = (int)std::max(1u, std::thread::hardware_concurrency());
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0)
      n = std::max(1, std::min(n, (int)((std::atol(quota) + period - 1) / period)));
    std::fclose(f);
  }
  return n;
}

}  // namespace

struct fnnue_backend;
namespace {
// Backends freed while a timed-out call's work was still on their streams
// (fnnue_backend_free): released here once the streams have drained.
std::mutex g_abandoned_mu;
std::vector<fnnue_backend*> g_abandoned;
void reap_abandoned();
}  // namespace

struct fnnue_backend {
  fnnue_ctx* ctx[kKinds] = {};  // one evaluator per net, all on one device
  int device = 0;
  int32_t norm = kNormalizeToPawnSf151;
  size_t piece_plies = 524288;  // FNNUE_BACKEND_PIECE_PLIES
  bool any_order = true;         // FNNUE_BACKEND_ANY_ORDER=0: wait for the nets' pieces in net order
  size_t tail_plies = 0;         // FNNUE_BACKEND_TAIL_PLIES: a net's last piece cut to about this many
  size_t fill_grain = 64;        // FNNUE_BACKEND_FILL_GRAIN: games per fill task
  size_t size_grain = 256;       // FNNUE_BACKEND_SIZE_GRAIN: batches per sizing task
  size_t stage_grain = 512;      // FNNUE_BACKEND_STAGE_GRAIN: games per text-staging task
  // The worker's time budget ([ref] src/main.rs:316, 343-351: a go() that
  // overruns it fails, and the engine is dropped — its child killed,
  // stockfish.rs:138).  Every wait of a go() is bounded by the call's
  // deadline; a call that overruns it returns FNNUE_E_TIMEOUT and breaks the
  // channel: the device may still be working on the call's pieces (in the
  // channel's buffers), so later calls fail fast and the caller opens a new
  // channel, as the worker restarts its engine.
  uint32_t timeout_ms = kDefaultTimeoutMs;
  bool broken = false;
  Clock::time_point deadline;
  // The capacity-1 channel: a go() runs on its caller's thread holding run_mu,
  // so a second caller waits until the first call is answered
  // (mpsc::channel(1) with one message in flight, without a thread hand-off
  // each way: ~10 µs of a one-batch call).
  std::mutex run_mu;
  bool closed = false;
  Workers pool;
  int pool_threads = 1;
  NetWork net[kKinds];
  std::vector<uint32_t> flen, mlen;  // per batch of the job in flight: FEN / moves text lengths
  std::vector<int8_t> kind;          // per batch: its net slot
  std::vector<uint8_t> bskip;        // per batch: has skipPositions
  std::vector<uint8_t> skip;         // per response of such a batch: skipped
  std::mutex stats_mu;
  fnnue_backend_stats stats{};
  // per go(): its clock, positions written so far, host time spent writing / waiting
  Clock::time_point t0;
  uint64_t filled = 0;
  double fill_ms = 0, wait_ms = 0;
  uint32_t syncs = 0, rebuilds = 0;
  // FNNUE_BACKEND_TRACE=1: each go() prints its host timeline (µs since the
  // call started) to stderr — diagnostics only
  bool trace = false;
  std::string tl;
  void mark(const char* what, int k = -1, long pi = -1) {
    if (!trace) return;
    char b[96];
    std::snprintf(b, sizeof(b), "%s[\"%s\",%d,%ld,%.1f]", tl.empty() ? "" : ",", what, k, pi, ms_since(t0) * 1e3);
    tl += b;
  }

  void run(Job& j);
  void release_device() {
    for (NetWork& W : net) W.release();
    for (fnnue_ctx*& c : ctx) {
      fnnue_ctx_free(c);
      c = nullptr;
    }
  }
  bool expired() const { return Clock::now() >= deadline; }
  int timed_out(const char* where);
  int wait_event(hipEvent_t e, const char* what);
  bool streams_idle();
  void abandon_unanswered(Job& j);
  void drain_streams();
  int prepare_moves(Job& j, int k);
  void layout(const Job& j, int k, Piece& P);
  int plan(Job& j, int k);
  int stage_up(Job& j, int k, size_t pi);
  int stage_eval(int k, size_t pi);
  int finish(Job& j, int k, bool wait, bool* ready);
  int recover(Job& j, int k, size_t pi);
  void fill(Job& j, int k, const Piece& P);
  void fill_roots(Job& j, int k, const Piece& P, uint64_t ms, uint32_t nps);
  void fill_hostonly(Job& j, const std::vector<size_t>& all_skipped);
};

int fnnue_backend::timed_out(const char* where) {
  return fail(FNNUE_E_TIMEOUT, std::string("go() overran its budget of ") + std::to_string(timeout_ms) +
                                   " ms (" + where + ", " + std::to_string(ms_since(t0)) + " ms in)");
}

// Waits for an event until the call's deadline: a few microseconds of
// spinning (a small call's piece is back within them), then the CPU is
// yielded between polls, so that a long wait does not hold a core the worker
// threads or the rest of fishnet could use.
int fnnue_backend::wait_event(hipEvent_t e, const char* what) {
  for (uint32_t i = 0;; ++i) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return FNNUE_OK;
    if (q != hipErrorNotReady) return hip_fail(q, what);
    if (expired()) return timed_out(what);
    if (i < 512) {
      for (int p = 0; p < 16; ++p) _mm_pause();
    } else {
      sched_yield();
    }
  }
}

// Nothing of the channel's is left on the device (its streams are drained).
bool fnnue_backend::streams_idle() {
  for (fnnue_ctx* c : ctx)
    if (c && hipStreamQuery(c->stream) == hipErrorNotReady) return false;
  return true;
}

// After a timeout: the batches whose responses were not written fail with
// FNNUE_E_TIMEOUT (those already written stand); the channel is broken.
void fnnue_backend::abandon_unanswered(Job& j) {
  for (NetWork& W : net) {
    for (size_t pi = W.next; pi < W.pieces.size(); ++pi)
      for (size_t i : W.pieces[pi].games) j.rc[i] = FNNUE_E_TIMEOUT;
    if (W.next < W.pieces.size())  // the move work rides in the net's last piece
      for (size_t i : W.roots) j.rc[i] = FNNUE_E_TIMEOUT;
  }
  broken = true;
}

// After an error other than the budget: the pinned images stay in use until
// the device's copies are done, so the streams are drained before the call
// returns — polled, and only until the call's deadline (a stuck device then
// breaks the channel instead of hanging the caller).
void fnnue_backend::drain_streams() {
  for (uint32_t i = 0; !streams_idle(); ++i) {
    if (expired()) {
      broken = true;
      return;
    }
    if (i < 512) {
      for (int p = 0; p < 16; ++p) _mm_pause();
    } else {
      sched_yield();
    }
  }
}

// Move batches of one net, host side: the position after all moves (one per
// batch) and its legal children with their game-end flags.  A batch whose
// root cannot be replayed fails alone; so does one with a child the
// evaluator would reject (e.g. a root with more than 32 pieces, a pocket
// beyond the variant's limits) — checked here, so that the device never
// latches an error for move work (one bad batch no longer fails
// the call).
// The roots are replayed on the pool's threads (each root ~40-70 us of host
// board work: its moves matched against the legal moves, then every child's
// legal moves for its game-end flags), then merged in batch order.
int fnnue_backend::prepare_moves(Job& j, int k) {
  NetWork& W = net[k];
  const bool chess = k == kVariantChess;
  const size_t nr = W.roots.size();
  std::vector<MoveRoot> R(nr);
  std::vector<std::vector<fnnue_pos>> kids(chess ? nr : 0);
  std::vector<std::vector<fnnue_vpos>> vkids(chess ? 0 : nr);
  std::vector<int> rcs(nr, FNNUE_OK);
  pool.run(nr, 1, [&](size_t lo, size_t hi) {
    for (size_t t = lo; t < hi; ++t) {
      const fnnue_acquired& a = j.batches[W.roots[t]];
      int rc = chess ? chess_move_root(a, R[t], kids[t]) : variant_move_root(k, a, R[t], vkids[t]);
      if (rc == FNNUE_OK && chess)
        for (const fnnue_pos& p : kids[t]) rc = rc ? rc : (valid_host_pos(p) ? 0 : (int)FNNUE_E_POSITION);
      if (rc == FNNUE_OK && !chess)
        for (const fnnue_vpos& p : vkids[t]) rc = rc ? rc : (host_vpos_state(p, k) ? 0 : (int)FNNUE_E_POSITION);
      rcs[t] = rc;
    }
  });
  std::vector<size_t> dev_roots;
  for (size_t t = 0; t < nr; ++t) {
    const size_t i = W.roots[t];
    if (rcs[t]) {
      j.rc[i] = rcs[t];
      continue;
    }
    if (R[t].uci.empty()) {
      W.terminal.push_back(i);
      W.troots.push_back(std::move(R[t]));
      continue;
    }
    const uint8_t* src = chess ? reinterpret_cast<const uint8_t*>(kids[t].data())
                               : reinterpret_cast<const uint8_t*>(vkids[t].data());
    const size_t cnt = chess ? kids[t].size() : vkids[t].size();
    W.kid_first.push_back(W.nk);
    W.kids.insert(W.kids.end(), src, src + cnt * W.rec);
    W.nk += cnt;
    W.mroots.push_back(std::move(R[t]));
    dev_roots.push_back(i);
  }
  W.roots.swap(dev_roots);
  return FNNUE_OK;
}

// A piece's image layout from its games (offsets relative to the piece).
void fnnue_backend::layout(const Job& j, int k, Piece& P) {
  const NetWork& W = net[k];
  size_t text = 0, plies = 0;
  for (size_t i : P.games) {
    text += flen[i] + 1 + mlen[i];
    plies += j.off[i + 1] - j.off[i];
  }
  P.ng = (uint32_t)P.games.size();
  P.n = (uint32_t)plies;
  P.nk = P.kids ? W.nk : 0;
  const size_t ng = P.ng, n = P.n, nk = P.nk;
  P.o_fen = align16(text);
  P.o_mv = P.o_fen + 4 * (ng + 1);
  P.o_ply = P.o_mv + 4 * ng;
  P.o_kids = align16(P.o_ply + 4 * (ng + 1));
  P.o_res = align16(P.o_kids + nk * W.rec);
  P.o_fin = P.o_res + 16;
  P.o_ps = align16(P.o_fin + ng);
  P.o_po = P.o_ps + 4 * (n + nk);
  P.end = P.o_po + 4 * (n + nk);
}

// Cuts the net's games into pieces and places them in its (grow-only) buffers.
int fnnue_backend::plan(Job& j, int k) {
  NetWork& W = net[k];
  W.pieces.clear();
  size_t acc = 0, plies = 0, text = 0;
  for (size_t i : W.games) {
    const size_t t = (size_t)flen[i] + 1 + mlen[i];
    if (W.pieces.empty() || acc >= piece_plies || text + t > kMaxPieceText) {
      W.pieces.emplace_back();
      acc = 0;
      text = 0;
    }
    W.pieces.back().games.push_back(i);
    acc += j.off[i + 1] - j.off[i];
    text += t;
    plies += j.off[i + 1] - j.off[i];
  }
  if (plies >= (1ull << 31)) return fail(FNNUE_E_ARG, "batch too large");
  // A short last piece: its fill is the one the device cannot hide
  if (tail_plies && W.pieces.size() > 1) {
    Piece& L = W.pieces.back();
    size_t t = 0, cut = L.games.size();
    while (cut > 1 && t < tail_plies) {
      --cut;
      t += j.off[L.games[cut] + 1] - j.off[L.games[cut]];
    }
    if (cut > 1 && cut < L.games.size()) {
      Piece T;
      T.games.assign(L.games.begin() + (long)cut, L.games.end());
      L.games.resize(cut);
      W.pieces.push_back(std::move(T));
    }
  }
  if (W.nk) {
    if (W.pieces.empty()) W.pieces.emplace_back();
    W.pieces.back().kids = true;
  }
  size_t up = 0, down = 0, dev = 0, pos = 0;
  for (Piece& P : W.pieces) {
    layout(j, k, P);
    if (P.o_fen >= (1ull << 31)) return fail(FNNUE_E_ARG, "batch text too large");
    P.up0 = up;
    P.down0 = down;
    P.dev0 = dev;
    P.pos0 = pos;
    up = align256(up + P.o_res + 16);
    down = align256(down + P.end - P.o_res);
    dev = align256(dev + P.end);
    pos = align256(pos + (size_t)P.n * W.rec);
  }
  if (int rc = W.dev.reserve(dev)) return rc;
  if (int rc = W.up.reserve(up)) return rc;
  if (int rc = W.down.reserve(down)) return rc;
  if (pos)
    if (int rc = W.pos.reserve(pos)) return rc;
  return W.events(W.pieces.size());
}

// Host image of a piece, then on the context's stream: its upload and the
// replay of its games.  Nothing waits.
int fnnue_backend::stage_up(Job& j, int k, size_t pi) {
  NetWork& W = net[k];
  Piece& P = W.pieces[pi];
  char* img = W.up.at<char>(P.up0);
  uint32_t* fo = reinterpret_cast<uint32_t*>(img + P.o_fen);
  uint32_t* mo = reinterpret_cast<uint32_t*>(img + P.o_mv);
  uint32_t* po = reinterpret_cast<uint32_t*>(img + P.o_ply);
  uint32_t text = 0, acc = 0;
  for (uint32_t g = 0; g < P.ng; ++g) {
    const size_t i = P.games[g];
    fo[g] = text;
    mo[g] = text + flen[i];
    po[g] = acc;
    text += flen[i] + 1 + mlen[i];
    acc += j.off[i + 1] - j.off[i];
  }
  fo[P.ng] = text;
  po[P.ng] = acc;
  pool.run(P.ng, stage_grain, [&](size_t lo, size_t hi) {
    for (size_t g = lo; g < hi; ++g) {
      const size_t i = P.games[g];
      const fnnue_acquired& a = j.batches[i];
      char* d = img + fo[g];
      const uint32_t fl = flen[i], ml = mlen[i];
      if (fl) std::memcpy(d, a.position, fl);
      d[fl] = ' ';
      if (ml) std::memcpy(d + fl + 1, a.moves, ml);
    }
  });
  if (P.nk) std::memcpy(img + P.o_kids, W.kids.data(), P.nk * W.rec);
  std::memset(img + P.o_res, 0, 16);
  char* dimg = W.dev.at<char>(P.dev0);
  hipStream_t us = ctx[k]->stream;
  HIP_TRY(hipMemcpyAsync(dimg, img, P.o_res + 16, hipMemcpyHostToDevice, us), "H2D(batch image)");
  if (P.ng)
    HIP_TRY(replay_games_device(k, dimg, reinterpret_cast<uint32_t*>(dimg + P.o_fen),
                                reinterpret_cast<uint32_t*>(dimg + P.o_mv), reinterpret_cast<uint32_t*>(dimg + P.o_ply),
                                P.ng, W.pos.at<char>(P.pos0), reinterpret_cast<uint8_t*>(dimg + P.o_fin),
                                reinterpret_cast<uint32_t*>(dimg + P.o_res), us),
            "batch replay launch");
  mark("up", k, (long)pi);
  return FNNUE_OK;
}

// On the context's stream, behind the piece's replay: the CHAIN evaluation of
// its plies and the children's evaluation (latching into the piece's own
// error word), then the results to the host.  Nothing waits.
int fnnue_backend::stage_eval(int k, size_t pi) {
  NetWork& W = net[k];
  Piece& P = W.pieces[pi];
  fnnue_ctx* c = ctx[k];
  hipStream_t s = c->stream;
  const bool chess = k == kVariantChess;
  char* dimg = W.dev.at<char>(P.dev0);
  int32_t* d_ps = reinterpret_cast<int32_t*>(dimg + P.o_ps);
  int32_t* d_po = reinterpret_cast<int32_t*>(dimg + P.o_po);
  struct ErrWord {  // the context's error word, redirected for this piece's launches
    fnnue_ctx* c;
    uint32_t* saved;
    ~ErrWord() { c->err = saved; }
  } ew{c, c->err};
  c->err = reinterpret_cast<uint32_t*>(dimg + P.o_res) + 3;
  if (P.ng) {
    const uint32_t* d_off = reinterpret_cast<const uint32_t*>(dimg + P.o_ply);
    const void* d_pos = W.pos.at<char>(P.pos0);
    const int rc = chess ? fnnue_eval_groups_device(c, static_cast<const fnnue_pos*>(d_pos), d_off, P.ng, P.n,
                                                    FNNUE_GROUP_CHAIN, d_ps, d_po, s)
                         : fnnue_eval_vgroups_device(c, static_cast<const fnnue_vpos*>(d_pos), d_off, P.ng, P.n,
                                                     FNNUE_GROUP_CHAIN, d_ps, d_po, s);
    if (rc) return rc;
  }
  if (P.nk) {
    const void* d_kids = dimg + P.o_kids;
    const int rc = chess ? fnnue_eval_positions_device(c, static_cast<const fnnue_pos*>(d_kids), P.nk, d_ps + P.n,
                                                       d_po + P.n, s)
                         : fnnue_eval_vpositions_device(c, static_cast<const fnnue_vpos*>(d_kids), P.nk, d_ps + P.n,
                                                        d_po + P.n, s);
    if (rc) return rc;
  }
  HIP_TRY(hipMemcpyAsync(W.down.at<char>(P.down0), dimg + P.o_res, P.end - P.o_res, hipMemcpyDeviceToHost, s),
          "D2H(results)");
  HIP_TRY(hipEventRecord(W.ev_done[pi], s), "hipEventRecord(results)");
  P.pending = true;
  mark("eval", k, (long)pi);
  return FNNUE_OK;
}

// The net's next piece: when its results are on the host (waiting for them if
// `wait`), writes its responses — after recovering, if the builder or the
// evaluator reported an error.  *ready = false: not there yet.
int fnnue_backend::finish(Job& j, int k, bool wait, bool* ready) {
  NetWork& W = net[k];
  const size_t pi = W.next;
  *ready = false;
  if (wait) {
    const auto tw = Clock::now();
    mark("wait", k, (long)pi);
    const int rc = wait_event(W.ev_done[pi], "waiting for a piece's results");
    wait_ms += ms_since(tw);
    ++syncs;
    if (rc) return rc;
  } else {
    const hipError_t q = hipEventQuery(W.ev_done[pi]);
    if (q == hipErrorNotReady) return FNNUE_OK;
    HIP_TRY(q, "hipEventQuery");
  }
  *ready = true;
  Piece& P = W.pieces[pi];
  P.pending = false;
  const uint32_t* err = W.down.at<uint32_t>(P.down0);
  if (err[0] || err[3])
    if (int rc = recover(j, k, pi)) return rc;
  fill(j, k, P);
  ++W.next;
  return FNNUE_OK;
}

// A game the builder rejected (FEN / move), or whose positions the evaluator
// rejects, fails its own batch: it is dropped from its piece and the piece is
// staged again (its own error words: the other pieces are not affected).
int fnnue_backend::recover(Job& j, int k, size_t pi) {
  NetWork& W = net[k];
  Piece& P = W.pieces[pi];
  for (;;) {
    const uint32_t* berr = W.down.at<uint32_t>(P.down0);
    const uint32_t cerr = berr[3];
    if (!berr[0] && !cerr) break;
    if (berr[0]) {
      // The replay flags every game it rejected (kFinalFailed | code in the
      // game's flag byte); those batches fail (PositionFailed) and the rest
      // are staged again, in one pass however many failed.  A count mismatch
      // or a game index outside the piece cannot be blamed on any batch: the
      // call fails.
      auto bad_word = [&](uint32_t code, uint32_t g) {
        return fail(FNNUE_E_DEVICE, "batch builder reported game " + std::to_string(g) + " of " +
                                        std::to_string(P.ng) + " (code " + std::to_string(code) + ")");
      };
      if (berr[0] == kBuildErrCount || berr[1] >= P.ng) return bad_word(berr[0], berr[1]);
      const uint8_t* fin = W.down.at<uint8_t>(P.down0) + (P.o_fin - P.o_res);
      std::vector<size_t> keep;
      keep.reserve(P.games.size());
      for (uint32_t g = 0; g < P.ng; ++g) {
        const uint32_t code = fin[g] & kFinalFailed ? fin[g] & ~kFinalFailed & 0xFFu : 0u;
        if (code == kBuildErrCount || code > kBuildErrCount) return bad_word(code, g);
        if (code)
          j.rc[P.games[g]] = code == kBuildErrFen ? FNNUE_E_FEN : FNNUE_E_MOVE;
        else
          keep.push_back(P.games[g]);
      }
      if (keep.size() == P.games.size()) return bad_word(berr[0], berr[1]);  // the named game carries no flag
      P.games.swap(keep);
    } else {
      // A FEN the builder parses but the evaluator cannot (kings, > 32
      // pieces): find the games holding such positions, fail those batches.
      // (Move-work children were checked on the host.)
      const size_t nbytes = (size_t)P.n * W.rec;
      if (int rc = W.scratch.reserve(nbytes + 1)) return rc;
      const uint8_t* hpos = W.scratch.at<uint8_t>(0);
      if (nbytes) {
        hipStream_t s = ctx[k]->stream;
        HIP_TRY(hipMemcpyAsync(W.scratch.p, W.pos.at<char>(P.pos0), nbytes, hipMemcpyDeviceToHost, s),
                "D2H(positions)");
        HIP_TRY(hipEventRecord(W.ev_done[pi], s), "hipEventRecord(positions)");
        if (int rc = wait_event(W.ev_done[pi], "reading a failing piece's positions")) return rc;
      }
      ++syncs;
      const uint32_t* ply = W.up.at<uint32_t>(P.up0 + P.o_ply);
      std::vector<size_t> keep;
      for (uint32_t g = 0; g < P.ng; ++g) {
        bool ok = true;
        for (uint32_t x = ply[g]; x < ply[g + 1] && ok; ++x) {
          const uint8_t* p = hpos + (size_t)x * W.rec;
          ok = k == kVariantChess ? valid_host_pos(*reinterpret_cast<const fnnue_pos*>(p))
                                  : host_vpos_state(*reinterpret_cast<const fnnue_vpos*>(p), k) != 0;
        }
        if (ok)
          keep.push_back(P.games[g]);
        else
          j.rc[P.games[g]] = FNNUE_E_POSITION;
      }
      if (keep.size() == P.games.size())
        return fail(cerr & 2u ? FNNUE_E_DEVICE : FNNUE_E_POSITION,
                    "the evaluator latched error " + std::to_string(cerr) + " on piece " + std::to_string(pi) + " of " +
                        std::to_string(W.pieces.size()) + " (net " + std::to_string(k) + ", " + std::to_string(P.ng) +
                        " games, " + std::to_string(P.n) + " plies, pass " + std::to_string(rebuilds) +
                        ") and no batch of the piece holds an invalid position");
      P.games.swap(keep);
    }
    ++rebuilds;
    layout(j, k, P);  // fewer games: the piece still fits its place
    if (int rc = stage_up(j, k, pi)) return rc;
    if (int rc = stage_eval(k, pi)) return rc;
    const int rc = wait_event(W.ev_done[pi], "waiting for a restaged piece");
    ++syncs;
    if (rc) return rc;
    P.pending = false;
  }
  return FNNUE_OK;
}

// Responses of one piece's games from its results image (several threads for
// large pieces): analysis plies as Score::Cp, a game's last ply with no legal
// move as mate 0 / cp 0; then the move work it carries.  time / nps: the wall
// time of the go() call until these results were on the host, and the
// positions evaluated by then per second.  Full records or the compact form.
void fnnue_backend::fill(Job& j, int k, const Piece& P) {
  const auto tf = Clock::now();
  NetWork& W = net[k];
  mark("fill", k, (long)(&P - W.pieces.data()));
  const char* res = W.down.at<char>(P.down0);  // the results image from o_res on
  const uint8_t* fin = reinterpret_cast<const uint8_t*>(res + (P.o_fin - P.o_res));
  const int32_t* ps = reinterpret_cast<const int32_t*>(res + (P.o_ps - P.o_res));
  const int32_t* po = reinterpret_cast<const int32_t*>(res + (P.o_po - P.o_res));
  const uint32_t* ply = W.up.at<uint32_t>(P.up0 + P.o_ply);
  filled += P.n + P.nk;
  const double el = ms_since(t0);
  const uint64_t ms = (uint64_t)el;
  const uint32_t nps = el > 0 ? (uint32_t)std::min(4.0e9, (double)filled / (el * 1e-3)) : 0;
  const int32_t nrm = norm;
  const ResponseTail tail(ms, nps);
  pool.run(P.ng, fill_grain, [&](size_t lo, size_t hi) {
    for (size_t g = lo; g < hi; ++g) {
      const size_t i = P.games[g];
      const uint32_t b = j.off[i], len = j.off[i + 1] - b;
      const uint8_t matrix = j.batches[i].multipv > 0 ? 1 : 0;  // Work::matrix_wanted: multipv is Some
      const bool sk = bskip[i];
      const int32_t* gps = ps + ply[g];
      const int32_t* gpo = po + ply[g];
      // The last ply is the only one that can have no legal move (nothing can
      // be played from it): mate 0 / cp 0 instead of an evaluation.
      const bool ends = fin[g] & kFinalNoMoves;
      const uint8_t end_kind = (fin[g] & (kFinalCheck | kFinalExtinct)) ? FNNUE_SCORE_MATE : FNNUE_SCORE_CP;
      if (j.cout) {
        fnnue_position_compact* r = j.cout + b;
        const uint8_t fl = matrix ? FNNUE_COMPACT_MATRIX : 0;
        for (uint32_t q = 0; q < len; ++q) {
          if (sk && skip[b + q])
            put_compact(r + q, 0, 0, 0, 0, 0, FNNUE_COMPACT_SKIPPED);
          else if (q + 1 == len && ends)
            put_compact(r + q, gps[q], gpo[q], 0, end_kind, 0, fl | FNNUE_COMPACT_NO_MOVES);
          else
            put_compact(r + q, gps[q], gpo[q], (int32_t)to_cp(gps[q], gpo[q], nrm), FNNUE_SCORE_CP, 0, fl);
        }
        fnnue_batch_compact& B = j.bout[i];
        B.time_ms = ms;
        B.nps = nps;
        B.nodes = 0;
        std::memset(B.best_move, 0, sizeof(B.best_move));
        continue;
      }
      fnnue_position_response* r = j.out + b;
      for (uint32_t q = 0; q < len; ++q) {
        if (sk && skip[b + q])
          put_response(r + q, response_head(q, 1, 0, 0, 0), 0, 0, 0, 0, tail);
        else if (q + 1 == len && ends)
          put_response(r + q, response_head(q, 0, end_kind, 0, matrix), 0, gps[q], gpo[q], 0, tail);
        else
          put_response(r + q, response_head(q, 0, FNNUE_SCORE_CP, 0, matrix), to_cp(gps[q], gpo[q], nrm), gps[q],
                       gpo[q], 1, tail);
      }
    }
  });
  if (P.kids) fill_roots(j, k, P, ms, nps);
  fill_ms += ms_since(tf);
  mark("filled", k, (long)(&P - W.pieces.data()));
}

// Move work: a one-ply search over each root's children.
void fnnue_backend::fill_roots(Job& j, int k, const Piece& P, uint64_t ms, uint32_t nps) {
  NetWork& W = net[k];
  const char* res = W.down.at<char>(P.down0);
  const int32_t* kps = reinterpret_cast<const int32_t*>(res + (P.o_ps - P.o_res)) + P.n;
  const int32_t* kpo = reinterpret_cast<const int32_t*>(res + (P.o_po - P.o_res)) + P.n;
  for (size_t t = 0; t < W.roots.size(); ++t) {
    const MoveRoot& R = W.mroots[t];
    const size_t i = W.roots[t];
    // rank: 2 = mates, 1 = evaluated, 0 = never (value orders within a rank)
    size_t best = 0;
    int best_rank = -1;
    int64_t bv = INT64_MIN;
    for (size_t q = 0; q < R.uci.size(); ++q) {
      const size_t x = W.kid_first[t] + q;
      const uint8_t f = R.kid_fin[q];
      int rank = 1;
      int64_t v;
      if (f & (kFinalCheck | kFinalExtinct) && (f & kFinalNoMoves)) {
        rank = 2;
        v = 0;
      } else if (f & kFinalNoMoves) {
        v = 0;  // stalemate
      } else {
        v = -(((int64_t)kps[x] + kpo[x]) / 16);  // Stockfish value of the child, negated
      }
      if (rank > best_rank || (rank == best_rank && v > bv)) {
        best_rank = rank;
        bv = v;
        best = q;
      }
    }
    const size_t x = W.kid_first[t] + best;
    const uint8_t kind = best_rank == 2 ? FNNUE_SCORE_MATE : FNNUE_SCORE_CP;
    const int64_t score = best_rank == 2 ? 1 : bv * 100 / norm;
    if (j.cout) {
      put_compact(j.cout + j.off[i], -kps[x], -kpo[x], (int32_t)score, kind, 1, 0);
      fnnue_batch_compact& B = j.bout[i];
      B.time_ms = ms;
      B.nps = nps;
      B.nodes = (uint32_t)R.uci.size();
      std::memset(B.best_move, 0, sizeof(B.best_move));
      std::strncpy(B.best_move, R.uci[best].c_str(), sizeof(B.best_move) - 1);
      continue;
    }
    fnnue_position_response& r = j.out[j.off[i]];
    std::memset(&r, 0, sizeof(r));
    r.time_ms = ms;
    r.nps = nps;
    r.psqt = -kps[x];
    r.positional = -kpo[x];
    r.depth = 1;
    r.nodes = R.uci.size();
    r.score_kind = kind;
    r.score = score;
    std::strncpy(r.best_move, R.uci[best].c_str(), sizeof(r.best_move) - 1);
  }
}

// The batches answered without the device: move-work roots without a legal
// move, analysis batches whose every position is skipped.
void fnnue_backend::fill_hostonly(Job& j, const std::vector<size_t>& all_skipped) {
  const double el = ms_since(t0);
  const uint64_t ms = (uint64_t)el;
  const uint32_t nps = el > 0 ? (uint32_t)std::min(4.0e9, (double)filled / (el * 1e-3)) : 0;
  auto batch = [&](size_t i) {
    fnnue_batch_compact& B = j.bout[i];
    std::memset(&B, 0, sizeof(B));
    B.time_ms = ms;
    B.nps = nps;
  };
  for (int k = 0; k < kKinds; ++k) {
    NetWork& W = net[k];
    for (size_t t = 0; t < W.terminal.size(); ++t) {
      const size_t i = W.terminal[t];
      const uint8_t fin = W.troots[t].fin;
      if (j.cout) {
        put_compact(j.cout + j.off[i], 0, 0, 0,
                    (fin & (kFinalCheck | kFinalExtinct)) ? FNNUE_SCORE_MATE : FNNUE_SCORE_CP, 0,
                    FNNUE_COMPACT_NO_MOVES);
        batch(i);
        continue;
      }
      fnnue_position_response& r = j.out[j.off[i]];
      std::memset(&r, 0, sizeof(r));
      r.time_ms = ms;
      r.nps = nps;
      terminal_response(r, fin);
    }
  }
  for (size_t i : all_skipped) {
    if (j.cout) batch(i);
    for (uint32_t q = j.off[i]; q < j.off[i + 1]; ++q) {
      if (j.cout) {
        put_compact(j.cout + q, 0, 0, 0, 0, 0, FNNUE_COMPACT_SKIPPED);
        continue;
      }
      fnnue_position_response& r = j.out[q];
      std::memset(&r, 0, sizeof(r));
      r.position_id = q - j.off[i];
      r.skipped = 1;
      r.time_ms = ms;
      r.nps = nps;
    }
  }
}

void fnnue_backend::run(Job& j) {
  t0 = Clock::now();
  deadline = t0 + std::chrono::milliseconds(j.timeout_ms ? j.timeout_ms : timeout_ms);
  tl.clear();
  filled = 0;
  fill_ms = wait_ms = 0;
  syncs = rebuilds = 0;
  const size_t nb = j.nb;
  flen.resize(nb);
  mlen.resize(nb);
  // sizes (IncomingBatch::from_acquired: moves + 1 positions, or 1 for move
  // work) and each batch's net; the strings are scattered in the caller's
  // memory, so the next batches' are prefetched
  kind.resize(nb);
  bskip.resize(nb);
  pool.run(nb, size_grain, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      if (i + 8 < hi) {
        __builtin_prefetch(j.batches[i + 8].moves);
        __builtin_prefetch(j.batches[i + 8].position);
      }
      const fnnue_acquired& a = j.batches[i];
      size_t fl = a.position ? std::strlen(a.position) : 0, ml = 0;
      int rc = FNNUE_OK;
      uint32_t n = 0;
      if (a.work == FNNUE_WORK_MOVE) {
        n = 1;
        ml = a.moves ? std::strlen(a.moves) : 0;
      } else if (a.work != FNNUE_WORK_ANALYSIS || (a.nskip && !a.skip_positions)) {
        rc = FNNUE_E_ARG;
      } else {
        n = (uint32_t)(a.moves ? scan_tokens(a.moves, &ml) : 0) + 1;
      }
      // text beyond any real batch fails that batch alone (it
      // used to be clamped, failing the whole call later)
      if (rc == FNNUE_OK && (fl > kMaxFenBytes || ml > kMaxMovesBytes)) {
        rc = FNNUE_E_ARG;
        fl = ml = 0;
      }
      flen[i] = (uint32_t)fl;
      mlen[i] = (uint32_t)ml;
      const int kd = kind_of(a.variant);
      if (rc == FNNUE_OK && (kd < 0 || !ctx[kd])) rc = FNNUE_E_ARCH;  // no net for this variant on this backend
      if (rc == FNNUE_OK && a.multipv < 0) rc = FNNUE_E_ARG;
      kind[i] = (int8_t)kd;
      bskip[i] = a.nskip != 0;
      j.rc[i] = rc;
      j.off[i + 1] = n;  // counts for now, offsets below (a failed batch keeps its responses' place)
    }
  });
  mark("sizes");
  j.off[0] = 0;
  uint64_t total = 0;
  for (size_t i = 0; i < nb; ++i) {
    total += j.off[i + 1];
    j.off[i + 1] = (uint32_t)total;
  }
  if (total > UINT32_MAX) {  // the offsets are 32-bit
    j.ret = fail(FNNUE_E_ARG, "the batches expand to " + std::to_string(total) + " responses, more than 2^32 - 1");
    j.err = g_err;
    return;
  }
  if (j.off[nb] > j.cap) {
    j.ret = fail(FNNUE_E_CAPACITY, "response buffer holds " + std::to_string(j.cap) + ", batches need " +
                                       std::to_string(j.off[nb]));
    j.err = g_err;
    return;
  }
  for (NetWork& W : net) W.clear();
  if (skip.size() < j.off[nb]) skip.resize(j.off[nb]);  // read only for batches with bskip set
  std::vector<size_t> all_skipped;
  for (size_t i = 0; i < nb; ++i) {
    if (j.rc[i]) continue;
    const fnnue_acquired& a = j.batches[i];
    const int kd = kind[i];
    if (a.work == FNNUE_WORK_MOVE) {
      net[kd].roots.push_back(i);
      continue;
    }
    if (bskip[i]) {
      const uint32_t n = j.off[i + 1] - j.off[i];
      uint32_t live = n;
      std::memset(skip.data() + j.off[i], 0, n);
      for (size_t q = 0; q < a.nskip; ++q)  // positions.get_mut(skip): out-of-range ids are ignored
        if (a.skip_positions[q] < n && !skip[j.off[i] + a.skip_positions[q]]) {
          skip[j.off[i] + a.skip_positions[q]] = 1;
          --live;
        }
      if (!live) {
        all_skipped.push_back(i);  // completed without the engine (IncomingError::AllSkipped)
        continue;
      }
    }
    net[kd].games.push_back(i);
  }
  mark("classified");
  int rc = FNNUE_OK;
  size_t rounds = 0;
  for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k) {
    NetWork& W = net[k];
    W.rec = k == kVariantChess ? sizeof(fnnue_pos) : sizeof(fnnue_vpos);
    if (!W.roots.empty()) rc = prepare_moves(j, k);
    if (rc == FNNUE_OK && (!W.games.empty() || W.nk)) rc = plan(j, k);
    rounds = std::max(rounds, W.pieces.size());
  }
  if (rc == FNNUE_OK && expired()) rc = timed_out("sizing and planning");
  mark("planned");
  // Enqueue order: every net's first upload + replay (the nets' streams run
  // side by side), then each round's evaluations behind the next round's
  // uploads; pieces whose results are back are written between the steps.
  auto poll = [&](bool wait) -> int {
    for (int k = 0; k < kKinds; ++k) {
      NetWork& W = net[k];
      while (W.next < W.pieces.size() && W.pieces[W.next].pending) {
        bool ready = false;
        if (int e = finish(j, k, wait, &ready)) return e;
        if (!ready) break;
      }
    }
    return FNNUE_OK;
  };
  for (size_t r = 0; r <= rounds && rc == FNNUE_OK; ++r) {
    if (r && expired()) {
      rc = timed_out("staging pieces");
      break;
    }
    for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k)
      if (r < net[k].pieces.size()) rc = stage_up(j, k, r);
    for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k)
      if (r >= 1 && r - 1 < net[k].pieces.size()) rc = stage_eval(k, r - 1);
    if (rc == FNNUE_OK && r >= 1 && r < rounds) rc = poll(false);
  }
  // The rest, in the order the results come back: a net's pieces that are
  // back are written while another net's are still on the device (the small
  // variant nets' usually are back first); the host blocks only when a
  // single net is left.
  uint32_t idle_polls = 0;
  while (rc == FNNUE_OK) {
    bool progress = false;
    int first = -1, left = 0;
    for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k) {
      NetWork& W = net[k];
      while (rc == FNNUE_OK && W.next < W.pieces.size()) {
        bool ready = false;
        rc = finish(j, k, false, &ready);
        if (!ready) break;
        progress = true;
      }
      if (W.next < W.pieces.size()) {
        ++left;
        if (first < 0) first = k;
      }
    }
    if (rc || !left) break;
    if (progress) continue;
    if (left == 1 || !any_order) {
      bool ready = false;
      rc = finish(j, first, true, &ready);
    } else {  // polling counts as waiting for the device; a long wait yields the CPU
      const auto tw = Clock::now();
      if (++idle_polls < 256) {
        for (int i = 0; i < 64; ++i) _mm_pause();
      } else {
        sched_yield();
      }
      wait_ms += ms_since(tw);
      if (expired()) rc = timed_out("waiting for the nets' pieces");
    }
    if (progress) idle_polls = 0;
  }
  if (rc == FNNUE_E_TIMEOUT) {
    // The device may still be running this call's pieces, which read and
    // write the channel's pinned buffers: nothing waits for them; the channel
    // is broken (later calls fail fast, fnnue_backend_free reclaims the
    // buffers once the streams have drained).
    abandon_unanswered(j);
    // the answers that need no device (roots without a legal move, batches
    // whose every position is skipped) are written: they are valid
    fill_hostonly(j, all_skipped);
    j.ret = rc;
    j.err = g_err;
    return;
  }
  if (rc) {
    const std::string err = g_err;
    drain_streams();
    j.ret = rc;
    j.err = err;
    return;
  }
  fill_hostonly(j, all_skipped);
  uint32_t npieces = 0;
  for (const NetWork& W : net) npieces += (uint32_t)W.pieces.size();
  j.ret = FNNUE_OK;
  mark("done");
  if (trace) std::fprintf(stderr, "FNNUE_BACKEND_TRACE {\"batches\":%zu,\"marks\":[%s]}\n", nb, tl.c_str());
  std::lock_guard<std::mutex> lk(stats_mu);
  stats.total_ms = ms_since(t0);
  stats.fill_ms = fill_ms;
  stats.device_ms = wait_ms;
  stats.prep_ms = stats.total_ms - fill_ms - wait_ms;
  stats.positions = filled;
  stats.stream_syncs = syncs;
  stats.rebuilds = rebuilds;
  stats.host_threads = pool_threads;
  stats.pieces = npieces;
}

namespace {
void reap_abandoned() {
  std::vector<fnnue_backend*> done;
  {
    std::lock_guard<std::mutex> lk(g_abandoned_mu);
    for (size_t i = 0; i < g_abandoned.size();) {
      fnnue_backend* b = g_abandoned[i];
      DeviceGuard g(b->device);
      if (b->streams_idle()) {
        done.push_back(b);
        g_abandoned[i] = g_abandoned.back();
        g_abandoned.pop_back();
      } else {
        ++i;
      }
    }
  }
  for (fnnue_backend* b : done) {
    DeviceGuard g(b->device);
    b->release_device();
    delete b;
  }
}
}  // namespace

extern "C" {

int fnnue_backend_batch_size(const fnnue_acquired* a, size_t* n) {
  if (!a || !n) return fail(FNNUE_E_ARG, "null argument");
  *n = 0;
  if (a->work == FNNUE_WORK_MOVE) {
    *n = 1;
    return FNNUE_OK;
  }
  if (a->work != FNNUE_WORK_ANALYSIS) return fail(FNNUE_E_ARG, "unknown work type");
  if (a->nskip && !a->skip_positions) return fail(FNNUE_E_ARG, "null skip_positions");
  *n = count_moves(a->moves) + 1;
  return FNNUE_OK;
}

int fnnue_backend_channel_nets(const fnnue_backend_nets* nets, int device, const fnnue_backend_init* init,
                               fnnue_backend** out) {
  if (!nets || !out) return fail(FNNUE_E_ARG, "null argument");
  *out = nullptr;
  const fnnue_net* slot[kKinds] = {nets->chess, nets->crazyhouse, nets->atomic};
  if (!slot[0] && !slot[1] && !slot[2]) return fail(FNNUE_E_ARG, "no net");
  static const char* const kName[kKinds] = {"chess (HalfKAv2_hm)", "crazyhouse", "atomic"};
  for (int k = 0; k < kKinds; ++k) {
    if (!slot[k]) continue;
    int variant = -1;
    if (int rc = fnnue_net_variant(slot[k], &variant)) return rc;
    if (variant != k) return fail(FNNUE_E_ARCH, std::string("the ") + kName[k] + " slot needs a " + kName[k] + " net");
  }
  if (init && init->normalize_to_pawn < 0) return fail(FNNUE_E_ARG, "normalize_to_pawn must be positive");
  reap_abandoned();
  fnnue_backend* b = nullptr;
  try {
    b = new fnnue_backend();
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  b->device = device;
  if (init && init->normalize_to_pawn > 0) b->norm = init->normalize_to_pawn;
  if (init && init->timeout_ms > 0) b->timeout_ms = init->timeout_ms;
  {
    // host threads for the text staging and response fill of large calls: up
    // to 8, at most the CPUs this process may run on (12 or 16: within the
    // box-to-box noise at 16384 batches per call, slower at 1024,
    // profiles/r05/backend_threads/)
    int nt = std::min(8, usable_cpus());
    if (const char* e = std::getenv("FNNUE_BACKEND_THREADS")) nt = std::max(1, std::min(64, std::atoi(e)));
    b->pool_threads = nt;
    b->trace = std::getenv("FNNUE_BACKEND_TRACE") != nullptr;
    if (const char* e = std::getenv("FNNUE_BACKEND_PIECE_PLIES")) b->piece_plies = (size_t)std::max(1024L, std::atol(e));
    if (const char* e = std::getenv("FNNUE_BACKEND_ANY_ORDER")) b->any_order = std::atoi(e) != 0;
    if (const char* e = std::getenv("FNNUE_BACKEND_TAIL_PLIES")) b->tail_plies = (size_t)std::max(0L, std::atol(e));
    if (const char* e = std::getenv("FNNUE_BACKEND_FILL_GRAIN")) b->fill_grain = (size_t)std::max(1L, std::atol(e));
    if (const char* e = std::getenv("FNNUE_BACKEND_SIZE_GRAIN")) b->size_grain = (size_t)std::max(1L, std::atol(e));
    if (const char* e = std::getenv("FNNUE_BACKEND_STAGE_GRAIN")) b->stage_grain = (size_t)std::max(1L, std::atol(e));
  }
  for (int k = 0; k < kKinds; ++k) {
    if (!slot[k]) continue;
    if (int rc = fnnue_ctx_create(slot[k], device, &b->ctx[k])) {
      for (fnnue_ctx* c : b->ctx) fnnue_ctx_free(c);
      delete b;
      return rc;
    }
  }
  try {
    b->pool.start(b->pool_threads);
  } catch (const std::system_error&) {
    b->pool.stop();
    for (fnnue_ctx* c : b->ctx) fnnue_ctx_free(c);
    delete b;
    return fail(FNNUE_E_OOM, "could not start the host worker threads");
  }
  *out = b;
  return FNNUE_OK;
}

int fnnue_backend_channel(const fnnue_net* net, int device, const fnnue_backend_init* init, fnnue_backend** out) {
  if (!net || !out) return fail(FNNUE_E_ARG, "null argument");
  int variant = 0;
  if (int rc = fnnue_net_variant(net, &variant)) return rc;
  fnnue_backend_nets nets{};
  if (variant == kVariantChess) nets.chess = net;
  else if (variant == kVariantCrazyhouse) nets.crazyhouse = net;
  else nets.atomic = net;
  return fnnue_backend_channel_nets(&nets, device, init, out);
}

void fnnue_backend_free(fnnue_backend* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> lk(b->run_mu);  // after the call in flight
    b->closed = true;
  }
  b->pool.stop();
  {
    DeviceGuard g(b->device);
    if (b->broken && !b->streams_idle()) {
      // A timed-out call's pieces are still on the device: freeing their
      // buffers (or the contexts) would wait for them.  The backend is parked
      // and released by a later channel() / free() once its streams drain.
      std::lock_guard<std::mutex> lk(g_abandoned_mu);
      g_abandoned.push_back(b);
      return;
    }
    b->release_device();
  }
  delete b;
  reap_abandoned();
}

namespace {
int go_job(fnnue_backend* b, Job& j, const fnnue_acquired* batches, size_t nbatches, size_t cap, uint32_t* off,
           int32_t* batch_rc, uint32_t timeout_ms) {
  j.batches = batches;
  j.nb = nbatches;
  j.cap = cap;
  j.off = off;
  j.rc = batch_rc;
  j.timeout_ms = timeout_ms;
  std::lock_guard<std::mutex> lk(b->run_mu);  // mpsc::Sender::send on a full channel waits
  if (b->closed) return fail(FNNUE_E_DEVICE, "backend actor stopped");
  if (b->broken) {
    for (size_t i = 0; i < nbatches; ++i) batch_rc[i] = FNNUE_E_TIMEOUT;
    return fail(FNNUE_E_TIMEOUT, "the channel is broken: an earlier go() overran its budget (open a new channel)");
  }
  DeviceGuard g(b->device);
  g_err.clear();
  b->run(j);
  if (j.ret) return fail(j.ret, j.err);
  return FNNUE_OK;
}
}  // namespace

int fnnue_backend_go_timeout(fnnue_backend* b, const fnnue_acquired* batches, size_t nbatches,
                             fnnue_position_response* out, size_t cap, uint32_t* off, int32_t* batch_rc,
                             uint32_t timeout_ms) {
  if (!b || !off || !batch_rc || (nbatches && !batches) || (cap && !out)) return fail(FNNUE_E_ARG, "null argument");
  if (nbatches > (1u << 24)) return fail(FNNUE_E_ARG, "too many batches");
  Job j;
  j.out = out;
  return go_job(b, j, batches, nbatches, cap, off, batch_rc, timeout_ms);
}

int fnnue_backend_go_compact(fnnue_backend* b, const fnnue_acquired* batches, size_t nbatches,
                             fnnue_position_compact* out, size_t cap, fnnue_batch_compact* bout, uint32_t* off,
                             int32_t* batch_rc, uint32_t timeout_ms) {
  if (!b || !off || !batch_rc || (nbatches && (!batches || !bout)) || (cap && !out))
    return fail(FNNUE_E_ARG, "null argument");
  if (nbatches > (1u << 24)) return fail(FNNUE_E_ARG, "too many batches");
  if (b->norm < 13) return fail(FNNUE_E_ARG, "compact results need normalize_to_pawn >= 13 (32-bit scores)");
  Job j;
  j.cout = out;
  j.bout = bout;
  return go_job(b, j, batches, nbatches, cap, off, batch_rc, timeout_ms);
}

int fnnue_backend_go(fnnue_backend* b, const fnnue_acquired* batches, size_t nbatches, fnnue_position_response* out,
                     size_t cap, uint32_t* off, int32_t* batch_rc) {
  return fnnue_backend_go_timeout(b, batches, nbatches, out, cap, off, batch_rc, 0);
}

int fnnue_backend_last_stats(fnnue_backend* b, fnnue_backend_stats* out) {
  if (!b || !out) return fail(FNNUE_E_ARG, "null argument");
  std::lock_guard<std::mutex> lk(b->stats_mu);
  *out = b->stats;
  return FNNUE_OK;
}

int fnnue_backend_analysis_json(const fnnue_position_response* r, size_t n, char* buf, size_t cap, size_t* len) {
  if ((n && !r) || !len || (cap && !buf)) return fail(FNNUE_E_ARG, "null argument");
  std::string s = "[";
  char tmp[192];
  for (size_t i = 0; i < n; ++i) {
    if (i) s += ',';
    if (r[i].skipped) {
      s += "{\"skipped\":true}";
      continue;
    }
    // AnalysisPart::Best: pv omitted when empty, nps omitted when None.
    // AnalysisPart::Matrix: pv / score matrices [multipv - 1][depth]; static
    // eval fills multipv 1 at depth 0 with an empty pv.
    const char* kind = r[i].score_kind == FNNUE_SCORE_MATE ? "mate" : "cp";
    if (r[i].matrix)
      std::snprintf(tmp, sizeof(tmp), "{\"pv\":[[[]]],\"score\":[[{\"%s\":%lld}]],\"depth\":%u,\"nodes\":%llu,"
                    "\"time\":%llu", kind, (long long)r[i].score, (unsigned)r[i].depth, (unsigned long long)r[i].nodes,
                    (unsigned long long)r[i].time_ms);
    else
      std::snprintf(tmp, sizeof(tmp), "{\"score\":{\"%s\":%lld},\"depth\":%u,\"nodes\":%llu,\"time\":%llu", kind,
                    (long long)r[i].score, (unsigned)r[i].depth, (unsigned long long)r[i].nodes,
                    (unsigned long long)r[i].time_ms);
    s += tmp;
    if (r[i].nps) {
      std::snprintf(tmp, sizeof(tmp), ",\"nps\":%u", r[i].nps);
      s += tmp;
    }
    s += '}';
  }
  s += ']';
  *len = s.size();
  if (cap < s.size() + 1) {
    if (cap) buf[0] = 0;
    return fail(FNNUE_E_CAPACITY, "JSON buffer too small");
  }
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return FNNUE_OK;
}

}  // extern "C"
