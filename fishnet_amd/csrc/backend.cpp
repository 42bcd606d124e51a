// backend.cpp — fnnue_backend (include/fnnue_backend.h): fishnet's engine
// actor shape over the evaluator.  The reference's pair
//   stockfish::channel -> (StockfishStub, StockfishActor)   [ref] src/stockfish.rs:23-61
// is a bounded mpsc channel (capacity 1) into an actor owning one engine
// process; StockfishStub::go sends a Position with a oneshot callback and
// maps any failure to PositionFailed{batch_id}.  Here the actor is a worker
// thread owning one fnnue_ctx per net (chess, and optionally the crazyhouse
// and atomic variant nets); a message carries whole acquired batches
// (AcquireResponseBody, [ref] src/api.rs:293-309), expanded the way
// IncomingBatch::from_acquired does ([ref] src/queue.rs:518-627) — but on the
// device: the FEN/UCI text goes to HBM once, the builder replays every game
// there and the plies are evaluated incrementally along each game.
//
// One go(), per net: the host counts each batch's plies (it must: the
// response offsets are part of the answer), stages the text, offsets and the
// move-work children in one pinned buffer and sends it with one copy; the
// stream runs the replay (one wave per game), the CHAIN evaluation and the
// children's evaluation, and one copy brings back the builder's error word,
// the game-end flags and every (psqt, positional); the host waits once.
// Buffers are grow-only (device and pinned host), so a steady stream of calls
// allocates nothing.  A failed batch costs a second pass for its net only.
// Large calls spread the host work (text staging, response fill) over a few
// threads.
#include "../../include/fnnue_backend.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "board.h"
#include "builder.h"
#include "internal.h"
#include "vboard.h"

using namespace fnnue;
using namespace fnnue::detail;

namespace {

constexpr int32_t kNormalizeToPawnSf151 = 361;  // upstream uci.h NormalizeToPawnValue (SF 15.1, recalled)
constexpr int kKinds = 3;                       // net slots: kVariantChess, kVariantCrazyhouse, kVariantAtomic
using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

// One message on the channel: StockfishMessage::Go with its callback.
struct Job {
  const fnnue_acquired* batches = nullptr;
  size_t nb = 0;
  fnnue_position_response* out = nullptr;
  size_t cap = 0;
  uint32_t* off = nullptr;
  int32_t* rc = nullptr;
  int ret = 0;
  std::string err;  // the actor thread's fnnue_last_error, handed to the caller
  bool done = false;
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

// A few host threads for the per-batch loops of large calls (the caller joins
// in): chunks of [0, n) handed out by an atomic counter.
class Workers {
 public:
  void start(int n) {
    for (int i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
    th_.clear();
  }
  // f(lo, hi) over [0, n) in chunks of `grain` items
  void run(size_t n, size_t grain, const std::function<void(size_t, size_t)>& f) {
    if (!n) return;
    if (th_.empty() || n <= grain) {
      f(0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      task_ = &f;
      total_ = n;
      step_ = grain;
      next_ = 0;
      active_ = th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return active_ == 0; });
    task_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const size_t lo = next_.fetch_add(step_);
      if (lo >= total_) return;
      (*task_)(lo, std::min(lo + step_, total_));
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
      if (quit_) return;
      seen = gen_;
      lk.unlock();
      work();
      lk.lock();
      if (--active_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t)>* task_ = nullptr;
  size_t total_ = 0, step_ = 1, active_ = 0;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  bool quit_ = false;
};

inline unsigned is_ws(unsigned char c) { return (c == ' ') | (c == '\t') | (c == '\n') | (c == '\r'); }

// Whitespace-separated tokens of s[0, n) — the builder's rule (replay_wave.h).
size_t count_tokens(const char* s, size_t n) {
  if (!n) return 0;
  const unsigned char* u = reinterpret_cast<const unsigned char*>(s);
  size_t c = is_ws(u[0]) ^ 1u;
  for (size_t i = 1; i < n; ++i) c += (is_ws(u[i]) ^ 1u) & is_ws(u[i - 1]);
  return c;
}

size_t count_moves(const char* s) { return s ? count_tokens(s, std::strlen(s)) : 0; }

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
  auto fin_of = [](const Board& x, const std::vector<Move>& ms) {
    return (uint8_t)((ms.empty() ? kFinalNoMoves : 0) | (x.in_check() ? kFinalCheck : 0));
  };
  std::vector<Move> ms, km;
  b.legal_moves(ms);
  R.fin = fin_of(b, ms);
  for (const Move& m : ms) {
    Board k = b;
    k.do_move(m);
    k.legal_moves(km);
    kids.push_back(k.pack());
    R.uci.push_back(b.uci(m, b.chess960));
    R.kid_fin.push_back(fin_of(k, km));
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

// One net's share of a go(): its analysis games and its move-work roots,
// staged in one pinned host image and one device image of the same layout
//   [text | fen_off | mv_off | ply_off | children | err | fin | psqt | positional]
// the first five parts (and the zeroed error word) go up with one copy, the
// last four come back with one.
struct NetWork {
  std::vector<size_t> games;      // analysis batches (job indices)
  std::vector<size_t> roots;      // move batches whose roots have legal children
  std::vector<MoveRoot> mroots;   // their replayed roots
  std::vector<size_t> kid_first;  // first child of each root
  std::vector<uint8_t> kids;      // children records
  std::vector<size_t> terminal;   // move batches whose root has no legal move
  std::vector<MoveRoot> troots;
  std::vector<uint32_t> toff;     // text offset of each game in the image
  size_t nk = 0, rec = 0;
  size_t o_fen = 0, o_mv = 0, o_ply = 0, o_kids = 0, o_res = 0, o_fin = 0, o_ps = 0, o_po = 0, end = 0;
  uint32_t ng = 0, n = 0;
  bool pending = false;
  DevBuf dev, pos;
  PinnedBuf up, down, cerr;
  void clear() {
    games.clear();
    roots.clear();
    mroots.clear();
    kid_first.clear();
    kids.clear();
    terminal.clear();
    troots.clear();
    nk = 0;
    ng = n = 0;
    pending = false;
  }
  void release() {
    dev.release();
    pos.release();
    up.release();
    down.release();
    cerr.release();
  }
};

}  // namespace

struct fnnue_backend {
  fnnue_ctx* ctx[kKinds] = {};  // one evaluator per net, all on one device
  int device = 0;
  int32_t norm = kNormalizeToPawnSf151;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;  // slot / done / stop changes
  Job* slot = nullptr;         // the capacity-1 channel
  bool stop = false;
  Workers pool;
  int pool_threads = 1;
  NetWork net[kKinds];
  std::vector<uint32_t> flen, mlen;  // per batch of the job in flight: FEN / moves text lengths
  std::vector<uint8_t> skip;         // per response: skipPositions
  std::mutex stats_mu;
  fnnue_backend_stats stats{};

  void run(Job& j);
  int prepare_moves(Job& j, int k);
  int stage(Job& j, int k);
  int collect(Job& j, int k, uint32_t* syncs, uint32_t* rebuilds);
  void fill(Job& j, int k, uint64_t ms, uint32_t nps);
  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return slot != nullptr || stop; });
      if (!slot) return;  // stop with an empty channel
      Job* j = slot;
      slot = nullptr;
      cv.notify_all();  // the channel has room again
      lk.unlock();
      g_err.clear();
      run(*j);
      lk.lock();
      j->done = true;
      cv.notify_all();
    }
  }
};

// Move batches of one net, host side: the position after all moves (one per
// batch) and its legal children with their game-end flags.  A batch whose
// root cannot be replayed fails alone; so does one with a child the
// evaluator would reject (e.g. a root with more than 32 pieces, a pocket
// beyond the variant's limits) — checked here, so that the device never
// latches an error for move work (one bad batch no longer fails
// the call).
int fnnue_backend::prepare_moves(Job& j, int k) {
  NetWork& W = net[k];
  const bool chess = k == kVariantChess;
  std::vector<fnnue_pos> kids;
  std::vector<fnnue_vpos> vkids;
  std::vector<size_t> dev_roots;
  for (size_t i : W.roots) {
    MoveRoot R;
    kids.clear();
    vkids.clear();
    int rc = chess ? chess_move_root(j.batches[i], R, kids) : variant_move_root(k, j.batches[i], R, vkids);
    if (rc == FNNUE_OK) {
      for (const fnnue_pos& p : kids) rc = rc ? rc : (valid_host_pos(p) ? 0 : (int)FNNUE_E_POSITION);
      for (const fnnue_vpos& p : vkids) rc = rc ? rc : (host_vpos_state(p, k) ? 0 : (int)FNNUE_E_POSITION);
    }
    if (rc) {
      j.rc[i] = rc;
      continue;
    }
    if (R.uci.empty()) {
      W.terminal.push_back(i);
      W.troots.push_back(std::move(R));
      continue;
    }
    const uint8_t* src = chess ? reinterpret_cast<const uint8_t*>(kids.data())
                               : reinterpret_cast<const uint8_t*>(vkids.data());
    const size_t cnt = chess ? kids.size() : vkids.size();
    W.kid_first.push_back(W.nk);
    W.kids.insert(W.kids.end(), src, src + cnt * W.rec);
    W.nk += cnt;
    W.mroots.push_back(std::move(R));
    dev_roots.push_back(i);
  }
  W.roots.swap(dev_roots);
  return FNNUE_OK;
}

// Host image of one net's work, then its device work on the net's stream:
// H2D, replay, CHAIN evaluation, children evaluation, D2H.  Nothing waits.
int fnnue_backend::stage(Job& j, int k) {
  NetWork& W = net[k];
  fnnue_ctx* c = ctx[k];
  hipStream_t s = c->stream;
  const bool chess = k == kVariantChess;
  W.ng = (uint32_t)W.games.size();
  size_t text = 0, plies = 0;
  W.toff.resize(W.ng);
  for (uint32_t g = 0; g < W.ng; ++g) {
    const size_t i = W.games[g];
    W.toff[g] = (uint32_t)text;
    text += flen[i] + 1 + mlen[i];
    plies += j.off[i + 1] - j.off[i];
  }
  if (text >= (1ull << 31) || plies >= (1ull << 31)) return fail(FNNUE_E_ARG, "batch text too large");
  W.n = (uint32_t)plies;
  const size_t ng = W.ng, n = W.n, nk = W.nk;
  W.o_fen = align16(text);
  W.o_mv = W.o_fen + 4 * (ng + 1);
  W.o_ply = W.o_mv + 4 * ng;
  W.o_kids = align16(W.o_ply + 4 * (ng + 1));
  W.o_res = align16(W.o_kids + nk * W.rec);
  W.o_fin = W.o_res + 16;
  W.o_ps = align16(W.o_fin + ng);
  W.o_po = W.o_ps + 4 * (n + nk);
  W.end = W.o_po + 4 * (n + nk);
  if (int rc = W.dev.reserve(W.end)) return rc;
  if (int rc = W.up.reserve(W.o_res + 16)) return rc;
  if (int rc = W.down.reserve(W.end - W.o_res)) return rc;
  if (int rc = W.cerr.reserve(4)) return rc;
  if (ng)
    if (int rc = W.pos.reserve(n * W.rec)) return rc;
  char* img = W.up.at<char>(0);
  uint32_t* fo = W.up.at<uint32_t>(W.o_fen);
  uint32_t* mo = W.up.at<uint32_t>(W.o_mv);
  uint32_t* po = W.up.at<uint32_t>(W.o_ply);
  uint32_t acc = 0;
  for (uint32_t g = 0; g < W.ng; ++g) {
    const size_t i = W.games[g];
    fo[g] = W.toff[g];
    mo[g] = W.toff[g] + flen[i];
    po[g] = acc;
    acc += j.off[i + 1] - j.off[i];
  }
  fo[ng] = (uint32_t)text;
  po[ng] = acc;
  pool.run(ng, 512, [&](size_t lo, size_t hi) {
    for (size_t g = lo; g < hi; ++g) {
      const fnnue_acquired& a = j.batches[W.games[g]];
      char* d = img + W.toff[g];
      const uint32_t fl = flen[W.games[g]], ml = mlen[W.games[g]];
      if (fl) std::memcpy(d, a.position, fl);
      d[fl] = ' ';
      if (ml) std::memcpy(d + fl + 1, a.moves, ml);
    }
  });
  if (nk) std::memcpy(img + W.o_kids, W.kids.data(), nk * W.rec);
  std::memset(img + W.o_res, 0, 16);
  HIP_TRY(hipMemcpyAsync(W.dev.p, W.up.p, W.o_res + 16, hipMemcpyHostToDevice, s), "H2D(batch image)");
  uint32_t* d_err = W.dev.at<uint32_t>(W.o_res);
  int32_t* d_ps = W.dev.at<int32_t>(W.o_ps);
  int32_t* d_po = W.dev.at<int32_t>(W.o_po);
  if (ng) {
    HIP_TRY(replay_games_device(k, W.dev.at<char>(0), W.dev.at<uint32_t>(W.o_fen), W.dev.at<uint32_t>(W.o_mv),
                                W.dev.at<uint32_t>(W.o_ply), W.ng, W.pos.p, W.dev.at<uint8_t>(W.o_fin), d_err, s),
            "batch replay launch");
    const uint32_t* d_off = W.dev.at<uint32_t>(W.o_ply);
    const int rc = chess ? fnnue_eval_groups_device(c, static_cast<const fnnue_pos*>(W.pos.p), d_off, ng, n,
                                                    FNNUE_GROUP_CHAIN, d_ps, d_po, s)
                         : fnnue_eval_vgroups_device(c, static_cast<const fnnue_vpos*>(W.pos.p), d_off, ng, n,
                                                     FNNUE_GROUP_CHAIN, d_ps, d_po, s);
    if (rc) return rc;
  }
  if (nk) {
    const void* d_kids = W.dev.at<char>(W.o_kids);
    const int rc = chess ? fnnue_eval_positions_device(c, static_cast<const fnnue_pos*>(d_kids), nk, d_ps + n, d_po + n, s)
                         : fnnue_eval_vpositions_device(c, static_cast<const fnnue_vpos*>(d_kids), nk, d_ps + n,
                                                        d_po + n, s);
    if (rc) return rc;
  }
  HIP_TRY(hipMemcpyAsync(W.down.p, W.dev.at<char>(W.o_res), W.end - W.o_res, hipMemcpyDeviceToHost, s),
          "D2H(results)");
  HIP_TRY(hipMemcpyAsync(W.cerr.p, c->err, 4, hipMemcpyDeviceToHost, s), "D2H(error word)");
  W.pending = true;
  return FNNUE_OK;
}

// Waits for one net's work.  A game the builder rejected (FEN / move) or
// whose positions the evaluator rejects fails its own batch: it is dropped
// and the net's work staged again.
int fnnue_backend::collect(Job& j, int k, uint32_t* syncs, uint32_t* rebuilds) {
  NetWork& W = net[k];
  fnnue_ctx* c = ctx[k];
  hipStream_t s = c->stream;
  for (;;) {
    HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    ++*syncs;
    W.pending = false;
    const uint32_t* berr = W.down.at<uint32_t>(0);
    const uint32_t cerr = *W.cerr.at<uint32_t>(0);
    if (!berr[0] && !cerr) return FNNUE_OK;
    if (cerr) HIP_TRY(hipMemsetAsync(c->err, 0, 4, s), "hipMemsetAsync(error word)");
    if (berr[0]) {
      // The builder names the failing game; that batch fails (PositionFailed)
      // and the rest are staged again.  A count mismatch or a game index
      // outside the batch cannot be blamed on any batch: the call fails.
      if (berr[0] == kBuildErrCount || berr[1] >= W.ng)
        return fail(FNNUE_E_DEVICE, "batch builder reported game " + std::to_string(berr[1]) + " of " +
                                        std::to_string(W.ng) + " (code " + std::to_string(berr[0]) + ")");
      j.rc[W.games[berr[1]]] = berr[0] == kBuildErrFen ? FNNUE_E_FEN : FNNUE_E_MOVE;
      W.games.erase(W.games.begin() + berr[1]);
    } else {
      // A FEN the builder parses but the evaluator cannot (kings, > 32
      // pieces): find the games holding such positions, fail those batches.
      // (Move-work children were checked on the host.)
      std::vector<uint8_t> hpos((size_t)W.n * W.rec);
      if (!hpos.empty())
        HIP_TRY(hipMemcpy(hpos.data(), W.pos.p, hpos.size(), hipMemcpyDeviceToHost), "D2H(positions)");
      ++*syncs;
      const uint32_t* ply = W.up.at<uint32_t>(W.o_ply);
      std::vector<size_t> keep;
      for (uint32_t g = 0; g < W.ng; ++g) {
        bool ok = true;
        for (uint32_t x = ply[g]; x < ply[g + 1] && ok; ++x) {
          const uint8_t* p = hpos.data() + (size_t)x * W.rec;
          ok = k == kVariantChess ? valid_host_pos(*reinterpret_cast<const fnnue_pos*>(p))
                                  : host_vpos_state(*reinterpret_cast<const fnnue_vpos*>(p), k) != 0;
        }
        if (ok)
          keep.push_back(W.games[g]);
        else
          j.rc[W.games[g]] = FNNUE_E_POSITION;
      }
      if (keep.size() == W.games.size())
        return fail(FNNUE_E_POSITION, "the evaluator rejected a position no batch holds");
      W.games.swap(keep);
    }
    ++*rebuilds;
    if (int rc = stage(j, k)) return rc;
  }
}

// Responses of one net's batches from the results image (several threads for
// large calls): analysis plies as Score::Cp, a game's last ply with no legal
// move as mate 0 / cp 0; move work as a one-ply search over the children.
void fnnue_backend::fill(Job& j, int k, uint64_t ms, uint32_t nps) {
  NetWork& W = net[k];
  const uint8_t* fin = W.down.at<uint8_t>(W.o_fin - W.o_res);
  const int32_t* ps = W.down.at<int32_t>(W.o_ps - W.o_res);
  const int32_t* po = W.down.at<int32_t>(W.o_po - W.o_res);
  const uint32_t* ply = W.up.at<uint32_t>(W.o_ply);
  const int32_t nrm = norm;
  pool.run(W.ng, 64, [&](size_t lo, size_t hi) {
    for (size_t g = lo; g < hi; ++g) {
      const size_t i = W.games[g];
      const uint32_t b = j.off[i], len = j.off[i + 1] - b;
      const uint8_t matrix = j.batches[i].multipv > 0 ? 1 : 0;  // Work::matrix_wanted: multipv is Some
      for (uint32_t q = 0; q < len; ++q) {
        fnnue_position_response r;
        std::memset(&r, 0, sizeof(r));
        r.position_id = q;
        r.time_ms = ms;
        r.nps = nps;
        if (skip[b + q]) {
          r.skipped = 1;
        } else {
          const size_t x = ply[g] + q;
          r.matrix = matrix;
          r.psqt = ps[x];
          r.positional = po[x];
          r.score_kind = FNNUE_SCORE_CP;
          r.score = to_cp(r.psqt, r.positional, nrm);
          r.nodes = 1;
          // The last ply is the only one that can have no legal move (nothing
          // can be played from it): mate 0 / cp 0 instead of an evaluation.
          if (q + 1 == len && (fin[g] & kFinalNoMoves)) terminal_response(r, fin[g]);
        }
        j.out[b + q] = r;
      }
    }
  });
  auto root_response = [&](size_t i) -> fnnue_position_response& {
    fnnue_position_response& r = j.out[j.off[i]];
    std::memset(&r, 0, sizeof(r));
    r.time_ms = ms;
    r.nps = nps;
    return r;
  };
  for (size_t t = 0; t < W.terminal.size(); ++t) terminal_response(root_response(W.terminal[t]), W.troots[t].fin);
  const int32_t* kps = ps + W.n;
  const int32_t* kpo = po + W.n;
  for (size_t t = 0; t < W.roots.size(); ++t) {
    const MoveRoot& R = W.mroots[t];
    fnnue_position_response& r = root_response(W.roots[t]);
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
    r.psqt = -kps[x];
    r.positional = -kpo[x];
    r.depth = 1;
    r.nodes = R.uci.size();
    if (best_rank == 2) {
      r.score_kind = FNNUE_SCORE_MATE;
      r.score = 1;
    } else {
      r.score_kind = FNNUE_SCORE_CP;
      r.score = bv * 100 / nrm;
    }
    std::strncpy(r.best_move, R.uci[best].c_str(), sizeof(r.best_move) - 1);
  }
}

void fnnue_backend::run(Job& j) {
  const auto t0 = Clock::now();
  const size_t nb = j.nb;
  flen.resize(nb);
  mlen.resize(nb);
  // sizes (IncomingBatch::from_acquired: moves + 1 positions, or 1 for move work)
  pool.run(nb, 2048, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const fnnue_acquired& a = j.batches[i];
      flen[i] = a.position ? (uint32_t)std::min<size_t>(std::strlen(a.position), 1u << 30) : 0;
      mlen[i] = a.moves ? (uint32_t)std::min<size_t>(std::strlen(a.moves), 1u << 30) : 0;
      int rc = FNNUE_OK;
      uint32_t n = 0;
      if (a.work == FNNUE_WORK_MOVE) n = 1;
      else if (a.work != FNNUE_WORK_ANALYSIS) rc = FNNUE_E_ARG;
      else if (a.nskip && !a.skip_positions) rc = FNNUE_E_ARG;
      else n = (uint32_t)count_tokens(a.moves ? a.moves : "", mlen[i]) + 1;
      j.rc[i] = rc;
      j.off[i + 1] = rc ? 0 : n;  // counts for now, offsets below
    }
  });
  j.off[0] = 0;
  for (size_t i = 0; i < nb; ++i) j.off[i + 1] += j.off[i];
  if (j.off[nb] > j.cap) {
    j.ret = fail(FNNUE_E_CAPACITY, "response buffer holds " + std::to_string(j.cap) + ", batches need " +
                                       std::to_string(j.off[nb]));
    j.err = g_err;
    return;
  }
  for (NetWork& W : net) W.clear();
  skip.assign(j.off[nb], 0);
  std::vector<size_t> all_skipped;
  for (size_t i = 0; i < nb; ++i) {
    const fnnue_acquired& a = j.batches[i];
    if (j.rc[i]) continue;
    const int kind = kind_of(a.variant);
    if (kind < 0 || !ctx[kind] || a.multipv < 0) {  // no net for this variant on this backend
      j.rc[i] = kind < 0 || !ctx[kind] ? FNNUE_E_ARCH : FNNUE_E_ARG;
      continue;
    }
    const uint32_t n = j.off[i + 1] - j.off[i];
    if (a.work == FNNUE_WORK_MOVE) {
      net[kind].roots.push_back(i);
      continue;
    }
    uint32_t live = n;
    for (size_t q = 0; q < a.nskip; ++q)  // positions.get_mut(skip): out-of-range ids are ignored
      if (a.skip_positions[q] < n && !skip[j.off[i] + a.skip_positions[q]]) {
        skip[j.off[i] + a.skip_positions[q]] = 1;
        --live;
      }
    if (live) net[kind].games.push_back(i);
    else all_skipped.push_back(i);  // completed without the engine (IncomingError::AllSkipped)
  }
  int rc = FNNUE_OK;
  for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k) {
    NetWork& W = net[k];
    W.rec = k == kVariantChess ? sizeof(fnnue_pos) : sizeof(fnnue_vpos);
    if (!W.roots.empty()) rc = prepare_moves(j, k);
    if (rc == FNNUE_OK && (!W.games.empty() || W.nk)) rc = stage(j, k);
  }
  const double prep_ms = ms_since(t0);
  uint32_t syncs = 0, rebuilds = 0;
  for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k)
    if (net[k].pending) rc = collect(j, k, &syncs, &rebuilds);
  if (rc) {
    for (int k = 0; k < kKinds; ++k)  // the pinned images stay in use until the copies are done
      if (net[k].pending) (void)hipStreamSynchronize(ctx[k]->stream);
    j.ret = rc;
    j.err = g_err;
    return;
  }
  const double dev_ms = ms_since(t0) - prep_ms;
  const double sec = ms_since(t0) * 1e-3;
  uint64_t evals = 0;
  for (const NetWork& W : net) evals += W.n + W.nk;
  const uint64_t ms = (uint64_t)(sec * 1e3);
  const uint32_t nps = sec > 0 ? (uint32_t)std::min(4.0e9, (double)evals / sec) : 0;
  const auto t2 = Clock::now();
  for (int k = 0; k < kKinds; ++k) fill(j, k, ms, nps);
  for (size_t i : all_skipped)
    for (uint32_t q = j.off[i]; q < j.off[i + 1]; ++q) {
      fnnue_position_response& r = j.out[q];
      std::memset(&r, 0, sizeof(r));
      r.position_id = q - j.off[i];
      r.skipped = 1;
      r.time_ms = ms;
      r.nps = nps;
    }
  j.ret = FNNUE_OK;
  std::lock_guard<std::mutex> lk(stats_mu);
  stats.prep_ms = prep_ms;
  stats.device_ms = dev_ms;
  stats.fill_ms = ms_since(t2);
  stats.total_ms = ms_since(t0);
  stats.positions = evals;
  stats.stream_syncs = syncs;
  stats.rebuilds = rebuilds;
  stats.host_threads = pool_threads;
}

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
  fnnue_backend* b = nullptr;
  try {
    b = new fnnue_backend();
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  b->device = device;
  if (init && init->normalize_to_pawn > 0) b->norm = init->normalize_to_pawn;
  {
    // host threads for the text staging and response fill of large calls
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    int nt = (int)std::min(8u, hw);
    if (const char* e = std::getenv("FNNUE_BACKEND_THREADS")) nt = std::max(1, std::min(64, std::atoi(e)));
    b->pool_threads = nt;
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
    b->th = std::thread([b] {
      DeviceGuard g(b->device);
      b->loop();
    });
  } catch (const std::system_error&) {
    b->pool.stop();
    for (fnnue_ctx* c : b->ctx) fnnue_ctx_free(c);
    delete b;
    return fail(FNNUE_E_OOM, "could not start the actor thread");
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
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
  }
  b->cv.notify_all();
  if (b->th.joinable()) b->th.join();
  b->pool.stop();
  {
    DeviceGuard g(b->device);
    for (NetWork& W : b->net) W.release();
  }
  for (fnnue_ctx* c : b->ctx) fnnue_ctx_free(c);
  delete b;
}

int fnnue_backend_go(fnnue_backend* b, const fnnue_acquired* batches, size_t nbatches, fnnue_position_response* out,
                     size_t cap, uint32_t* off, int32_t* batch_rc) {
  if (!b || !off || !batch_rc || (nbatches && !batches) || (cap && !out)) return fail(FNNUE_E_ARG, "null argument");
  if (nbatches > (1u << 24)) return fail(FNNUE_E_ARG, "too many batches");
  Job j;
  j.batches = batches;
  j.nb = nbatches;
  j.out = out;
  j.cap = cap;
  j.off = off;
  j.rc = batch_rc;
  std::unique_lock<std::mutex> lk(b->mu);
  b->cv.wait(lk, [&] { return b->slot == nullptr || b->stop; });  // mpsc::Sender::send on a full channel
  if (b->stop) return fail(FNNUE_E_DEVICE, "backend actor stopped");
  b->slot = &j;
  b->cv.notify_all();
  b->cv.wait(lk, [&] { return j.done; });  // the oneshot callback
  lk.unlock();
  if (j.ret) return fail(j.ret, j.err);
  return FNNUE_OK;
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
