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
#include "../../include/fnnue_backend.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstring>
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
  T* as() const {
    return static_cast<T*>(p);
  }
};

size_t count_moves(const char* s) {
  size_t n = 0;
  for (bool in = false; s && *s; ++s) {
    const bool sp = *s == ' ' || *s == '\t' || *s == '\n' || *s == '\r';
    if (!sp && !in) ++n;
    in = !sp;
  }
  return n;
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
  DevBuf text, fen_off, mv_off, pos, goff, psqt, positional, fin;
  std::vector<uint8_t> hpos;  // positions read back to find an invalid one (36 or 48 B records)
  std::vector<int32_t> hpsqt, hpositional;
  std::vector<uint32_t> hgoff;
  std::vector<uint8_t> hfin;

  void run(Job& j);
  int analysis(Job& j, int kind, const std::vector<size_t>& games, const std::vector<uint8_t>& skip);
  int moves(Job& j, int kind, const std::vector<size_t>& games);
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

// Analysis batches of one net: the games' text to HBM, the device builder
// replays them (one CHAIN group per game) and flags each game's last
// position, CHAIN evaluation, responses written in place.  A game the builder
// rejects (FEN / move) or whose positions the evaluator rejects fails its own
// batch only: it is dropped and the rest rebuilt.
int fnnue_backend::analysis(Job& j, int kind, const std::vector<size_t>& games_in, const std::vector<uint8_t>& skip) {
  fnnue_ctx* c = ctx[kind];
  const bool chess = kind == kVariantChess;
  const size_t rec = chess ? sizeof(fnnue_pos) : sizeof(fnnue_vpos);
  std::vector<size_t> live = games_in;
  hipStream_t s = c->stream;
  while (!live.empty()) {
    std::string t;
    std::vector<uint32_t> fo(live.size() + 1), mo(live.size());
    for (size_t g = 0; g < live.size(); ++g) {
      const fnnue_acquired& a = j.batches[live[g]];
      fo[g] = (uint32_t)t.size();
      t += a.position ? a.position : "";
      mo[g] = (uint32_t)t.size();
      t += ' ';
      t += a.moves ? a.moves : "";
    }
    fo[live.size()] = (uint32_t)t.size();
    if (t.size() >= (1ull << 31)) return fail(FNNUE_E_ARG, "batch text too large");
    const uint32_t ng = (uint32_t)live.size();
    if (int rc = text.reserve(t.size() + 1)) return rc;
    if (int rc = fen_off.reserve(fo.size() * 4)) return rc;
    if (int rc = mv_off.reserve(mo.size() * 4)) return rc;
    if (int rc = fin.reserve(ng)) return rc;
    HIP_TRY(hipMemcpyAsync(text.p, t.data(), t.size(), hipMemcpyHostToDevice, s), "H2D(text)");
    HIP_TRY(hipMemcpyAsync(fen_off.p, fo.data(), fo.size() * 4, hipMemcpyHostToDevice, s), "H2D(fen offsets)");
    HIP_TRY(hipMemcpyAsync(mv_off.p, mo.data(), mo.size() * 4, hipMemcpyHostToDevice, s), "H2D(move offsets)");
    // The builder names the failing game; that batch fails (PositionFailed)
    // and the rest are retried.  A game index outside the batch cannot be
    // blamed on any batch: the whole call fails instead.
    auto drop = [&](const BuildResult& R) {
      if (R.err_game >= ng)
        return fail(FNNUE_E_DEVICE, "batch builder reported game " + std::to_string(R.err_game) + " of " +
                                        std::to_string(ng));
      j.rc[live[R.err_game]] = R.err_code == kBuildErrFen ? FNNUE_E_FEN : FNNUE_E_MOVE;
      live.erase(live.begin() + (long)R.err_game);
      return (int)FNNUE_OK;
    };
    auto build = [&](void* out, size_t cap, uint32_t* goffp, size_t ocap) {
      return chess ? build_batch_device(text.as<char>(), fen_off.as<uint32_t>(), mv_off.as<uint32_t>(), ng, false,
                                        static_cast<fnnue_pos*>(out), cap, goffp, ocap, s, fin.as<uint8_t>())
                   : build_vbatch_device(kind, text.as<char>(), fen_off.as<uint32_t>(), mv_off.as<uint32_t>(), ng,
                                         false, static_cast<fnnue_vpos*>(out), cap, goffp, ocap, s,
                                         fin.as<uint8_t>());
    };
    // sizing pass, then the outputs (both synchronise the stream)
    BuildResult R = build(nullptr, 0, nullptr, 0);
    if (R.hip != hipSuccess) return hip_fail(R.hip, "device batch builder");
    if (R.err_code) {
      if (int rc = drop(R)) return rc;
      continue;
    }
    const size_t n = R.n_out;
    if (int rc = pos.reserve(n * rec)) return rc;
    if (int rc = goff.reserve((ng + 1) * 4)) return rc;
    if (int rc = psqt.reserve(n * 4)) return rc;
    if (int rc = positional.reserve(n * 4)) return rc;
    R = build(pos.p, n, goff.as<uint32_t>(), ng + 1);
    if (R.hip != hipSuccess) return hip_fail(R.hip, "device batch builder");
    if (R.err_code) {
      if (int rc = drop(R)) return rc;
      continue;
    }
    if (R.capacity || R.n_out != n || R.n_groups != ng) return fail(FNNUE_E_DEVICE, "batch builder sizes changed");
    int rc = chess ? fnnue_eval_groups_device(c, pos.as<fnnue_pos>(), goff.as<uint32_t>(), ng, n, FNNUE_GROUP_CHAIN,
                                              psqt.as<int32_t>(), positional.as<int32_t>(), s)
                   : fnnue_eval_vgroups_device(c, pos.as<fnnue_vpos>(), goff.as<uint32_t>(), ng, n, FNNUE_GROUP_CHAIN,
                                               psqt.as<int32_t>(), positional.as<int32_t>(), s);
    if (rc == FNNUE_OK) rc = fnnue_ctx_check(c);  // synchronises; latched invalid positions
    hgoff.resize(ng + 1);
    HIP_TRY(hipMemcpy(hgoff.data(), goff.p, (ng + 1) * 4, hipMemcpyDeviceToHost), "D2H(group offsets)");
    if (rc == FNNUE_E_POSITION) {
      // A FEN the builder parses but the evaluator cannot (kings, > 32
      // pieces): find the games holding such positions, fail those batches.
      hpos.resize(n * rec);
      HIP_TRY(hipMemcpy(hpos.data(), pos.p, n * rec, hipMemcpyDeviceToHost), "D2H(positions)");
      std::vector<size_t> keep;
      for (size_t g = 0; g < ng; ++g) {
        bool ok = true;
        for (uint32_t k = hgoff[g]; k < hgoff[g + 1] && ok; ++k) {
          const uint8_t* p = hpos.data() + (size_t)k * rec;
          ok = chess ? valid_host_pos(*reinterpret_cast<const fnnue_pos*>(p))
                     : host_vpos_state(*reinterpret_cast<const fnnue_vpos*>(p), kind) != 0;
        }
        if (ok)
          keep.push_back(live[g]);
        else
          j.rc[live[g]] = FNNUE_E_POSITION;
      }
      if (keep.size() == live.size()) return rc;  // not attributable to a game
      live.swap(keep);
      continue;
    }
    if (rc) return rc;
    hpsqt.resize(n);
    hpositional.resize(n);
    hfin.resize(ng);
    HIP_TRY(hipMemcpy(hpsqt.data(), psqt.p, n * 4, hipMemcpyDeviceToHost), "D2H(psqt)");
    HIP_TRY(hipMemcpy(hpositional.data(), positional.p, n * 4, hipMemcpyDeviceToHost), "D2H(positional)");
    HIP_TRY(hipMemcpy(hfin.data(), fin.p, ng, hipMemcpyDeviceToHost), "D2H(final flags)");
    for (size_t g = 0; g < ng; ++g) {
      const size_t i = live[g];
      const uint32_t b = j.off[i], len = j.off[i + 1] - b;
      if (hgoff[g + 1] - hgoff[g] != len) return fail(FNNUE_E_DEVICE, "builder ply count differs from the moves");
      for (uint32_t k = 0; k < len; ++k) {
        fnnue_position_response& r = j.out[b + k];
        if (skip[b + k]) continue;
        const size_t x = hgoff[g] + k;
        r.matrix = j.batches[i].multipv > 0 ? 1 : 0;  // Work::matrix_wanted: multipv is Some
        r.psqt = hpsqt[x];
        r.positional = hpositional[x];
        r.score_kind = FNNUE_SCORE_CP;
        r.score = to_cp(r.psqt, r.positional, norm);
        r.depth = 0;
        r.nodes = 1;
      }
      // The last ply is the only one that can have no legal move (nothing can
      // be played from it): mate 0 / cp 0 instead of an evaluation.
      if (len && (hfin[g] & kFinalNoMoves) && !skip[b + len - 1]) terminal_response(j.out[b + len - 1], hfin[g]);
    }
    return FNNUE_OK;
  }
  return FNNUE_OK;
}

// Move batches of one net: the position after all moves (host replay: one
// position per batch) and its legal children.  A one-ply search: a child that
// mates (checkmate, or atomic: the other king exploded) wins outright (score
// mate 1), a stalemating child is a draw (0), every other child is worth
// -v(child) from its NNUE evaluation; best = the first maximum.  A root with
// no legal move answers as the engine does: no best move, mate 0 / cp 0.
int fnnue_backend::moves(Job& j, int kind, const std::vector<size_t>& games) {
  struct Cand {
    size_t batch;
    MoveRoot root;
    size_t first;
  };
  std::vector<Cand> cands;
  std::vector<fnnue_pos> kids;
  std::vector<fnnue_vpos> vkids;
  for (size_t i : games) {
    Cand c{i, {}, kind == kVariantChess ? kids.size() : vkids.size()};
    const int rc = kind == kVariantChess ? chess_move_root(j.batches[i], c.root, kids)
                                         : variant_move_root(kind, j.batches[i], c.root, vkids);
    if (rc) {
      j.rc[i] = rc;
      if (kind == kVariantChess) kids.resize(c.first);
      else vkids.resize(c.first);
      continue;
    }
    cands.push_back(std::move(c));
  }
  const size_t nk = kind == kVariantChess ? kids.size() : vkids.size();
  std::vector<int32_t> ps(nk), po(nk);
  if (nk) {
    const int rc = kind == kVariantChess ? fnnue_eval_positions(ctx[kind], kids.data(), nk, ps.data(), po.data())
                                         : fnnue_eval_vpositions(ctx[kind], vkids.data(), nk, ps.data(), po.data());
    if (rc) return rc;
  }
  for (const Cand& c : cands) {
    fnnue_position_response& r = j.out[j.off[c.batch]];
    if (c.root.uci.empty()) {
      terminal_response(r, c.root.fin);
      continue;
    }
    // rank: 2 = mates, 1 = evaluated, 0 = never (value orders within a rank)
    size_t best = 0;
    int best_rank = -1;
    int64_t bv = INT64_MIN;
    for (size_t k = 0; k < c.root.uci.size(); ++k) {
      const size_t x = c.first + k;
      const uint8_t f = c.root.kid_fin[k];
      int rank = 1;
      int64_t v;
      if (f & (kFinalCheck | kFinalExtinct) && (f & kFinalNoMoves)) {
        rank = 2;
        v = 0;
      } else if (f & kFinalNoMoves) {
        v = 0;  // stalemate
      } else {
        v = -(((int64_t)ps[x] + po[x]) / 16);  // Stockfish value of the child, negated
      }
      if (rank > best_rank || (rank == best_rank && v > bv)) {
        best_rank = rank;
        bv = v;
        best = k;
      }
    }
    const size_t x = c.first + best;
    r.psqt = -ps[x];
    r.positional = -po[x];
    r.depth = 1;
    r.nodes = c.root.uci.size();
    if (best_rank == 2) {
      r.score_kind = FNNUE_SCORE_MATE;
      r.score = 1;
    } else {
      r.score_kind = FNNUE_SCORE_CP;
      r.score = bv * 100 / norm;
    }
    std::strncpy(r.best_move, c.root.uci[best].c_str(), sizeof(r.best_move) - 1);
  }
  return FNNUE_OK;
}

void fnnue_backend::run(Job& j) {
  const auto t0 = std::chrono::steady_clock::now();
  const size_t nb = j.nb;
  j.off[0] = 0;
  for (size_t i = 0; i < nb; ++i) {
    size_t n = 0;
    j.rc[i] = fnnue_backend_batch_size(&j.batches[i], &n);
    if (j.rc[i]) n = 0;
    j.off[i + 1] = j.off[i] + (uint32_t)n;
  }
  if (j.off[nb] > j.cap) {
    j.ret = fail(FNNUE_E_CAPACITY, "response buffer holds " + std::to_string(j.cap) + ", batches need " +
                                       std::to_string(j.off[nb]));
    j.err = g_err;
    return;
  }
  std::vector<size_t> ana[kKinds], mov[kKinds];
  std::vector<uint8_t> skip(j.off[nb], 0);
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
      mov[kind].push_back(i);
      continue;
    }
    uint32_t live = n;
    for (size_t k = 0; k < a.nskip; ++k)  // positions.get_mut(skip): out-of-range ids are ignored
      if (a.skip_positions[k] < n && !skip[j.off[i] + a.skip_positions[k]]) {
        skip[j.off[i] + a.skip_positions[k]] = 1;
        --live;
      }
    if (live) ana[kind].push_back(i);  // all skipped: completed without the engine (IncomingError::AllSkipped)
  }
  std::memset(j.out, 0, j.off[nb] * sizeof(fnnue_position_response));
  int rc = FNNUE_OK;
  for (int k = 0; k < kKinds && rc == FNNUE_OK; ++k) {
    if (!ana[k].empty()) rc = analysis(j, k, ana[k], skip);
    if (rc == FNNUE_OK && !mov[k].empty()) rc = moves(j, k, mov[k]);
  }
  if (rc) {
    j.ret = rc;
    j.err = g_err;
    return;
  }
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t nodes = 0;
  for (size_t i = 0; i < nb; ++i) {
    if (j.rc[i]) continue;
    for (uint32_t k = j.off[i]; k < j.off[i + 1]; ++k) nodes += j.out[k].nodes;
  }
  const uint64_t ms = (uint64_t)(sec * 1e3);
  const uint32_t nps = sec > 0 ? (uint32_t)std::min(4.0e9, (double)nodes / sec) : 0;
  for (size_t i = 0; i < nb; ++i) {
    if (j.rc[i]) continue;
    for (uint32_t k = j.off[i]; k < j.off[i + 1]; ++k) {
      fnnue_position_response& r = j.out[k];
      r.position_id = k - j.off[i];
      r.time_ms = ms;
      r.nps = nps;
      if (skip[k]) r.skipped = 1;
    }
  }
  j.ret = FNNUE_OK;
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
  for (int k = 0; k < kKinds; ++k) {
    if (!slot[k]) continue;
    if (int rc = fnnue_ctx_create(slot[k], device, &b->ctx[k])) {
      for (fnnue_ctx* c : b->ctx) fnnue_ctx_free(c);
      delete b;
      return rc;
    }
  }
  try {
    b->th = std::thread([b] {
      DeviceGuard g(b->device);
      b->loop();
    });
  } catch (const std::system_error&) {
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
  {
    DeviceGuard g(b->device);
    for (DevBuf* d : {&b->text, &b->fen_off, &b->mv_off, &b->pos, &b->goff, &b->psqt, &b->positional, &b->fin})
      d->release();
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
