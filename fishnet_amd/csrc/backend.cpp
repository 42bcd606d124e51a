// backend.cpp — fnnue_backend (include/fnnue_backend.h): fishnet's engine
// actor shape over the evaluator.  The reference's pair
//   stockfish::channel -> (StockfishStub, StockfishActor)   [ref] src/stockfish.rs:23-61
// is a bounded mpsc channel (capacity 1) into an actor owning one engine
// process; StockfishStub::go sends a Position with a oneshot callback and
// maps any failure to PositionFailed{batch_id}.  Here the actor is a worker
// thread owning one fnnue_ctx; a message carries whole acquired batches
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

using namespace fnnue;
using namespace fnnue::detail;

namespace {

constexpr int32_t kNormalizeToPawnSf151 = 361;  // upstream uci.h NormalizeToPawnValue (SF 15.1, recalled)

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

// Variants this backend evaluates with the chess net (EngineFlavor::Official,
// queue.rs:530-539); everything else the reference sends to Fairy-Stockfish.
bool chess_variant(const char* v) {
  return !v || !*v || !std::strcmp(v, "standard") || !std::strcmp(v, "chess960") ||
         !std::strcmp(v, "fromPosition") || !std::strcmp(v, "chess");
}

int64_t to_cp(int32_t psqt, int32_t positional, int32_t norm) {
  const int64_t v = ((int64_t)psqt + positional) / 16;  // OutputScale, C truncation
  return v * 100 / norm;
}

}  // namespace

struct fnnue_backend {
  fnnue_ctx* ctx = nullptr;
  int32_t norm = kNormalizeToPawnSf151;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;  // slot / done / stop changes
  Job* slot = nullptr;         // the capacity-1 channel
  bool stop = false;
  DevBuf text, fen_off, mv_off, pos, goff, psqt, positional;
  std::vector<fnnue_pos> hpos;
  std::vector<int32_t> hpsqt, hpositional;
  std::vector<uint32_t> hgoff;

  void run(Job& j);
  int analysis(Job& j, const std::vector<size_t>& games, std::vector<size_t>& base);
  int moves(Job& j, const std::vector<size_t>& games);
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

// Analysis batches: the games' text to HBM, the device builder replays them
// (one CHAIN group per game), CHAIN evaluation, results back.  A game the
// builder rejects (FEN / move) or whose positions the evaluator rejects fails
// its own batch only: it is dropped and the rest rebuilt.  base[i] = first
// position of games[i] in the host result arrays.
int fnnue_backend::analysis(Job& j, const std::vector<size_t>& games_in, std::vector<size_t>& base) {
  std::vector<size_t> live = games_in;
  hipStream_t s = ctx->stream;
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
    // sizing pass, then the outputs (both synchronise the stream)
    BuildResult R = build_batch_device(text.as<char>(), fen_off.as<uint32_t>(), mv_off.as<uint32_t>(), ng, false,
                                       nullptr, 0, nullptr, 0, s);
    if (R.hip != hipSuccess) return hip_fail(R.hip, "device batch builder");
    if (R.err_code) {
      if (int rc = drop(R)) return rc;
      continue;
    }
    const size_t n = R.n_out;
    if (int rc = pos.reserve(n * sizeof(fnnue_pos))) return rc;
    if (int rc = goff.reserve((ng + 1) * 4)) return rc;
    if (int rc = psqt.reserve(n * 4)) return rc;
    if (int rc = positional.reserve(n * 4)) return rc;
    R = build_batch_device(text.as<char>(), fen_off.as<uint32_t>(), mv_off.as<uint32_t>(), ng, false,
                           pos.as<fnnue_pos>(), n, goff.as<uint32_t>(), ng + 1, s);
    if (R.hip != hipSuccess) return hip_fail(R.hip, "device batch builder");
    if (R.err_code) {
      if (int rc = drop(R)) return rc;
      continue;
    }
    if (R.capacity || R.n_out != n || R.n_groups != ng) return fail(FNNUE_E_DEVICE, "batch builder sizes changed");
    int rc = fnnue_eval_groups_device(ctx, pos.as<fnnue_pos>(), goff.as<uint32_t>(), ng, n, FNNUE_GROUP_CHAIN,
                                      psqt.as<int32_t>(), positional.as<int32_t>(), s);
    if (rc == FNNUE_OK) rc = fnnue_ctx_check(ctx);  // synchronises; latched invalid positions
    hgoff.resize(ng + 1);
    HIP_TRY(hipMemcpy(hgoff.data(), goff.p, (ng + 1) * 4, hipMemcpyDeviceToHost), "D2H(group offsets)");
    if (rc == FNNUE_E_POSITION) {
      // A FEN the builder parses but the evaluator cannot (kings, > 32
      // pieces): find the games holding such positions, fail those batches.
      hpos.resize(n);
      HIP_TRY(hipMemcpy(hpos.data(), pos.p, n * sizeof(fnnue_pos), hipMemcpyDeviceToHost), "D2H(positions)");
      std::vector<size_t> keep;
      for (size_t g = 0; g < ng; ++g) {
        bool ok = true;
        for (uint32_t k = hgoff[g]; k < hgoff[g + 1] && ok; ++k) ok = valid_host_pos(hpos[k]);
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
    HIP_TRY(hipMemcpy(hpsqt.data(), psqt.p, n * 4, hipMemcpyDeviceToHost), "D2H(psqt)");
    HIP_TRY(hipMemcpy(hpositional.data(), positional.p, n * 4, hipMemcpyDeviceToHost), "D2H(positional)");
    for (size_t g = 0; g < ng; ++g) {
      const size_t i = live[g];
      const size_t expect = j.off[i + 1] - j.off[i];
      if (hgoff[g + 1] - hgoff[g] != expect) return fail(FNNUE_E_DEVICE, "builder ply count differs from the moves");
      base[i] = hgoff[g];
    }
    return FNNUE_OK;
  }
  return FNNUE_OK;
}

// Move batches: the position after all moves (host replay: one position per
// batch), its legal children evaluated from scratch, best = argmax -v(child).
int fnnue_backend::moves(Job& j, const std::vector<size_t>& games) {
  struct Cand {
    size_t batch;
    std::vector<std::string> uci;
    size_t first;
  };
  std::vector<Cand> cands;
  std::vector<fnnue_pos> kids;
  for (size_t i : games) {
    const fnnue_acquired& a = j.batches[i];
    Board b;
    std::string e;
    if (!board_from_fen(a.position ? a.position : "", b, &e)) {
      j.rc[i] = FNNUE_E_FEN;
      continue;
    }
    bool ok = true;
    std::string tok;
    for (const char* p = a.moves ? a.moves : "";; ++p) {
      if (*p && *p != ' ' && *p != '\t' && *p != '\n' && *p != '\r') {
        tok += *p;
        continue;
      }
      if (!tok.empty()) {
        Move m;
        if (!parse_uci(b, tok.c_str(), m)) {
          ok = false;
          break;
        }
        b.do_move(m);
        tok.clear();
      }
      if (!*p) break;
    }
    if (!ok) {
      j.rc[i] = FNNUE_E_MOVE;
      continue;
    }
    std::vector<Move> ms;
    b.legal_moves(ms);
    if (ms.empty()) {  // mate / stalemate: nothing to play
      j.rc[i] = FNNUE_E_MOVE;
      continue;
    }
    Cand c{i, {}, kids.size()};
    for (const Move& m : ms) {
      Board k = b;
      k.do_move(m);
      kids.push_back(k.pack());
      c.uci.push_back(b.uci(m, b.chess960));
    }
    cands.push_back(std::move(c));
  }
  if (kids.empty()) return FNNUE_OK;
  std::vector<int32_t> ps(kids.size()), po(kids.size());
  if (int rc = fnnue_eval_positions(ctx, kids.data(), kids.size(), ps.data(), po.data())) return rc;
  for (const Cand& c : cands) {
    fnnue_position_response& r = j.out[j.off[c.batch]];
    size_t best = 0;
    int64_t bv = INT64_MIN;
    for (size_t k = 0; k < c.uci.size(); ++k) {
      const size_t x = c.first + k;
      const int64_t v = -(((int64_t)ps[x] + po[x]) / 16);  // Stockfish value of the child, negated
      if (v > bv) {
        bv = v;
        best = k;
      }
    }
    const size_t x = c.first + best;
    r.psqt = -ps[x];
    r.positional = -po[x];
    r.score_kind = FNNUE_SCORE_CP;
    r.score = bv * 100 / norm;
    r.depth = 1;
    r.nodes = c.uci.size();
    std::strncpy(r.best_move, c.uci[best].c_str(), sizeof(r.best_move) - 1);
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
  std::vector<size_t> ana, mov;
  std::vector<uint8_t> skip(j.off[nb], 0);
  for (size_t i = 0; i < nb; ++i) {
    const fnnue_acquired& a = j.batches[i];
    if (j.rc[i]) continue;
    if (!chess_variant(a.variant) || a.multipv < 0) {  // Fairy-Stockfish (routed by flavour): not this backend
      j.rc[i] = FNNUE_E_ARG;
      continue;
    }
    const uint32_t n = j.off[i + 1] - j.off[i];
    if (a.work == FNNUE_WORK_MOVE) {
      mov.push_back(i);
      continue;
    }
    uint32_t live = n;
    for (size_t k = 0; k < a.nskip; ++k)  // positions.get_mut(skip): out-of-range ids are ignored
      if (a.skip_positions[k] < n && !skip[j.off[i] + a.skip_positions[k]]) {
        skip[j.off[i] + a.skip_positions[k]] = 1;
        --live;
      }
    if (live) ana.push_back(i);  // all skipped: completed without the engine (IncomingError::AllSkipped)
  }
  std::memset(j.out, 0, j.off[nb] * sizeof(fnnue_position_response));
  std::vector<size_t> base(nb, 0);
  int rc = analysis(j, ana, base);
  if (rc == FNNUE_OK) rc = moves(j, mov);
  if (rc) {
    j.ret = rc;
    j.err = g_err;
    return;
  }
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  uint64_t nodes = 0;
  for (size_t i = 0; i < nb; ++i) {
    if (j.rc[i]) continue;
    if (j.batches[i].work == FNNUE_WORK_MOVE) {
      nodes += j.out[j.off[i]].nodes;
      continue;
    }
    for (uint32_t k = j.off[i]; k < j.off[i + 1]; ++k) nodes += skip[k] ? 0 : 1;
  }
  const uint64_t ms = (uint64_t)(sec * 1e3);
  const uint32_t nps = sec > 0 ? (uint32_t)std::min(4.0e9, (double)nodes / sec) : 0;
  for (size_t i = 0; i < nb; ++i) {
    if (j.rc[i]) continue;
    const bool is_move = j.batches[i].work == FNNUE_WORK_MOVE;
    for (uint32_t k = j.off[i]; k < j.off[i + 1]; ++k) {
      fnnue_position_response& r = j.out[k];
      r.position_id = k - j.off[i];
      r.time_ms = ms;
      r.nps = nps;
      if (is_move) continue;  // filled by moves()
      if (skip[k]) {
        r.skipped = 1;
        continue;
      }
      const size_t x = base[i] + r.position_id;
      r.matrix = j.batches[i].multipv > 0 ? 1 : 0;  // Work::matrix_wanted: multipv is Some
      r.psqt = hpsqt[x];
      r.positional = hpositional[x];
      r.score_kind = FNNUE_SCORE_CP;
      r.score = to_cp(r.psqt, r.positional, norm);
      r.depth = 0;
      r.nodes = 1;
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

int fnnue_backend_channel(const fnnue_net* net, int device, const fnnue_backend_init* init, fnnue_backend** out) {
  if (!net || !out) return fail(FNNUE_E_ARG, "null argument");
  *out = nullptr;
  int variant = 0;
  if (int rc = fnnue_net_variant(net, &variant)) return rc;
  if (variant != 0) return fail(FNNUE_E_ARCH, "the backend evaluates standard chess: a chess (HalfKAv2_hm) net");
  if (init && init->normalize_to_pawn < 0) return fail(FNNUE_E_ARG, "normalize_to_pawn must be positive");
  fnnue_backend* b = nullptr;
  try {
    b = new fnnue_backend();
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  if (init && init->normalize_to_pawn > 0) b->norm = init->normalize_to_pawn;
  if (int rc = fnnue_ctx_create(net, device, &b->ctx)) {
    delete b;
    return rc;
  }
  try {
    b->th = std::thread([b] {
      DeviceGuard g(b->ctx->device);
      b->loop();
    });
  } catch (const std::system_error&) {
    fnnue_ctx_free(b->ctx);
    delete b;
    return fail(FNNUE_E_OOM, "could not start the actor thread");
  }
  *out = b;
  return FNNUE_OK;
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
    DeviceGuard g(b->ctx->device);
    for (DevBuf* d : {&b->text, &b->fen_off, &b->mv_off, &b->pos, &b->goff, &b->psqt, &b->positional}) d->release();
  }
  fnnue_ctx_free(b->ctx);
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
