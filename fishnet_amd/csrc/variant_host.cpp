// variant_host.cpp — host side of the Fairy-Stockfish variant path: FEN with
// crazyhouse holdings -> fnnue_vpos, and seeded random walks that produce
// variant positions for tests and the bench (include/fnnue.h).
#include <cstring>
#include <thread>
#include <string>
#include <vector>

#include "board.h"
#include "builder.h"
#include "internal.h"
#include "vboard.h"

using namespace fnnue;
using namespace fnnue::detail;

namespace {

struct VState {
  uint8_t b[64];
  int stm;
  uint8_t hand[10];  // white P N B R Q, black P N B R Q
};

fnnue_vpos pack_v(const VState& v) {
  fnnue_vpos p;
  std::memset(&p, 0, sizeof p);
  for (int s = 0; s < 64; ++s) p.sq[s >> 1] |= (uint8_t)(v.b[s] << (4 * (s & 1)));
  p.stm = (uint8_t)v.stm;
  std::memcpy(p.hand, v.hand, 10);
  return p;
}

void start_position(VState& v) {
  std::memset(&v, 0, sizeof v);
  const int back[8] = {4, 2, 3, 5, 6, 3, 2, 4};
  for (int f = 0; f < 8; ++f) {
    v.b[f] = (uint8_t)back[f];
    v.b[8 + f] = 1;
    v.b[48 + f] = 9;
    v.b[56 + f] = (uint8_t)(back[f] | 8);
  }
}

bool near_king(const VState& v, int sq) {
  for (int dr = -1; dr <= 1; ++dr)
    for (int df = -1; df <= 1; ++df) {
      const int r = (sq >> 3) + dr, f = (sq & 7) + df;
      if (r < 0 || r > 7 || f < 0 || f > 7) continue;
      if ((v.b[r * 8 + f] & 7) == 6) return true;
    }
  return false;
}

// One pseudo-legal step (no chess movement rules: any own piece to any square
// not holding an own piece or a king; kings step to a neighbour).  Feature-wise
// it exercises exactly what real play does: moves, captures, promotions and,
// per variant, pockets (crazyhouse) or explosions (atomic).
void random_step(VState& v, uint64_t& st, int variant) {
  const int us = v.stm;
  uint8_t* hand = v.hand + 5 * us;
  int htot = 0;
  for (int i = 0; i < 5; ++i) htot += hand[i];
  if (variant == kVariantCrazyhouse && htot && splitmix64(st) % 3 == 0) {
    int k = (int)(splitmix64(st) % (uint64_t)htot), pt = 0;
    while (k >= hand[pt]) k -= hand[pt++];
    for (int tries = 0; tries < 64; ++tries) {
      const int sq = (int)(splitmix64(st) % 64);
      if (v.b[sq] || (pt == 0 && (sq < 8 || sq >= 56))) continue;
      v.b[sq] = (uint8_t)((us << 3) | (pt + 1));
      --hand[pt];
      v.stm ^= 1;
      return;
    }
  }
  int own[32], n = 0;
  for (int s = 0; s < 64; ++s)
    if (v.b[s] && (v.b[s] >> 3) == us) own[n++] = s;
  for (int tries = 0; tries < 64; ++tries) {
    const int from = own[splitmix64(st) % (uint64_t)n];
    const int pc = v.b[from];
    int to;
    if ((pc & 7) == 6) {
      const int dr = (int)(splitmix64(st) % 3) - 1, df = (int)(splitmix64(st) % 3) - 1;
      const int r = (from >> 3) + dr, f = (from & 7) + df;
      if ((!dr && !df) || r < 0 || r > 7 || f < 0 || f > 7) continue;
      to = r * 8 + f;
    } else {
      to = (int)(splitmix64(st) % 64);
    }
    const int cap = v.b[to];
    if (to == from || (cap && (cap >> 3) == us) || (cap & 7) == 6) continue;
    int moved = pc;
    if ((pc & 7) == 1 && (to < 8 || to >= 56)) moved = (us << 3) | 5;  // promotion to a queen
    if (cap && variant == kVariantCrazyhouse) {
      const int t = (cap & 7) - 1;  // captured piece joins the capturer's hand
      if (hand[t] >= kVHandSlots) continue;
      ++hand[t];
    }
    if (cap && variant == kVariantAtomic) {
      if ((pc & 7) == 6 || near_king(v, to)) continue;  // an explosion never takes a king here
      v.b[from] = 0;
      v.b[to] = 0;  // the capturer explodes with its victim
      for (int dr = -1; dr <= 1; ++dr)
        for (int df = -1; df <= 1; ++df) {
          const int r = (to >> 3) + dr, f = (to & 7) + df;
          if (r < 0 || r > 7 || f < 0 || f > 7) continue;
          uint8_t& x = v.b[r * 8 + f];
          if (x && (x & 7) != 1) x = 0;  // pawns survive
        }
      v.stm ^= 1;
      return;
    }
    v.b[from] = 0;
    v.b[to] = (uint8_t)moved;
    v.stm ^= 1;
    return;
  }
  v.stm ^= 1;  // nothing found: pass
}

// fnnue_vpos of a parsed board, with the evaluator's limits checked on the
// host: at most 32 pieces on board and in hand, at most 16 of a type in a hand.
int pack_checked(const vb::VBoard& b, fnnue_vpos* out) {
  int n = vb::vpopcnt(vb::occupied(b));
  for (int c = 0; c < 2; ++c)
    for (int t = 0; t < 5; ++t) {
      if (vb::in_hand(b, c, t + 1) > kVHandSlots) return fail(FNNUE_E_FEN, "more than 16 pieces of a type in hand");
      n += vb::in_hand(b, c, t + 1);
    }
  if (n > 32) return fail(FNNUE_E_FEN, "more than 32 pieces on board and in hand");
  *out = vb::pack(b);
  return FNNUE_OK;
}


bool valid_variant(int variant) { return variant == FNNUE_VARIANT_CRAZYHOUSE || variant == FNNUE_VARIANT_ATOMIC; }

uint64_t vperft(const vb::VBoard& b, int depth) {
  if (depth == 0) return 1;
  uint64_t n = 0;
  vb::for_each_legal(b, [&](const vb::VMove& m) -> bool {
    if (depth == 1) {
      ++n;
    } else {
      vb::VBoard c = b;
      vb::do_move(c, m);
      n += vperft(c, depth - 1);
    }
    return true;
  });
  return n;
}

// Replays `moves` from `fen`: f(board) after the root and after every move.
template <class F>
int vreplay(int variant, const char* fen, const char* moves, F&& f) {
  vb::VBoard b;
  if (!vb::parse_fen(fen, 0, (uint32_t)std::strlen(fen), variant, b))
    return fail(FNNUE_E_FEN, std::string("unparsable variant FEN: ") + fen);
  if (int rc = f(b)) return rc;
  if (!moves) return FNNUE_OK;
  const uint32_t end = (uint32_t)std::strlen(moves);
  uint32_t p = 0, st;
  int len, ply = 0;
  while ((len = vb::next_token(moves, p, end, st)) > 0) {
    ++ply;
    vb::VMove m;
    if (!vb::match_uci(b, moves + st, len, m))
      return fail(FNNUE_E_MOVE, "illegal move " + std::string(moves + st, (size_t)len) + " at ply " + std::to_string(ply));
    vb::do_move(b, m);
    if (int rc = f(b)) return rc;
  }
  return FNNUE_OK;
}

}  // namespace

extern "C" {

int fnnue_vpos_from_fen(int variant, const char* fen, fnnue_vpos* out) {
  if (!fen || !out) return fail(FNNUE_E_ARG, "null argument");
  if (variant != FNNUE_VARIANT_CRAZYHOUSE && variant != FNNUE_VARIANT_ATOMIC)
    return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  vb::VBoard b;
  if (!vb::parse_fen(fen, 0, (uint32_t)std::strlen(fen), variant, b))
    return fail(FNNUE_E_FEN, std::string("unparsable ") + (variant == FNNUE_VARIANT_CRAZYHOUSE ? "crazyhouse" : "atomic") +
                                 " FEN (placement, holdings, side to move, one king per side): " + fen);
  return pack_checked(b, out);
}

int fnnue_random_vpositions(uint64_t seed, int variant, size_t count, uint32_t max_plies, int mode, fnnue_vpos* out,
                            size_t cap, uint32_t* off, size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  if (variant != FNNUE_VARIANT_CRAZYHOUSE && variant != FNNUE_VARIANT_ATOMIC)
    return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  if (mode != FNNUE_PLAYOUT_FINAL && mode != FNNUE_PLAYOUT_PLIES) return fail(FNNUE_E_ARG, "bad mode");
  std::vector<fnnue_vpos> res;
  std::vector<uint32_t> offs{0};
  try {
    for (size_t i = 0; i < count; ++i) {
      uint64_t st = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
      const uint32_t L = (uint32_t)(splitmix64(st) % ((uint64_t)max_plies + 1));
      VState v;
      start_position(v);
      if (mode == FNNUE_PLAYOUT_PLIES) res.push_back(pack_v(v));
      for (uint32_t k = 0; k < L; ++k) {
        random_step(v, st, variant);
        if (mode == FNNUE_PLAYOUT_PLIES) res.push_back(pack_v(v));
      }
      if (mode == FNNUE_PLAYOUT_FINAL) res.push_back(pack_v(v));
      else offs.push_back((uint32_t)res.size());
    }
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  *n_out = res.size();
  *n_groups = offs.size() - 1;
  if (!out || cap < res.size()) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  if (mode == FNNUE_PLAYOUT_PLIES && (!off || off_cap < offs.size())) return fail(FNNUE_E_CAPACITY, "offset buffer too small");
  std::memcpy(out, res.data(), res.size() * sizeof(fnnue_vpos));
  if (mode == FNNUE_PLAYOUT_PLIES) std::memcpy(off, offs.data(), offs.size() * sizeof(uint32_t));
  return FNNUE_OK;
}

int fnnue_game_vpositions(int variant, const char* fen, const char* moves, fnnue_vpos* out, size_t cap,
                          size_t* n_out) {
  if (!fen || !n_out) return fail(FNNUE_E_ARG, "null argument");
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  std::vector<fnnue_vpos> res;
  const int rc = vreplay(variant, fen, moves, [&](const vb::VBoard& b) {
    res.push_back(vb::pack(b));
    return (int)FNNUE_OK;
  });
  if (rc) return rc;
  *n_out = res.size();
  if (!out || cap < res.size()) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  std::memcpy(out, res.data(), res.size() * sizeof(fnnue_vpos));
  return FNNUE_OK;
}

int fnnue_game_vchildren(int variant, const char* fen, const char* moves, fnnue_vpos* out, size_t cap, uint32_t* off,
                         size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!fen || !n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  std::vector<fnnue_vpos> res;
  std::vector<uint32_t> offs{0};
  const int rc = vreplay(variant, fen, moves, [&](const vb::VBoard& b) {
    res.push_back(vb::pack(b));
    vb::for_each_legal(b, [&](const vb::VMove& m) -> bool {
      vb::VBoard c = b;
      vb::do_move(c, m);
      res.push_back(vb::pack(c));
      return true;
    });
    offs.push_back((uint32_t)res.size());
    return (int)FNNUE_OK;
  });
  if (rc) return rc;
  *n_out = res.size();
  *n_groups = offs.size() - 1;
  if (!out || !off || cap < res.size() || off_cap < offs.size()) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  std::memcpy(out, res.data(), res.size() * sizeof(fnnue_vpos));
  std::memcpy(off, offs.data(), offs.size() * sizeof(uint32_t));
  return FNNUE_OK;
}

int fnnue_game_end(int variant, const char* fen, const char* moves, int* flags) {
  if (!fen || !flags) return fail(FNNUE_E_ARG, "null argument");
  *flags = 0;
  if (variant == FNNUE_VARIANT_CHESS) return game_end_chess(fen, moves, flags);
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  vb::VBoard last{};
  const int rc = vreplay(variant, fen, moves, [&](const vb::VBoard& b) {
    last = b;
    return (int)FNNUE_OK;
  });
  if (rc) return rc;
  *flags = vb::final_state(last);
  return FNNUE_OK;
}

int fnnue_vperft(int variant, const char* fen, int depth, uint64_t* nodes) {
  if (!fen || !nodes || depth < 0) return fail(FNNUE_E_ARG, "bad argument");
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  vb::VBoard b;
  if (!vb::parse_fen(fen, 0, (uint32_t)std::strlen(fen), variant, b)) return fail(FNNUE_E_FEN, "unparsable variant FEN");
  *nodes = vperft(b, depth);
  return FNNUE_OK;
}

int fnnue_random_vgame(uint64_t seed, int variant, const char* fen, uint32_t plies, char* moves, size_t cap,
                       size_t* len) {
  if (!fen || !len) return fail(FNNUE_E_ARG, "null argument");
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  vb::VBoard b;
  if (!vb::parse_fen(fen, 0, (uint32_t)std::strlen(fen), variant, b)) return fail(FNNUE_E_FEN, "unparsable variant FEN");
  uint64_t st = seed;
  std::string out;
  std::vector<vb::VMove> legal;
  for (uint32_t i = 0; i < plies; ++i) {
    if (vb::king_sq(b, 0) < 0 || vb::king_sq(b, 1) < 0) break;  // atomic: a king exploded
    legal.clear();
    vb::for_each_legal(b, [&](const vb::VMove& m) -> bool {
      legal.push_back(m);
      return true;
    });
    if (legal.empty()) break;
    const vb::VMove m = legal[splitmix64(st) % legal.size()];
    if (!out.empty()) out += ' ';
    out += vb::vuci(b, m);
    vb::do_move(b, m);
  }
  *len = out.size();
  if (!moves || cap < out.size() + 1) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  std::memcpy(moves, out.c_str(), out.size() + 1);
  return FNNUE_OK;
}

int fnnue_random_vgames(uint64_t seed, int variant, size_t count, uint32_t max_plies, int threads, fnnue_vpos* out,
                        size_t cap, uint32_t* off, size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  const char* start = variant == FNNUE_VARIANT_CRAZYHOUSE ? "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1"
                                                          : "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1";
  vb::VBoard root;
  vb::parse_fen(start, 0, (uint32_t)std::strlen(start), variant, root);
  // Game i: L ~ U[0, max_plies] uniformly random legal moves from (seed, i),
  // stopping when no move is left or a king exploded (that last position is
  // kept: an atomic game's final ply, which the evaluator answers with (0, 0)
  // and the backend with mate 0).  Independent of the thread count.
  struct Part {
    std::vector<fnnue_vpos> pos;
    std::vector<uint32_t> sizes;
  };
  std::vector<Part> parts(threads);
  auto work = [&](int t) {
    const size_t b = count * t / threads, e = count * (t + 1) / threads;
    Part& P = parts[t];
    std::vector<vb::VMove> legal;
    for (size_t i = b; i < e; ++i) {
      uint64_t st = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
      const uint32_t L = (uint32_t)(splitmix64(st) % ((uint64_t)max_plies + 1));
      vb::VBoard v = root;
      const size_t before = P.pos.size();
      P.pos.push_back(vb::pack(v));
      for (uint32_t k = 0; k < L; ++k) {
        legal.clear();
        vb::for_each_legal(v, [&](const vb::VMove& m) -> bool {
          legal.push_back(m);
          return true;
        });
        if (legal.empty()) break;
        vb::do_move(v, legal[splitmix64(st) % legal.size()]);
        P.pos.push_back(vb::pack(v));
        if (vb::king_sq(v, 0) < 0 || vb::king_sq(v, 1) < 0) break;
      }
      P.sizes.push_back((uint32_t)(P.pos.size() - before));
    }
  };
  try {
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  } catch (const std::exception& ex) {
    return fail(FNNUE_E_OOM, std::string("variant game generation failed: ") + ex.what());
  }
  size_t total = 0, groups = 0;
  for (auto& P : parts) {
    total += P.pos.size();
    groups += P.sizes.size();
  }
  *n_out = total;
  *n_groups = groups;
  if (!out || cap < total) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  if (!off || off_cap < groups + 1) return fail(FNNUE_E_CAPACITY, "offset buffer too small");
  size_t k = 0, gk = 0;
  off[0] = 0;
  for (auto& P : parts) {
    std::memcpy(out + k, P.pos.data(), P.pos.size() * sizeof(fnnue_vpos));
    for (uint32_t sz : P.sizes) {
      off[gk + 1] = off[gk] + sz;
      ++gk;
    }
    k += P.pos.size();
  }
  return FNNUE_OK;
}

int fnnue_build_vbatch_device(fnnue_ctx* ctx, int variant, const char* d_text, const uint32_t* d_fen_off,
                              const uint32_t* d_moves_off, size_t ngames, int mode, fnnue_vpos* d_out, size_t cap,
                              uint32_t* d_off, size_t off_cap, size_t* n_out, size_t* n_groups, void* stream) {
  if (!ctx || !n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  if (!valid_variant(variant)) return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  if (mode != FNNUE_PLAYOUT_PLIES && mode != FNNUE_PLAYOUT_CHILDREN) return fail(FNNUE_E_ARG, "bad build mode");
  *n_out = *n_groups = 0;
  if (ngames == 0) return FNNUE_OK;
  if (!d_text || !d_fen_off || !d_moves_off) return fail(FNNUE_E_ARG, "null buffer");
  if (ngames > (1u << 26)) return fail(FNNUE_E_ARG, "too many games");
  DeviceGuard g(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const BuildResult R = build_vbatch_device(variant, d_text, d_fen_off, d_moves_off, (uint32_t)ngames,
                                            mode == FNNUE_PLAYOUT_CHILDREN, d_out, cap, d_off, off_cap, s,
                                            ctx->bscratch);
  if (R.hip != hipSuccess) return hip_fail(R.hip, "device variant batch builder");
  *n_out = R.n_out;
  *n_groups = R.n_groups;
  if (R.err_code == kBuildErrFen) return fail(FNNUE_E_FEN, "unparsable variant FEN in game " + std::to_string(R.err_game));
  if (R.err_code == kBuildErrMove)
    return fail(FNNUE_E_MOVE, "illegal move at ply " + std::to_string(R.err_ply) + " of game " +
                                  std::to_string(R.err_game));
  if (R.capacity) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  return FNNUE_OK;
}

int fnnue_build_vbatch(fnnue_ctx* ctx, int variant, const char* text, size_t text_len, const uint32_t* fen_off,
                       const uint32_t* moves_off, size_t ngames, int mode, fnnue_vpos* out, size_t cap, uint32_t* off,
                       size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!ctx || !n_out || !n_groups || (ngames && (!text || !fen_off || !moves_off)))
    return fail(FNNUE_E_ARG, "null argument");
  *n_out = *n_groups = 0;
  if (ngames == 0) return FNNUE_OK;
  if (fen_off[ngames] > text_len) return fail(FNNUE_E_ARG, "offsets exceed the text");
  for (size_t i = 0; i < ngames; ++i)
    if (fen_off[i] > moves_off[i] || moves_off[i] > fen_off[i + 1]) return fail(FNNUE_E_ARG, "offsets out of order");
  DeviceGuard g(ctx->device);
  const size_t text_bytes = (text_len + 255) / 256 * 256;
  const size_t fo_bytes = (ngames + 1) * 4, mo_bytes = ngames * 4;
  int rc = ensure_builder_input(ctx, text_bytes + fo_bytes + mo_bytes);
  if (rc) return rc;
  char* d_text = ctx->d_btext;
  uint32_t* d_fo = reinterpret_cast<uint32_t*>(d_text + text_bytes);
  uint32_t* d_mo = d_fo + (ngames + 1);
  hipStream_t s = ctx->stream;
  HIP_TRY(hipMemcpyAsync(d_text, text, text_len, hipMemcpyHostToDevice, s), "H2D");
  HIP_TRY(hipMemcpyAsync(d_fo, fen_off, fo_bytes, hipMemcpyHostToDevice, s), "H2D");
  HIP_TRY(hipMemcpyAsync(d_mo, moves_off, mo_bytes, hipMemcpyHostToDevice, s), "H2D");
  rc = fnnue_build_vbatch_device(ctx, variant, d_text, d_fo, d_mo, ngames, mode, nullptr, 0, nullptr, 0, n_out,
                                 n_groups, s);
  if (rc != FNNUE_E_CAPACITY) return rc;  // sizing pass
  if (!out || !off || cap < *n_out || off_cap < *n_groups + 1) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  if ((rc = ensure_stage(ctx, *n_out, *n_groups + 1))) return rc;
  fnnue_vpos* d_out = reinterpret_cast<fnnue_vpos*>(ctx->d_pos);  // staging sized for fnnue_vpos
  uint32_t* d_off = ctx->d_off;
  rc = fnnue_build_vbatch_device(ctx, variant, d_text, d_fo, d_mo, ngames, mode, d_out, *n_out, d_off, *n_groups + 1,
                                 n_out, n_groups, s);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, d_out, *n_out * sizeof(fnnue_vpos), hipMemcpyDeviceToHost, s), "D2H");
  HIP_TRY(hipMemcpyAsync(off, d_off, (*n_groups + 1) * 4, hipMemcpyDeviceToHost, s), "D2H");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return FNNUE_OK;
}

}  // extern "C"
