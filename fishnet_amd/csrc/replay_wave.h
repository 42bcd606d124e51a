// replay_wave.h — the batch builder's game replay, one 64-lane wave per game
// (builder.hip: chess, vbuilder.hip: crazyhouse / atomic).
//
// IncomingBatch::from_acquired ([ref] src/queue.rs:543-606) parses a root FEN
// and plays every UCI move of the batch, checking each (shakmaty's
// Uci::to_move); the positions after every move are the batch.  Replay is a
// chain (ply k needs ply k - 1), but only a small part of each ply is: what
// the board becomes.  Whether the token names a legal move, and the packed
// record, are per-ply work once the boards are known.  So a wave
//   (a) tokenises the game's move text 64 characters at a time (lane =
//       character: token starts by ballot, each starting lane decodes its
//       token into a move code),
//   (b) plays up to 64 moves in a row: interprets each code on the current
//       board (castling / en passant / promotion / drop — no move generation)
//       and applies it; every lane runs this wave-uniform chain, lane 0 keeps
//       each board in LDS,
//   (c) checks in parallel, lane j for move j, that the token names exactly
//       the move (b) applied — the rules' match over the legal moves of the
//       board before it (the same test the one-thread-per-ply host replay
//       makes) — and packs the board after it into the output record,
// and repeats until the game's text is consumed.  The first move whose check
// fails ends the game with a latched error (the batch fails: PositionFailed);
// records after it (inside the game's own range) are meaningless, the game
// is dropped.  The last board gets the game-end flags
// (no legal move / check / exploded king), its legal-move search split over
// the lanes by from-square.
//
// Output offsets are the host's (ply_off: 1 + moves per game, counted with the
// same whitespace rule), so no sizing pass or read-back is needed; a game
// whose token count differs latches kBuildErrCount and writes nothing outside
// its own range.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "builder.h"

namespace fnnue {
namespace replay {

// Token codes: bits 0-5 from, 6-11 to, 12-14 promotion / drop piece type,
// bit 15 drop, bit 31 malformed (no legal move can match it).
constexpr uint32_t kTokBad = 1u << 31, kTokDrop = 1u << 15;
__device__ __forceinline__ uint32_t tok_from(uint32_t c) { return c & 63; }
__device__ __forceinline__ uint32_t tok_to(uint32_t c) { return (c >> 6) & 63; }
__device__ __forceinline__ uint32_t tok_piece(uint32_t c) { return (c >> 12) & 7; }

__device__ __forceinline__ int tok_sq(char f, char r) {
  return (f >= 'a' && f <= 'h' && r >= '1' && r <= '8') ? (r - '1') * 8 + (f - 'a') : -1;
}

__device__ __forceinline__ bool space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

__device__ __forceinline__ void lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lane `l`'s value of v, l wave-uniform (a scalar register read).
__device__ __forceinline__ uint32_t lane_value(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int l) {
  return (uint64_t)lane_value((uint32_t)v, l) | (uint64_t)lane_value((uint32_t)(v >> 32), l) << 32;
}

// v held in vector registers: the compiler treats a value read from one LDS
// address by every lane as uniform and moves it to scalar registers, which
// the per-lane move generation around it then exhausts (spilling to lanes).
template <class T>
__device__ __forceinline__ T in_vgprs(const T& v) {
  static_assert(sizeof(T) % 4 == 0, "32-bit words");
  uint32_t w[sizeof(T) / 4];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (unsigned i = 0; i < sizeof(T) / 4; ++i) asm volatile("" : "+v"(w[i]));
  T out;
  __builtin_memcpy(&out, w, sizeof(T));
  return out;
}

// A wave-uniform copy of a trivially copyable value: every 32-bit word read
// from the first active lane.
template <class T>
__device__ __forceinline__ T first_lane(const T& v) {
  static_assert(sizeof(T) % 4 == 0, "32-bit words");
  uint32_t w[sizeof(T) / 4];
  __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
  for (unsigned i = 0; i < sizeof(T) / 4; ++i) w[i] = __builtin_amdgcn_readfirstlane(w[i]);
  T out;
  __builtin_memcpy(&out, w, sizeof(T));
  return out;
}

__device__ __forceinline__ void latch(uint32_t* err, uint32_t code, uint32_t game, uint32_t ply) {
  if (atomicCAS(&err[0], 0u, code) == 0u) {
    err[1] = game;
    err[2] = ply;
  }
}

// A failing game: the error word names the first one (err[0..2]); the game's
// own flag byte says that it failed and why (kFinalFailed | code), so that a
// caller drops every failing game of a launch in one pass.
__device__ __forceinline__ void fail_game(uint32_t* err, uint8_t* final, uint32_t code, uint32_t game, uint32_t ply) {
  latch(err, code, game, ply);
  if (final) final[game] = (uint8_t)(kFinalFailed | code);
}

constexpr int kTokRing = 128;  // pending move codes (<= 63 left + 32 new per 64 characters)
constexpr int kTxt = 2048;     // move text staged in LDS at a time

// Bit k of every byte of a 64-byte board snapshot (byte s = square s), as a
// bitboard: the lane-parallel form of a board the chain keeps, turned back
// into bitboards by each checking lane.
__device__ __forceinline__ uint64_t byte_plane(const uint32_t (&w)[16], int k) {
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint32_t x = (w[i] >> k) & 0x01010101u;
    x |= x >> 7;
    x |= x >> 14;
    x &= 0xFu;  // bit j = byte j of dword i
    if (i < 8) lo |= x << (4 * i);
    else hi |= x << (4 * (i - 8));
  }
  return ((uint64_t)hi << 32) | lo;
}

// The 64 nibbles of fnnue_pos / fnnue_vpos (square s in nibble s) from the
// snapshot's piece codes (low nibble of each byte).
__device__ __forceinline__ void pack_nibbles(const uint32_t (&w)[16], uint32_t (&out)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t a = w[2 * i] & 0x0F0F0F0Fu, c = w[2 * i + 1] & 0x0F0F0F0Fu;
    a = (a | (a >> 4)) & 0x00FF00FFu;
    c = (c | (c >> 4)) & 0x00FF00FFu;
    a = (a | (a >> 8)) & 0xFFFFu;
    c = (c | (c >> 8)) & 0xFFFFu;
    out[i] = a | (c << 16);
  }
}

// Rules (builder.hip ChessRules, vbuilder.hip VariantRules):
//   Board, Move, Pos, Scalars (the board's non-square state, whole dwords)
//   bool parse_fen(const char* text, uint32_t p, uint32_t end, int variant, Board&)
//   const char* start_fen(int variant), uint32_t start_fen_len(int variant), Board start_board(int variant)
//                                                       the standard start (< 64 characters) and its board
//   uint32_t encode(const char* c, int len)             token -> code (kTokBad if malformed)
//   Scalars scalars(const Board&); uint32_t lane_square(const Board&, int sq)
//   Win window(const Scalars&, uint32_t code, uint32_t k, int lane)
//                                                       lane-parallel per window (k moves, lane j's code):
//                                                       what the chain and the checks derive scalars from
//   bool step(Scalars&, const Win&, uint32_t j, uint32_t code, uint32_t& sqv, int lane, uint32_t& mv)
//                                                       one chain step (move j): the move the code names,
//                                                       played on the lane bytes; mv = that move packed
//                                                       (false: the code names none, the replay stops)
//   kVary; void fix(Scalars&, const Scalars& s0, const Win&, uint32_t j, bool after)
//                                                       the first kVary words change along the chain and
//                                                       are collected; fix sets the rest for the board
//                                                       before (after) move j
//   void advance(Scalars&, const Win&, uint32_t k)      the scalars after the window's k moves
//   Move unpack_move(uint32_t)
//   Board board_from(const uint32_t (&w)[16], const Scalars&)   snapshot -> board (per lane)
//   Pos pack_from(const uint32_t (&w)[16], const Scalars&)      snapshot -> record (per lane)
//   bool verify(const Board&, const Move&)              the move step() played is legal
//   Pos pack(const Board&)
//   bool any_legal_from(const Board&, int sq, bool drops) legal moves of the piece on sq (+ drops)
//   uint8_t end_flags(const Board&, bool any)             kFinal* of a last position
// ---- phases, shared by the one-wave and the two-wave kernel ----

// The root: the FEN through LDS (TXT), parsed by every lane alike.  One longer
// than kTxt characters (a legal FEN has < 100) is rejected as unparsable.
template <class R>
__device__ __forceinline__ bool root_board(int variant, const char* __restrict__ text, uint32_t f0, uint32_t m0,
                                           char* TXT, int lane, typename R::Board& root) {
  const uint32_t flen = m0 - f0;
  if (flen > (uint32_t)kTxt) return false;
  for (uint32_t i = lane; i < flen; i += 64) TXT[i] = text[f0 + i];
  lds_fence();
  // Most games start from the variant's standard position: recognised by one
  // lane-parallel compare, its board is a constant (the parser's own result,
  // tests/test_gpu_builder.py); any other FEN is parsed.
  const char* sf = R::start_fen(variant);
  const uint32_t sl = R::start_fen_len(variant);
  const bool same = flen == sl && __ballot((uint32_t)lane < sl && TXT[lane] != sf[lane]) == 0;
  if (same) {
    root = R::start_board(variant);
    return true;
  }
  return R::parse_fen(TXT, 0, flen, variant, root);
}

// The tokeniser's place in the game's move text [p, e): TXT holds the text
// from tbase on (kTxt characters at a time, ' ' past the end), TK[0, ntok) the
// pending codes.
struct Tok {
  uint32_t p, tbase, ntok;
  bool staged;
  char prev;  // the character before p
};

// Tokenise 64 characters at a time (lane = character: token starts by
// ballot, each starting lane encodes its token) until `need` codes are
// pending or the text ends.
template <class R>
__device__ __forceinline__ void tokenise(Tok& t, const char* __restrict__ text, uint32_t e, char* TXT, uint32_t* TK,
                                         uint32_t need, int lane) {
  while (t.ntok < need && t.p < e) {
    if (!t.staged || t.p + 64 + 6 > t.tbase + (uint32_t)kTxt) {
      t.tbase = t.p;
      t.staged = true;
      const uint32_t lim = min((uint32_t)kTxt, e - t.tbase + 72);  // the text, then spaces for any token tail
      for (uint32_t q = lane; q < lim; q += 64) TXT[q] = t.tbase + q < e ? text[t.tbase + q] : ' ';
      lds_fence();
    }
    const uint32_t i = t.p - t.tbase + lane;
    const char c = TXT[i];
    const char cprev = (char)__shfl_up((int)c, 1, 64);
    const bool start = !space(c) && space(lane == 0 ? t.prev : cprev);
    const uint64_t starts = __ballot(start);
    if (start) {
      char w[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) w[q] = TXT[i + q];
      int len = 1;
      bool more = true;
#pragma unroll
      for (int q = 1; q < 6; ++q) {
        more = more && !space(w[q]);
        len += more ? 1 : 0;
      }
      const uint32_t code = (len == 4 || len == 5) ? R::encode(w, len) : kTokBad;
      const uint32_t idx = t.ntok + (uint32_t)__popcll(starts & ((1ull << lane) - 1));
      if (idx < (uint32_t)kTokRing) TK[idx] = code;
    }
    t.ntok += (uint32_t)__popcll(starts);
    t.prev = (char)__shfl((int)c, 63, 64);
    t.p += 64;
  }
  lds_fence();
}

// Drops the k codes a window took from the ring.
__device__ __forceinline__ void tok_consume(Tok& t, uint32_t* TK, uint32_t k, int lane) {
  t.ntok -= k;
  uint32_t keep[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const uint32_t src = k + lane + 64 * r;
    keep[r] = src < (uint32_t)kTokRing ? TK[src] : 0;
  }
  lds_fence();
#pragma unroll
  for (int r = 0; r < 2; ++r)
    if ((uint32_t)lane + 64 * r < t.ntok) TK[lane + 64 * r] = keep[r];
  lds_fence();
}

// After the game's last code: is there text left that holds another token?
__device__ __forceinline__ bool tok_extra(Tok& t, const char* __restrict__ text, uint32_t e, int lane) {
  bool extra = t.ntok != 0;
  for (uint32_t q = t.p; q < e && !extra; q += 64) {
    const uint32_t i = q + lane;
    const char c = i < e ? text[i] : ' ';
    const char cprev = (char)__shfl_up((int)c, 1, 64);
    extra = __ballot(!space(c) && space(lane == 0 ? t.prev : cprev)) != 0;
    t.prev = (char)__shfl((int)c, 63, 64);
  }
  return extra;
}

// The chain, wave-uniform: interpret and play the window's k moves (lane j's
// code myc is move j).  The board is lane bytes — lane l holds square l's
// piece (sqv), so a move is a handful of lane-parallel selects — plus the
// wave-uniform scalars.  SNAP[0] gets the window's first board, SNAP[j + 1]
// the board after move j; lane j collects move j packed (mvw) and the kVary
// scalar words after it (scw).  Returns the moves played (< k: a code that
// names no move; that ply fails its check).
template <class R>
__device__ __forceinline__ uint32_t chain(typename R::Scalars& sc, uint32_t& sqv, uint32_t myc, uint32_t k,
                                          const typename R::Win& win, uint32_t (*SNAP)[16], int lane, uint32_t& mvw,
                                          uint32_t (&scw)[R::kVary]) {
  if constexpr (R::kLaneChain) return R::lane_chain(sc, sqv, myc, k, win, SNAP, lane, mvw, scw);
  using Sc = typename R::Scalars;
  constexpr int kScw = sizeof(Sc) / 4;
  reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;
  // the codes are in registers before the chain starts, so the loop head
  // waits for nothing (its only LDS access is the snapshot byte store)
  asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(myc) : "memory");
  mvw = 0;
#pragma unroll
  for (int w = 0; w < R::kVary; ++w) scw[w] = 0;
  uint32_t kplay = k;
  for (uint32_t j = 0; j < k; ++j) {
    const uint32_t code = lane_value(myc, (int)j);
    uint32_t mv;
    if ((code & kTokBad) || !R::step(sc, win, j, code, sqv, lane, mv)) {
      kplay = j;
      break;
    }
    reinterpret_cast<uint8_t*>(SNAP[j + 1])[lane] = (uint8_t)sqv;
    const bool mine = (uint32_t)lane == j;
    mvw = mine ? mv : mvw;
    uint32_t cur[kScw];
    __builtin_memcpy(cur, &sc, sizeof(Sc));
#pragma unroll
    for (int w = 0; w < R::kVary; ++w) scw[w] = mine ? cur[w] : scw[w];
  }
  lds_fence();
  return kplay;
}

// Lane j checks move j of a chained window against the board before it and
// packs the board after it (records o1 + j).  Returns the first failing move
// (>= k: none).
template <class R>
__device__ __forceinline__ uint32_t check(const typename R::Scalars& sc0, const typename R::Win& win,
                                          const uint32_t (*SNAP)[16], uint32_t kplay, uint32_t k, uint32_t mvw,
                                          const uint32_t (&scw)[R::kVary], int lane, typename R::Pos* __restrict__ out,
                                          typename R::Board* __restrict__ states, uint32_t o1) {
  using Sc = typename R::Scalars;
  constexpr int kScw = sizeof(Sc) / 4;
  bool fail = false;
  // scalars before move j: after move j - 1, or the window's own; the words
  // the chain does not collect follow from the window's first
  uint32_t sb[kScw], sa[kScw];
  __builtin_memcpy(sb, &sc0, sizeof(Sc));
  __builtin_memcpy(sa, &sc0, sizeof(Sc));
#pragma unroll
  for (int w = 0; w < R::kVary; ++w) {
    const uint32_t up = (uint32_t)__shfl_up((int)scw[w], 1, 64);
    sb[w] = lane == 0 ? sb[w] : up;
    sa[w] = scw[w];
  }
  if ((uint32_t)lane < kplay) {
    Sc before_sc, after_sc;
    __builtin_memcpy(&before_sc, sb, sizeof(Sc));
    __builtin_memcpy(&after_sc, sa, sizeof(Sc));
    R::fix(before_sc, sc0, win, (uint32_t)lane, false);
    R::fix(after_sc, sc0, win, (uint32_t)lane, true);
    uint32_t wb[16], wa[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      wb[i] = SNAP[lane][i];
      wa[i] = SNAP[lane + 1][i];
    }
    fail = !R::verify(R::board_from(wb, before_sc), R::unpack_move(mvw));
    if (!fail) {
      const uint32_t o = o1 + lane;
      if (out) out[o] = R::pack_from(wa, after_sc);
      if (states) states[o] = R::board_from(wa, after_sc);
    }
  }
  const uint64_t fails = __ballot(fail);
  return fails ? (uint32_t)__builtin_ctzll(fails) : kplay;
}

// kFinal* of the last board (its bytes in B), its legal-move search split
// over the lanes by from-square.
template <class R>
__device__ __forceinline__ uint8_t final_flags(const uint32_t* B, const typename R::Scalars& sc, int lane) {
  uint32_t wl[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) wl[i] = B[i];
  const typename R::Board last = in_vgprs(R::board_from(wl, sc));
  const bool any = __ballot(R::any_legal_from(last, lane, lane == 0)) != 0;
  return R::end_flags(last, any);
}

// ---- one wave per game ----
template <class R>
__global__ __launch_bounds__(64) void replay_wave_kernel(int variant, const char* __restrict__ text,
                                                         const uint32_t* __restrict__ fen_off,
                                                         const uint32_t* __restrict__ mv_off, uint32_t ngames,
                                                         const uint32_t* __restrict__ ply_off,
                                                         typename R::Pos* __restrict__ out,
                                                         typename R::Board* __restrict__ states,
                                                         uint32_t* __restrict__ err, uint8_t* __restrict__ final) {
  using Board = typename R::Board;
  using Sc = typename R::Scalars;
  static_assert(sizeof(Sc) % 4 == 0, "scalars as dwords");
  __shared__ alignas(16) uint32_t SNAP[65][16];  // byte s of SNAP[j] = square s before the window's move j
  __shared__ uint32_t TK[kTokRing];  // pending token codes
  __shared__ char TXT[kTxt];         // move text from tbase on (' ' past the game's end)
  const uint32_t g = blockIdx.x;
  const int lane = threadIdx.x;
  if (g >= ngames) return;
  const uint32_t f0 = fen_off[g], m0 = mv_off[g], e = fen_off[g + 1];
  const uint32_t o0 = ply_off[g], nply = ply_off[g + 1] - o0;
  if (nply == 0) {
    if (lane == 0) fail_game(err, final, kBuildErrCount, g, 0);
    return;
  }
  const uint32_t nmoves = nply - 1;
  Board root;
  if (!root_board<R>(variant, text, f0, m0, TXT, lane, root)) {
    if (lane == 0) fail_game(err, final, kBuildErrFen, g, 0);
    return;
  }
  if (lane == 0) {
    if (out) out[o0] = R::pack(root);
    if (states) states[o0] = root;
  }
  Sc sc = first_lane(R::scalars(root));
  uint32_t sqv = R::lane_square(root, lane);
  // windows of up to 64 moves: tokenise, chain, check
  Tok t{m0, 0u, 0u, false, ' '};
  uint32_t done = 0, bad = 0, bad_ply = 0;
  while (done < nmoves) {
    tokenise<R>(t, text, e, TXT, TK, 64, lane);
    if (t.ntok == 0 || t.ntok > (uint32_t)kTokRing) {  // fewer tokens than the host counted (or a ring overrun)
      bad = kBuildErrCount;
      bad_ply = done + 1;
      break;
    }
    const uint32_t k = min(min(t.ntok, 64u), nmoves - done);
    const uint32_t myc = TK[lane];
    const Sc sc0 = sc;
    const typename R::Win win = R::window(sc, myc, k, lane);
    uint32_t mvw, scw[R::kVary];
    const uint32_t kplay = chain<R>(sc, sqv, myc, k, win, SNAP, lane, mvw, scw);
    const uint32_t first = check<R>(sc0, win, SNAP, kplay, k, mvw, scw, lane, out, states, o0 + done + 1);
    if (first < k) {
      bad = kBuildErrMove;
      bad_ply = done + first + 1;
      break;
    }
    R::advance(sc, win, k);
    done += k;
    tok_consume(t, TK, k, lane);
  }
  if (!bad && tok_extra(t, text, e, lane)) {  // text left after the host's count: more tokens than plies
    bad = kBuildErrCount;
    bad_ply = nmoves + 1;
  }
  if (bad) {
    if (lane == 0) fail_game(err, final, bad, g, bad_ply);
    return;
  }
  if (final) {
    reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;
    lds_fence();
    const uint8_t f = final_flags<R>(SNAP[0], sc, lane);
    if (lane == 0) final[g] = f;
  }
}

// ---- two waves per game (latency: a few games per call) ----
// Wave 0 runs the chain of window s while wave 1 checks window s - 1 and
// tokenises window s + 1 (double-buffered snapshots, codes and chain
// outputs in LDS, one workgroup barrier per window); the last window's check
// runs beside the game-end flags.  Same records, errors and flags as the
// one-wave kernel, in about 0.7 of its time for one game (the chain alone is
// the critical path), but twice its waves: for calls of up to a round of the
// device's wave slots.
template <class R>
struct PairLds {
  using Sc = typename R::Scalars;
  static constexpr int kScw = sizeof(Sc) / 4;
  static constexpr int kWinW = sizeof(typename R::Win) / 4 > 0 ? sizeof(typename R::Win) / 4 : 1;
  alignas(16) uint32_t SNAP[2][65][16];
  uint32_t TKW[2][64];          // the window's codes
  uint32_t MV[2][64];           // chain outputs per lane: move, scalars, Win
  uint32_t SCW[2][R::kVary][64];
  uint32_t WIN[2][kWinW][64];
  uint32_t SC0[2][kScw];        // the window's first scalars
  uint32_t KW[2], KP[2];        // codes, moves played
  uint32_t TK[kTokRing];        // the tokeniser's ring
  uint32_t FIN[16];             // the last board's bytes
  // Control words (windows, count error ply, bad-move code and ply), double
  // buffered by barrier: the copy written before barrier m is slot m & 1,
  // read by both waves right after it; the next writes go to the other slot,
  // so a wave that runs ahead never overwrites what the other still reads.
  uint32_t CTL[2][4];
  char TXT[kTxt];
};

template <class R>
__global__ __launch_bounds__(128) void replay_pair_kernel(int variant, const char* __restrict__ text,
                                                          const uint32_t* __restrict__ fen_off,
                                                          const uint32_t* __restrict__ mv_off, uint32_t ngames,
                                                          const uint32_t* __restrict__ ply_off,
                                                          typename R::Pos* __restrict__ out,
                                                          typename R::Board* __restrict__ states,
                                                          uint32_t* __restrict__ err, uint8_t* __restrict__ final) {
  using Board = typename R::Board;
  using Sc = typename R::Scalars;
  using Win = typename R::Win;
  using L_t = PairLds<R>;
  constexpr int kScw = L_t::kScw, kWinW = L_t::kWinW;
  __shared__ L_t L;
  const uint32_t g = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (g >= ngames) return;
  const uint32_t f0 = fen_off[g], m0 = mv_off[g], e = fen_off[g + 1];
  const uint32_t o0 = ply_off[g], nply = ply_off[g + 1] - o0;
  if (nply == 0) {
    if (threadIdx.x == 0) fail_game(err, final, kBuildErrCount, g, 0);
    return;
  }
  const uint32_t nmoves = nply - 1;
  const uint32_t nw0 = (nmoves + 63) / 64;
  // the control words in registers (wave-uniform): reloaded after every barrier
  uint32_t nw = nw0, cnt_ply = 0, bad = 0, bad_ply = 0;
  auto publish = [&](int slot) {  // lane 0 of the writing wave
    L.CTL[slot][0] = nw;
    L.CTL[slot][1] = cnt_ply;
    L.CTL[slot][2] = bad;
    L.CTL[slot][3] = bad_ply;
  };
  auto reload = [&](int slot) {
    nw = L.CTL[slot][0];
    cnt_ply = L.CTL[slot][1];
    bad = L.CTL[slot][2];
    bad_ply = L.CTL[slot][3];
  };
  // wave 0: the root; wave 1 waits (the FEN goes through TXT, which wave 1
  // then uses for the move text)
  Sc sc;
  uint32_t sqv = 0;
  if (wv == 0) {
    Board root;
    const bool ok = root_board<R>(variant, text, f0, m0, L.TXT, lane, root);
    if (lane == 0) {
      bad = ok ? 0u : kBuildErrFen;
      publish(0);  // barrier 0
      if (ok && out) out[o0] = R::pack(root);
      if (ok && states) states[o0] = root;
    }
    if (ok) {
      sc = first_lane(R::scalars(root));
      sqv = R::lane_square(root, lane);
    }
  }
  __syncthreads();
  reload(0);
  if (bad) {
    if (threadIdx.x == 0) fail_game(err, final, bad, g, 0);
    return;
  }
  // wave 1: the codes of window w (k = its moves, fewer when the text ends:
  // a count error, reported after the earlier windows' checks)
  Tok t{m0, 0u, 0u, false, ' '};
  auto produce = [&](uint32_t w) {
    const uint32_t need = min(64u, nmoves - 64 * w);
    tokenise<R>(t, text, e, L.TXT, L.TK, need, lane);
    const uint32_t got = t.ntok > (uint32_t)kTokRing ? 0u : min(t.ntok, need);  // (0: a ring overrun)
    L.TKW[w & 1][lane] = (uint32_t)lane < got ? L.TK[lane] : 0u;
    lds_fence();
    if (lane == 0) L.KW[w & 1] = got;
    if (got < need) {  // the text ended: this window is the game's last
      cnt_ply = 64 * w + got + 1;
      nw = w + 1;
    } else {
      tok_consume(t, L.TK, got, lane);
      if (w + 1 == nw0 && tok_extra(t, text, e, lane)) cnt_ply = nmoves + 1;
    }
  };
  if (wv == 1) {
    if (nw0 > 0) produce(0);
    if (lane == 0) publish(1);  // barrier 1
  }
  __syncthreads();
  reload(1);
  uint8_t fl = 0;
  for (uint32_t s = 0;; ++s) {
    // nw (as of this iteration's barrier) is the same in both waves
    if (wv == 0) {
      if (s < nw) {
        const uint32_t b = s & 1, k = L.KW[b];
        const uint32_t myc = L.TKW[b][lane];
        const Win win = R::window(sc, myc, k, lane);
        uint32_t sw[kScw];
        __builtin_memcpy(sw, &sc, sizeof(Sc));
        uint32_t mvw, scw[R::kVary];
        const uint32_t kplay = chain<R>(sc, sqv, myc, k, win, L.SNAP[b], lane, mvw, scw);
        L.MV[b][lane] = mvw;
#pragma unroll
        for (int w = 0; w < R::kVary; ++w) L.SCW[b][w][lane] = scw[w];
        uint32_t ww[kWinW] = {};
        if constexpr (sizeof(Win) >= 4) __builtin_memcpy(ww, &win, sizeof(Win));
#pragma unroll
        for (int w = 0; w < kWinW; ++w) L.WIN[b][w][lane] = ww[w];
        if (lane < kScw) {
          uint32_t v = 0;
#pragma unroll
          for (int w = 0; w < kScw; ++w) v = lane == w ? sw[w] : v;
          L.SC0[b][lane] = v;
        }
        if (lane == 0) L.KP[b] = kplay;
        R::advance(sc, win, k);
      } else if (s == nw && final) {
        reinterpret_cast<uint8_t*>(L.FIN)[lane] = (uint8_t)sqv;
        lds_fence();
        fl = final_flags<R>(L.FIN, sc, lane);
      }
    } else {
      const uint32_t nw_s = nw;
      if (s >= 1 && s - 1 < nw_s) {
        const uint32_t w0 = s - 1, b = w0 & 1, k = L.KW[b], kplay = L.KP[b];
        Sc sc0;
        uint32_t sw[kScw];
#pragma unroll
        for (int w = 0; w < kScw; ++w) sw[w] = L.SC0[b][w];
        __builtin_memcpy(&sc0, sw, sizeof(Sc));
        Win win;
        uint32_t ww[kWinW];
#pragma unroll
        for (int w = 0; w < kWinW; ++w) ww[w] = L.WIN[b][w][lane];
        if constexpr (sizeof(Win) >= 4) __builtin_memcpy(&win, ww, sizeof(Win));
        uint32_t scw[R::kVary];
#pragma unroll
        for (int w = 0; w < R::kVary; ++w) scw[w] = L.SCW[b][w][lane];
        const uint32_t first = check<R>(sc0, win, L.SNAP[b], kplay, k, L.MV[b][lane], scw, lane, out, states,
                                        o0 + 64 * w0 + 1);
        if (first < k) {
          bad = kBuildErrMove;
          bad_ply = 64 * w0 + first + 1;
        }
      }
      if (s + 1 < nw_s) produce(s + 1);
      if (lane == 0) publish((int)(s & 1));  // barrier s + 2
    }
    __syncthreads();
    reload((int)(s & 1));
    if (bad || s >= nw) break;
  }
  if (threadIdx.x == 0) {
    if (bad) fail_game(err, final, bad, g, bad_ply);
    else if (cnt_ply) fail_game(err, final, kBuildErrCount, g, cnt_ply);
    else if (final) final[g] = fl;
  }
}

// Two waves per game up to kPairGames games (a call that fits one round of
// wave slots: latency), one wave per game above (throughput).
// FNNUE_REPLAY_PAIR_MAX overrides the bound (A/B only).
constexpr uint32_t kPairGames = 1024;
inline uint32_t pair_games_max() {
  static const uint32_t v = [] {
    const char* e = std::getenv("FNNUE_REPLAY_PAIR_MAX");
    return e ? (uint32_t)std::strtoul(e, nullptr, 10) : kPairGames;
  }();
  return v;
}
template <class R>
hipError_t launch_replay(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                         uint32_t ngames, const uint32_t* d_ply_off, typename R::Pos* d_out,
                         typename R::Board* d_states, uint32_t* d_err, uint8_t* d_final, hipStream_t s) {
  if (!ngames) return hipSuccess;
  if (ngames <= pair_games_max())
    hipLaunchKernelGGL(replay_pair_kernel<R>, dim3(ngames), dim3(128), 0, s, variant, d_text, d_fen_off, d_mv_off,
                       ngames, d_ply_off, d_out, d_states, d_err, d_final);
  else
    hipLaunchKernelGGL(replay_wave_kernel<R>, dim3(ngames), dim3(64), 0, s, variant, d_text, d_fen_off, d_mv_off,
                       ngames, d_ply_off, d_out, d_states, d_err, d_final);
  return hipGetLastError();
}

}  // namespace replay
}  // namespace fnnue
