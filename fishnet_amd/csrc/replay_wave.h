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
  constexpr int kScw = sizeof(Sc) / 4;
  static_assert(sizeof(Sc) % 4 == 0, "scalars as dwords");
  __shared__ uint32_t SNAP[65][16];  // byte s of SNAP[j] = square s before the window's move j
  __shared__ uint32_t TK[kTokRing];  // pending token codes
  __shared__ char TXT[kTxt];         // move text from tbase on (' ' past the game's end)
  const uint32_t g = blockIdx.x;
  const int lane = threadIdx.x;
  if (g >= ngames) return;
  const uint32_t f0 = fen_off[g], m0 = mv_off[g], e = fen_off[g + 1];
  const uint32_t o0 = ply_off[g], nply = ply_off[g + 1] - o0;
  if (nply == 0) {
    if (lane == 0) latch(err, kBuildErrCount, g, 0);
    return;
  }
  const uint32_t nmoves = nply - 1;

  // ---- root: FEN through LDS, parsed by every lane alike ----
  Board root;
  bool ok;
  {
    // The FEN goes through the move-text buffer (free until tokenising
    // starts); one longer than it (kTxt characters: a legal FEN has < 100)
    // is rejected as unparsable.
    const uint32_t flen = m0 - f0;
    ok = flen <= (uint32_t)kTxt;
    if (ok) {
      for (uint32_t i = lane; i < flen; i += 64) TXT[i] = text[f0 + i];
      lds_fence();
      // Most games start from the variant's standard position: recognised
      // by one lane-parallel compare, its board is a constant (the parser's
      // own result, tests/test_gpu_builder.py); any other FEN is parsed.
      const char* sf = R::start_fen(variant);
      const uint32_t sl = R::start_fen_len(variant);
      const bool same = flen == sl && __ballot((uint32_t)lane < sl && TXT[lane] != sf[lane]) == 0;
      if (same) root = R::start_board(variant);
      else ok = R::parse_fen(TXT, 0, flen, variant, root);
    }
  }
  if (!ok) {
    if (lane == 0) latch(err, kBuildErrFen, g, 0);
    return;
  }
  if (lane == 0) {
    if (out) out[o0] = R::pack(root);
    if (states) states[o0] = root;
  }
  // The chain keeps the board as lane bytes — lane l holds square l's piece
  // (sqv), so a move is a handful of lane-parallel selects — plus the
  // wave-uniform scalars (side to move, castling rooks, en passant, pockets).
  // Each ply's board is one byte per lane into SNAP; the checking lanes turn
  // snapshots back into bitboards.
  Sc sc = first_lane(R::scalars(root));
  uint32_t sqv = R::lane_square(root, lane);
  reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;

  // ---- windows of up to 64 moves ----
  uint32_t p = m0;   // next text character to tokenise
  uint32_t tbase = 0;  // text offset of TXT[0]
  bool staged = false;
  char prev = ' ';   // the character before p
  uint32_t ntok = 0; // pending codes in TK[0 .. ntok)
  uint32_t done = 0; // moves played and checked
  uint32_t bad = 0;  // kBuildErr* of this game
  uint32_t bad_ply = 0;
  while (done < nmoves) {
    // (a) tokenise until a full window is pending or the text ends; the
    // characters come from an LDS copy of the move text (kTxt at a time,
    // loaded with independent loads), so a token's tail is an LDS read
    while (ntok < 64 && p < e) {
      if (!staged || p + 64 + 6 > tbase + (uint32_t)kTxt) {
        tbase = p;
        staged = true;
        const uint32_t lim = min((uint32_t)kTxt, e - tbase + 72);  // the text, then spaces for any token tail
        for (uint32_t q = lane; q < lim; q += 64) TXT[q] = tbase + q < e ? text[tbase + q] : ' ';
        lds_fence();
      }
      const uint32_t i = p - tbase + lane;
      const char c = TXT[i];
      const char cprev = (char)__shfl_up((int)c, 1, 64);
      const bool start = !space(c) && space(lane == 0 ? prev : cprev);
      const uint64_t starts = __ballot(start);
      if (start) {
        char t[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) t[q] = TXT[i + q];
        int len = 1;
        bool more = true;
#pragma unroll
        for (int q = 1; q < 6; ++q) {
          more = more && !space(t[q]);
          len += more ? 1 : 0;
        }
        const uint32_t code = (len == 4 || len == 5) ? R::encode(t, len) : kTokBad;
        const uint32_t idx = ntok + (uint32_t)__popcll(starts & ((1ull << lane) - 1));
        if (idx < (uint32_t)kTokRing) TK[idx] = code;
      }
      ntok += (uint32_t)__popcll(starts);
      prev = (char)__shfl((int)c, 63, 64);
      p += 64;
    }
    lds_fence();
    if (ntok == 0 || ntok > (uint32_t)kTokRing) {  // fewer tokens than the host counted (or a ring overrun)
      bad = kBuildErrCount;
      bad_ply = done + 1;
      break;
    }
    const uint32_t k = min(min(ntok, 64u), nmoves - done);
    // (b) the chain, wave-uniform: interpret and play each move.  Lane j
    // collects move j's code, the move and the scalars after it,
    // SNAP[j + 1] the board after it.
    const uint32_t myc = TK[lane];
    // the codes are in registers before the chain starts, so the loop head
    // waits for nothing (its only LDS access is the snapshot byte store)
    asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(myc) : "memory");
    const Sc sc0 = sc;
    const typename R::Win win = R::window(sc, myc, k, lane);
    uint32_t mvw = 0;
    uint32_t scw[R::kVary];
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
    // (c) lane j checks move j against the board before it and packs the board after it
    bool fail = false;
    {
      // scalars before move j: after move j - 1, or the window's own; the
      // words the chain does not collect follow from the window's first
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
          const uint32_t o = o0 + done + lane + 1;
          if (out) out[o] = R::pack_from(wa, after_sc);
          if (states) states[o] = R::board_from(wa, after_sc);
        }
      }
    }
    const uint64_t fails = __ballot(fail);
    const uint32_t first = fails ? (uint32_t)__builtin_ctzll(fails) : kplay;
    if (first < k) {
      bad = kBuildErrMove;
      bad_ply = done + first + 1;
      break;
    }
    R::advance(sc, win, k);
    done += k;
    ntok -= k;
    // drop the consumed codes; the next window starts from the board after
    // this one's last move (the lanes' bytes)
    uint32_t keep[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const uint32_t src = k + lane + 64 * r;
      keep[r] = src < (uint32_t)kTokRing ? TK[src] : 0;
    }
    lds_fence();
    reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if ((uint32_t)lane + 64 * r < ntok) TK[lane + 64 * r] = keep[r];
    lds_fence();
  }
  if (!bad) {
    // text left after the host's count: more tokens than plies
    bool extra = ntok != 0;
    for (uint32_t q = p; q < e && !extra; q += 64) {
      const uint32_t i = q + lane;
      const char c = i < e ? text[i] : ' ';
      const char cprev = (char)__shfl_up((int)c, 1, 64);
      extra = __ballot(!space(c) && space(lane == 0 ? prev : cprev)) != 0;
      prev = (char)__shfl((int)c, 63, 64);
    }
    if (extra) {
      bad = kBuildErrCount;
      bad_ply = nmoves + 1;
    }
  }
  if (bad) {
    if (lane == 0) latch(err, bad, g, bad_ply);
    return;
  }
  if (final) {
    lds_fence();
    uint32_t wl[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) wl[i] = SNAP[0][i];
    const Board last = in_vgprs(R::board_from(wl, sc));
    const bool any = __ballot(R::any_legal_from(last, lane, lane == 0)) != 0;
    if (lane == 0) final[g] = R::end_flags(last, any);
  }
}

}  // namespace replay
}  // namespace fnnue
