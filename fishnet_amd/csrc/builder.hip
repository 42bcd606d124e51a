// builder.hip — device-side batch builder: FEN parse, UCI-move replay
// (standard + Chess960 castling, en passant, promotion) and legal 1-ply
// children, producing packed fnnue_pos records in HBM.
//
// Replaces on the device what board.cpp does on the host, i.e. the role
// shakmaty 0.23.0 plays in the reference's batch expansion
// ([ref] src/queue.rs:518-627: VariantPosition::from_setup, Uci::to_move,
// play_unchecked; wire format src/api.rs:293-309).  Semantics are those of the
// host builder (board.cpp), which is perft-checked; tests compare the two
// record for record, and fnnue_perft_device pins the move generator on the
// published perft counts.
//
// Replay is one 64-lane wave per game (replay_wave.h: the board chain plays a
// window of moves wave-uniformly, lanes then check the moves and pack the
// boards in parallel); children are one thread per ply.  Boards are bitboards
// in registers: no tables, attacks from shifts and ray walks.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <string>
#include <vector>

#include "board.h"
#include "builder.h"
#include "net.h"
#include "replay_wave.h"

namespace fnnue {

namespace {

constexpr uint64_t kNotA = 0xFEFEFEFEFEFEFEFEull, kNotH = 0x7F7F7F7F7F7F7F7Full;
constexpr uint64_t kNotAB = 0xFCFCFCFCFCFCFCFCull, kNotGH = 0x3F3F3F3F3F3F3F3Full;

// Every rule below is force-inlined and indexes the board's arrays only with
// compile-time indices (colour and castling-rook accessors select instead of
// indexing): a board passed by reference to an out-of-line function, or an
// array indexed at run time, lives in scratch memory, and the replay's board
// chain then waits on scratch loads every ply.

__device__ __forceinline__ int lsb(uint64_t b) { return __builtin_ctzll(b); }

__device__ __forceinline__ uint64_t knight_att(int s) {
  const uint64_t b = 1ull << s;
  return ((b << 17) & kNotA) | ((b << 15) & kNotH) | ((b << 10) & kNotAB) | ((b << 6) & kNotGH) |
         ((b >> 17) & kNotH) | ((b >> 15) & kNotA) | ((b >> 10) & kNotGH) | ((b >> 6) & kNotAB);
}

__device__ __forceinline__ uint64_t king_att(int s) {
  const uint64_t b = 1ull << s;
  return ((b << 1) & kNotA) | ((b >> 1) & kNotH) | (b << 8) | (b >> 8) | ((b << 9) & kNotA) | ((b << 7) & kNotH) |
         ((b >> 7) & kNotA) | ((b >> 9) & kNotH);
}

// Squares a pawn of colour c on s attacks.
__device__ __forceinline__ uint64_t pawn_att(int c, int s) {
  const uint64_t b = 1ull << s;
  return c == WHITE ? ((b << 9) & kNotA) | ((b << 7) & kNotH) : ((b >> 7) & kNotA) | ((b >> 9) & kNotH);
}

// Sliding attacks by occluded fill (Kogge-Stone): a fixed instruction
// sequence, so lanes holding different boards never diverge.  SH > 0 shifts
// left; `mask` removes squares that wrapped around a board edge.
template <int SH>
__device__ __forceinline__ uint64_t shl(uint64_t b) {
  if constexpr (SH > 0) return b << SH;
  else return b >> -SH;
}
template <int SH>
__device__ __forceinline__ uint64_t fill(uint64_t gen, uint64_t empty, uint64_t mask) {
  uint64_t pro = empty & mask;
  gen |= pro & shl<SH>(gen);
  pro &= shl<SH>(pro);
  gen |= pro & shl<2 * SH>(gen);
  pro &= shl<2 * SH>(pro);
  gen |= pro & shl<4 * SH>(gen);
  return shl<SH>(gen) & mask;
}

__device__ __forceinline__ uint64_t bishop_att(int s, uint64_t occ) {
  const uint64_t g = 1ull << s, e = ~occ;
  return fill<9>(g, e, kNotA) | fill<7>(g, e, kNotH) | fill<-7>(g, e, kNotA) | fill<-9>(g, e, kNotH);
}
__device__ __forceinline__ uint64_t rook_att(int s, uint64_t occ) {
  const uint64_t g = 1ull << s, e = ~occ;
  return fill<8>(g, e, ~0ull) | fill<-8>(g, e, ~0ull) | fill<1>(g, e, kNotA) | fill<-1>(g, e, kNotH);
}

struct DMove {
  int from, to, promo, castle;  // castle: to = rook square (king takes rook)
};

__device__ __forceinline__ uint64_t colour(const DBoard& b, int c) { return c ? b.bc[1] : b.bc[0]; }

// Castling rook square of colour c, side s (-1: none).
__device__ __forceinline__ int cr_get(const DBoard& b, int c, int side) {
  const uint32_t v = (b.cr >> (8 * (2 * c + side))) & 0xFFu;
  return v == 0xFFu ? -1 : (int)v;
}
__device__ __forceinline__ void cr_set(DBoard& b, int c, int side, int sq) {
  const int sh = 8 * (2 * c + side);
  b.cr = (b.cr & ~(0xFFu << sh)) | ((uint32_t)(sq < 0 ? 0xFF : sq) << sh);
}
__device__ __forceinline__ void cr_clear(DBoard& b, int c) { b.cr |= 0xFFFFu << (16 * c); }

// Piece type on the square(s) of mask m (0: empty).
__device__ __forceinline__ int type_at(const DBoard& b, uint64_t m) {
  int t = 0;
#pragma unroll
  for (int k = 1; k <= KING; ++k) t = (b.bt[k] & m) ? k : t;
  return t;
}

__device__ __forceinline__ int piece_at(const DBoard& b, int s) {
  const uint64_t m = 1ull << s;
  const int t = type_at(b, m);
  return t ? make_piece_d((b.bc[1] & m) ? 1 : 0, t) : 0;
}

__device__ __forceinline__ void put(DBoard& b, int s, int pc) {
  const uint64_t m = 1ull << s;
  const int c = pc >> 3, t = pc & 7;
  b.bc[0] |= c ? 0ull : m;
  b.bc[1] |= c ? m : 0ull;
#pragma unroll
  for (int k = 1; k <= KING; ++k) b.bt[k] |= k == t ? m : 0ull;
}

__device__ __forceinline__ void remove_sq(DBoard& b, int s) {
  const uint64_t m = ~(1ull << s);
  b.bc[0] &= m;
  b.bc[1] &= m;
#pragma unroll
  for (int t = 1; t < 7; ++t) b.bt[t] &= m;
}

__device__ __forceinline__ int king_sq(const DBoard& b, int c) {
  const uint64_t k = b.bt[KING] & colour(b, c);
  return k ? lsb(k) : -1;
}

__device__ __forceinline__ bool attacked(const DBoard& b, int s, int by, uint64_t occ) {
  const uint64_t them = colour(b, by);
  return ((pawn_att(by ^ 1, s) & b.bt[PAWN]) | (knight_att(s) & b.bt[KNIGHT]) | (king_att(s) & b.bt[KING]) |
          (bishop_att(s, occ) & (b.bt[BISHOP] | b.bt[QUEEN])) | (rook_att(s, occ) & (b.bt[ROOK] | b.bt[QUEEN]))) &
         them;
}

// Board::do_move (board.cpp), on bitboards.
__device__ __forceinline__ void do_move(DBoard& b, const DMove& m) {
  const int us = b.stm;
  const int pc = piece_at(b, m.from);
  const int back = us == WHITE ? 0 : 56;
  int new_ep = -1;
  if (m.castle) {
    const bool king_side = m.to > m.from;
    const int kto = back + (king_side ? 6 : 2), rto = back + (king_side ? 5 : 3);
    const int rook = piece_at(b, m.to);
    remove_sq(b, m.from);
    remove_sq(b, m.to);
    put(b, kto, pc);
    put(b, rto, rook);
    cr_clear(b, us);
  } else {
    remove_sq(b, m.to);
    if ((pc & 7) == PAWN) {
      if (m.to == b.ep && (m.from & 7) != (m.to & 7)) remove_sq(b, m.to + (us == WHITE ? -8 : 8));
      if ((m.from ^ m.to) == 16) new_ep = (m.from + m.to) / 2;
    }
    remove_sq(b, m.from);
    put(b, m.to, m.promo ? make_piece_d(us, m.promo) : pc);
    if ((pc & 7) == KING) cr_clear(b, us);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int side = 0; side < 2; ++side)
        if (cr_get(b, c, side) == m.from || cr_get(b, c, side) == m.to) cr_set(b, c, side, -1);
  }
  b.ep = new_ep;
  b.stm = (uint32_t)(us ^ 1);
}

__device__ __forceinline__ bool legal(const DBoard& b, const DMove& m) {
  DBoard c = b;
  do_move(c, m);
  const int k = king_sq(c, b.stm);
  return k >= 0 && !attacked(c, k, b.stm ^ 1, c.bc[0] | c.bc[1]);
}

// Board::pseudo_moves' castling conditions for the rook on rsq (side 0 king
// side, 1 queen side): rook in place, king on its back rank, the squares
// between and the destinations empty, the king not in check and not passing
// an attacked square.
__device__ __forceinline__ bool castle_ok(const DBoard& b, int ksq, int rsq, int side) {
  const int us = b.stm, them = us ^ 1;
  const int back = us == WHITE ? 0 : 56;
  const uint64_t occ = b.bc[0] | b.bc[1];
  if (rsq < 0 || piece_at(b, rsq) != make_piece_d(us, ROOK)) return false;
  const int kto = back + (side == 0 ? 6 : 2), rto = back + (side == 0 ? 5 : 3);
  const int lo = min(min(ksq, rsq), min(kto, rto)), hi = max(max(ksq, rsq), max(kto, rto));
  // [lo, hi] without the king and the rook must be empty
  const uint64_t span = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
  if (occ & span & ~(1ull << ksq) & ~(1ull << rsq)) return false;
  if (attacked(b, ksq, them, occ)) return false;
  const int step = kto > ksq ? 1 : -1;
  bool ok = true;
  for (int t = ksq; t != kto && ok;) {
    t += step;
    if (attacked(b, t, them, occ)) ok = false;
  }
  return ok;
}

// Legal moves in the order of Board::pseudo_moves + is_legal (board.cpp):
// own pieces by square; a pawn's push (promotions Q, R, B, N), double push,
// captures by square, en passant; then castling king side, queen side.
// f(move) returns false to stop early.  Only pieces on `from_mask` move.
template <class F>
__device__ void for_each_legal(const DBoard& b, F&& f, uint64_t from_mask = ~0ull) {
  const int us = b.stm, them = us ^ 1;
  const uint64_t occ = b.bc[0] | b.bc[1], own = colour(b, us), opp = colour(b, them);
  const int up = us == WHITE ? 8 : -8;
  const int rank7 = us == WHITE ? 6 : 1, rank2 = us == WHITE ? 1 : 6;
  auto emit = [&](int from, int to, int promo, int castle) -> bool {
    const DMove m{from, to, promo, castle};
    return !legal(b, m) || f(m);
  };
  for (uint64_t pcs = own & from_mask; pcs; pcs &= pcs - 1) {
    const int s = lsb(pcs);
    const uint64_t sm = 1ull << s;
    if (b.bt[PAWN] & sm) {
      const bool promo = (s >> 3) == rank7;
      auto pawn_to = [&](int t) -> bool {
        if (promo) {
          for (int p = QUEEN; p >= KNIGHT; --p)
            if (!emit(s, t, p, 0)) return false;
          return true;
        }
        return emit(s, t, 0, 0);
      };
      const int t1 = s + up;
      if (!(occ & (1ull << t1))) {
        if (!pawn_to(t1)) return;
        const int t2 = t1 + up;
        if ((s >> 3) == rank2 && !(occ & (1ull << t2)) && !emit(s, t2, 0, 0)) return;
      }
      for (uint64_t a = pawn_att(us, s) & opp; a; a &= a - 1)
        if (!pawn_to(lsb(a))) return;
      if (b.ep >= 0 && (pawn_att(us, s) & (1ull << b.ep)) && !emit(s, b.ep, 0, 0)) return;
      continue;
    }
    uint64_t targets;
    if (b.bt[KNIGHT] & sm) targets = knight_att(s);
    else if (b.bt[BISHOP] & sm) targets = bishop_att(s, occ);
    else if (b.bt[ROOK] & sm) targets = rook_att(s, occ);
    else if (b.bt[QUEEN] & sm) targets = bishop_att(s, occ) | rook_att(s, occ);
    else targets = king_att(s);
    for (uint64_t t = targets & ~own; t; t &= t - 1)
      if (!emit(s, lsb(t), 0, 0)) return;
  }
  const int ksq = king_sq(b, us);
  const int back = us == WHITE ? 0 : 56;
  if (ksq < 0 || (ksq & 56) != back || !((from_mask >> ksq) & 1)) return;
  for (int side = 0; side < 2; ++side) {
    const int rsq = cr_get(b, us, side);
    if (castle_ok(b, ksq, rsq, side) && !emit(ksq, rsq, 0, 1)) return;  // legal() re-checks the king
  }
}

// Is m one of Board::pseudo_moves' moves?  (The set the host builder matches
// UCI tokens against, before the legality filter.)
__device__ __forceinline__ bool pseudo_member(const DBoard& b, const DMove& m) {
  const int us = b.stm, them = us ^ 1;
  const uint64_t occ = b.bc[0] | b.bc[1], own = colour(b, us), opp = colour(b, them);
  const uint64_t fm = 1ull << m.from, tm = 1ull << m.to;
  if (!(own & fm)) return false;
  if (m.castle) {
    const int ksq = king_sq(b, us), back = us == WHITE ? 0 : 56;
    if (m.promo || m.from != ksq || (ksq & 56) != back) return false;
    const int side = cr_get(b, us, 0) == m.to ? 0 : cr_get(b, us, 1) == m.to ? 1 : -1;
    return side >= 0 && castle_ok(b, ksq, m.to, side);
  }
  const int t = type_at(b, fm);
  if (t == PAWN) {
    const int r = m.from >> 3, up = us == WHITE ? 8 : -8;
    const bool promo_rank = r == (us == WHITE ? 6 : 1);
    const bool promo_ok = promo_rank ? m.promo != 0 : m.promo == 0;
    const int t1 = m.from + up, t2 = t1 + up;
    bool ok = false;
    if (!(occ & (1ull << t1))) {
      ok = m.to == t1 && promo_ok;
      ok = ok || (m.to == t2 && r == (us == WHITE ? 1 : 6) && !(occ & (1ull << t2)) && m.promo == 0);
    }
    const uint64_t pa = pawn_att(us, m.from);
    ok = ok || ((pa & opp & tm) && promo_ok);
    ok = ok || (b.ep >= 0 && m.to == b.ep && (pa & tm) && m.promo == 0);
    return ok;
  }
  uint64_t targets;
  if (t == KNIGHT) targets = knight_att(m.from);
  else if (t == BISHOP) targets = bishop_att(m.from, occ);
  else if (t == ROOK) targets = rook_att(m.from, occ);
  else if (t == QUEEN) targets = bishop_att(m.from, occ) | rook_att(m.from, occ);
  else targets = king_att(m.from);
  return m.promo == 0 && (targets & ~own & tm);
}

// Packed record from the bitboards, branch-free: bit k of a square's nibble
// is bit k of the piece code (type bits 0-2: P=1 N=2 B=3 R=4 Q=5 K=6; bit 3
// black), so each nibble plane is an OR of type bitboards, spread from 8 bits
// of a rank to 8 nibbles.  Board::pack on every consistent board.
__device__ __forceinline__ uint32_t spread8(uint32_t x) {
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return (x | (x << 3)) & 0x11111111u;
}

__device__ __forceinline__ fnnue_pos pack(const DBoard& b) {
  const uint64_t q0 = b.bt[PAWN] | b.bt[BISHOP] | b.bt[QUEEN];
  const uint64_t q1 = b.bt[KNIGHT] | b.bt[BISHOP] | b.bt[KING];
  const uint64_t q2 = b.bt[ROOK] | b.bt[QUEEN] | b.bt[KING];
  const uint64_t q3 = b.bc[BLACK];
  uint32_t w[9];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int sh = 8 * r;
    w[r] = spread8((uint32_t)(q0 >> sh) & 255u) | (spread8((uint32_t)(q1 >> sh) & 255u) << 1) |
           (spread8((uint32_t)(q2 >> sh) & 255u) << 2) | (spread8((uint32_t)(q3 >> sh) & 255u) << 3);
  }
  w[8] = b.stm;
  fnnue_pos p;
  memcpy(&p, w, sizeof(p));
  return p;
}

// ---- text ----
__device__ __forceinline__ bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// Next whitespace-separated token of [*p, end): returns its length (0 = none).
__device__ __forceinline__ int next_token(const char* text, uint32_t& p, uint32_t end, uint32_t& start) {
  while (p < end && is_space(text[p])) ++p;
  start = p;
  while (p < end && !is_space(text[p])) ++p;
  return (int)(p - start);
}

__device__ __forceinline__ int count_tokens(const char* text, uint32_t p, uint32_t end) {
  int n = 0;
  uint32_t st;
  while (next_token(text, p, end, st) > 0) ++n;
  return n;
}

// board_from_fen (board.cpp) on the device.  Returns false on malformed FEN.
__device__ __forceinline__ bool parse_fen(const char* text, uint32_t p, uint32_t end, DBoard& b) {
  for (int i = 0; i < 2; ++i) b.bc[i] = 0;
  for (int i = 0; i < 7; ++i) b.bt[i] = 0;
  b.cr = 0xFFFFFFFFu;
  b.ep = -1;
  b.stm = WHITE;
  b.c960 = 0;
  uint32_t st;
  int len = next_token(text, p, end, st);
  if (len == 0) return false;
  int r = 7, f = 0;
  for (uint32_t i = st; i < st + (uint32_t)len; ++i) {
    const char ch = text[i];
    if (ch == '/') {
      if (f != 8) return false;
      --r;
      f = 0;
      continue;
    }
    if (ch >= '1' && ch <= '8') {
      f += ch - '0';
      if (f > 8) return false;
      continue;
    }
    int pc = 0;
    const char lc = (char)(ch | 32);
    const int col = (ch >= 'a' && ch <= 'z') ? BLACK : WHITE;
    switch (lc) {
      case 'p': pc = PAWN; break;
      case 'n': pc = KNIGHT; break;
      case 'b': pc = BISHOP; break;
      case 'r': pc = ROOK; break;
      case 'q': pc = QUEEN; break;
      case 'k': pc = KING; break;
      default: return false;
    }
    if ((ch < 'A' || ch > 'Z') && (ch < 'a' || ch > 'z')) return false;
    if (r < 0 || f > 7) return false;
    put(b, r * 8 + f, make_piece_d(col, pc));
    ++f;
  }
  if (r != 0 || f != 8) return false;
  len = next_token(text, p, end, st);
  if (len != 1 || (text[st] != 'w' && text[st] != 'b')) return false;
  b.stm = text[st] == 'w' ? WHITE : BLACK;
  if (__popcll(b.bt[KING] & b.bc[WHITE]) != 1 || __popcll(b.bt[KING] & b.bc[BLACK]) != 1) return false;
  uint32_t cst;
  const int clen = next_token(text, p, end, cst);
  if (clen > 0 && !(clen == 1 && text[cst] == '-')) {
    for (uint32_t i = cst; i < cst + (uint32_t)clen; ++i) {
      const char ch = text[i];
      const int col = (ch >= 'a' && ch <= 'z') ? BLACK : WHITE;
      const char lc = (char)(ch | 32);
      const int back = col == WHITE ? 0 : 56;
      const int k = king_sq(b, col);
      const int rook = make_piece_d(col, ROOK);
      int rsq = -1, side = -1;
      if ((k & 56) != back) continue;  // as the host: ignored before the character is checked
      if (lc == 'k') {
        side = 0;
      } else if (lc == 'q') {
        side = 1;
      } else if (lc >= 'a' && lc <= 'h') {
        side = 2;
      } else {
        return false;
      }
      if (side == 0) {
        for (int x = back + 7; x > k; --x)
          if (piece_at(b, x) == rook) { rsq = x; break; }
      } else if (side == 1) {
        for (int x = back; x < k; ++x)
          if (piece_at(b, x) == rook) { rsq = x; break; }
      } else {
        rsq = back + (lc - 'a');
        if (piece_at(b, rsq) != rook) rsq = -1;
        side = rsq > k ? 0 : 1;
        b.c960 = 1;
      }
      if (rsq >= 0) cr_set(b, col, side, rsq);
    }
  }
  for (int col = 0; col < 2; ++col) {
    const int k = king_sq(b, col);
    for (int side = 0; side < 2; ++side) {
      const int rsq = cr_get(b, col, side);
      if (rsq < 0) continue;
      if ((k & 7) != 4 || ((rsq & 7) != (side == 0 ? 7 : 0))) b.c960 = 1;
    }
  }
  uint32_t est;
  const int elen = next_token(text, p, end, est);
  if (elen == 2 && text[est] >= 'a' && text[est] <= 'h' && text[est + 1] >= '1' && text[est + 1] <= '8')
    b.ep = (text[est + 1] - '1') * 8 + (text[est] - 'a');
  return true;
}

// Chess rules of the wave replay (replay_wave.h).
struct ChessRules {
  using Board = DBoard;
  using Move = DMove;
  using Pos = fnnue_pos;
  // The board's non-square state.  The chain keeps en passant and the side to
  // move; castling rights are not kept along it: a right (colour c, side) is
  // alive while neither its rook's square nor c's king square at the game's
  // start has been touched (a from / to square of any move so far: the king
  // moved, the rook moved or was taken — DBoard::cr's update rule), so with
  // the squares the game's moves touch (m: before the window; a window's own
  // by a lane-parallel prefix OR) every ply's rights follow from the start's.
  struct Scalars {
    int32_t ep;
    uint32_t stm;
    uint32_t c960;
    uint32_t cr;    // derived: the rights for m (window starts, last board) or per checking lane
    uint32_t cr0;   // the start's castling rooks (DBoard::cr packing)
    uint32_t ksq;   // the start's king squares, white | black << 8 (64: none)
    uint32_t mlo, mhi;  // squares touched before the window
  };
  // per window, per lane j: the touched squares before move j (m included)
  // and move j's own
  struct Win {
    uint64_t pre, own;
  };
  __device__ static bool parse_fen(const char* t, uint32_t p, uint32_t e, int, DBoard& b) {
    return fnnue::parse_fen(t, p, e, b);
  }
  __device__ static const char* start_fen(int) { return "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"; }
  __device__ static uint32_t start_fen_len(int) { return 56; }
  __device__ static DBoard start_board(int) {
    DBoard b;
    b.bc[WHITE] = 0x000000000000FFFFull;
    b.bc[BLACK] = 0xFFFF000000000000ull;
    b.bt[0] = 0;
    b.bt[PAWN] = 0x00FF00000000FF00ull;
    b.bt[KNIGHT] = 0x4200000000000042ull;
    b.bt[BISHOP] = 0x2400000000000024ull;
    b.bt[ROOK] = 0x8100000000000081ull;
    b.bt[QUEEN] = 0x0800000000000008ull;
    b.bt[KING] = 0x1000000000000010ull;
    b.cr = 7u | (0u << 8) | (63u << 16) | (56u << 24);  // [white][king side] h1, [white][queen side] a1, black h8, a8
    b.ep = -1;
    b.stm = WHITE;
    b.c960 = 0;
    return b;
  }
  // "e2e4" / "e7e8q" (board.cpp's UCI: lowercase promotion letters n b r q;
  // 'k' / 'p' or anything else never names a generated move)
  __device__ static uint32_t encode(const char* c, int len) {
    const int from = replay::tok_sq(c[0], c[1]), to = replay::tok_sq(c[2], c[3]);
    if (from < 0 || to < 0) return replay::kTokBad;
    uint32_t promo = 0;
    if (len == 5) {
      switch (c[4]) {
        case 'n': promo = KNIGHT; break;
        case 'b': promo = BISHOP; break;
        case 'r': promo = ROOK; break;
        case 'q': promo = QUEEN; break;
        default: return replay::kTokBad;
      }
    }
    return (uint32_t)from | ((uint32_t)to << 6) | (promo << 12);
  }
  __device__ static Scalars scalars(const DBoard& b) {
    const uint64_t wk = b.bc[WHITE] & b.bt[KING], bk = b.bc[BLACK] & b.bt[KING];
    const uint32_t k0 = wk ? (uint32_t)__builtin_ctzll(wk) : 64u, k1 = bk ? (uint32_t)__builtin_ctzll(bk) : 64u;
    return Scalars{b.ep, b.stm, b.c960, b.cr, b.cr, k0 | k1 << 8, 0u, 0u};
  }
  __device__ static int sc_cr(uint32_t cr, int c, int side) {
    const uint32_t v = (cr >> (8 * (2 * c + side))) & 0xFFu;
    return v == 0xFFu ? -1 : (int)v;
  }
  __device__ static bool touched(uint64_t m, uint32_t sq) { return sq < 64 && ((m >> sq) & 1u); }
  // the castling rooks still alive after the squares m were touched
  __device__ static uint32_t rights(uint32_t cr0, uint32_t ksq, uint64_t m) {
    uint32_t cr = cr0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t r = (cr0 >> (8 * i)) & 0xFFu, k = (ksq >> (8 * (i >> 1))) & 0xFFu;
      if (r == 0xFFu || touched(m, r) || touched(m, k)) cr |= 0xFFu << (8 * i);
    }
    return cr;
  }
  // Before the chain: each lane's move squares and the exclusive prefix OR of
  // the window's (k moves) in front of it, m included.
  __device__ static Win window(const Scalars& sc, uint32_t code, uint32_t k, int lane) {
    uint64_t own = 0;
    if ((uint32_t)lane < k && !(code & replay::kTokBad))
      own = (1ull << replay::tok_from(code)) | (1ull << replay::tok_to(code));
    uint32_t lo = (uint32_t)own, hi = (uint32_t)(own >> 32);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // inclusive prefix OR
      const uint32_t ulo = (uint32_t)__shfl_up((int)lo, o, 64), uhi = (uint32_t)__shfl_up((int)hi, o, 64);
      if (lane >= o) {
        lo |= ulo;
        hi |= uhi;
      }
    }
    uint32_t elo = (uint32_t)__shfl_up((int)lo, 1, 64), ehi = (uint32_t)__shfl_up((int)hi, 1, 64);
    if (lane == 0) elo = ehi = 0;
    return Win{((uint64_t)elo | (uint64_t)ehi << 32) | ((uint64_t)sc.mlo | (uint64_t)sc.mhi << 32), own};
  }
  // After a window of k moves: m and the rights for the board after them.
  __device__ static void advance(Scalars& sc, const Win& w, uint32_t k) {
    const uint64_t m = replay::lane_u64(w.pre, (int)k - 1) | replay::lane_u64(w.own, (int)k - 1);
    sc.mlo = (uint32_t)m;
    sc.mhi = (uint32_t)(m >> 32);
    sc.cr = rights(sc.cr0, sc.ksq, m);
  }
  // Along the chain only ep changes (collected per lane); the checking lane of
  // move j derives the rest: stm by parity, the rights from the squares
  // touched before move j (after: and by it).
  static constexpr int kVary = 1;
  __device__ static void fix(Scalars& s, const Scalars& s0, const Win& w, uint32_t j, bool after) {
    s.stm = s0.stm ^ ((j + (after ? 1u : 0u)) & 1u);
    s.c960 = s0.c960;
    s.cr = rights(s0.cr0, s0.ksq, after ? w.pre | w.own : w.pre);
  }
  __device__ static uint32_t lane_square(const DBoard& b, int sq) { return (uint32_t)piece_at(b, sq); }
  // One chain step (move j of the window): the move the code names, played on
  // the lane bytes (lane l holds square l's piece code) and the scalars;
  // returns it packed.  It is castling when the own king goes to a castling
  // rook's square or (standard positions) to its two-square destination, with
  // the rights of move j's board (Win); everything else as written.  Nothing
  // is checked here: verify() tests the move against the board before it (a
  // code that names no move of the side to move fails there, at its own ply —
  // and a failed ply ends the game's replay).
  __device__ __forceinline__ static bool step(Scalars& b, const Win& w, uint32_t j, uint32_t code, uint32_t& sqv,
                                              int lane, uint32_t& mv) {
    const int from = (int)replay::tok_from(code), to = (int)replay::tok_to(code), promo = (int)replay::tok_piece(code);
    const int us = (int)b.stm;
    const uint32_t pc = replay::lane_value(sqv, from);
    const int back = us == WHITE ? 0 : 56;
    uint32_t v = sqv;
    int new_ep = -1;
    mv = (uint32_t)from | ((uint32_t)to << 6) | ((uint32_t)promo << 12);
    if ((pc & 7) == KING) {  // castling, or a king move
      int rsq = -1;
      if (!promo) {
        const uint32_t cr = rights(b.cr0, b.ksq, replay::lane_u64(w.pre, (int)j));
#pragma unroll
        for (int side = 0; side < 2; ++side) {
          const int r = sc_cr(cr, us, side);
          if (rsq < 0 && r >= 0 && (to == r || (!b.c960 && to == back + (side == 0 ? 6 : 2)))) rsq = r;
        }
      }
      if (rsq >= 0) {
        const bool king_side = rsq > from;
        const int kto = back + (king_side ? 6 : 2), rto = back + (king_side ? 5 : 3);
        v = (lane == from || lane == rsq) ? 0u : v;
        v = lane == kto ? pc : v;
        v = lane == rto ? (uint32_t)make_piece_d(us, ROOK) : v;
        mv = (uint32_t)from | ((uint32_t)rsq << 6) | (1u << 15);
      } else {
        v = lane == from ? 0u : v;
        v = lane == to ? (promo ? (uint32_t)make_piece_d(us, promo) : pc) : v;
      }
    } else {
      const bool pawn = (pc & 7) == PAWN;
      const int cap = (pawn && to == b.ep && ((from ^ to) & 7)) ? to + (us == WHITE ? -8 : 8) : -1;
      v = (lane == from || lane == cap) ? 0u : v;
      v = lane == to ? (promo ? (uint32_t)make_piece_d(us, promo) : pc) : v;
      if (pawn && (from ^ to) == 16) new_ep = (from + to) >> 1;
    }
    sqv = v;
    b.ep = new_ep;
    b.stm = (uint32_t)(us ^ 1);
    return true;
  }
  // The whole window's chain lane-parallel (lane j = move j), for the same
  // boards, moves and ep words as k calls of step().  step() needs the board
  // only for the mover's piece pc (castling is the own king onto a castling
  // square, ep and the double push need a pawn); every other effect is a
  // select on known squares.  So:
  //   1. the piece on from_j before move j is what the last earlier move that
  //      wrote from_j put there (an LDS table of writers per square, one
  //      64-bit mask each: the highest writer below j), or the window's first
  //      board; a write puts the mover's piece (or its promotion), so the
  //      pieces follow by pointer jumping over the writers (6 rounds);
  //   2. castling moves are detected from those pieces; a castling move writes
  //      two squares (king to kto, rook to rto), so if any, step 1 runs again
  //      with them;
  //   3. ep squares by a shuffle from the move before, en passant captures;
  //   4. the snapshots, square = lane, one select chain per move on values
  //      that are all known (no per-move readlane of the board).
  // Exact for every move up to a window's first illegal one (the only part
  // check() and the records use): with all earlier moves legal, each mover's
  // square was last written by an earlier move or holds its first-board
  // piece; a castling move kills its colour's rights (its king's square is
  // touched), so no later detection depends on step 2's second pass; a move
  // whose piece the table gets wrong (it moves from a square emptied since)
  // is illegal on its exact board, and fails its check as in step().
  static constexpr bool kLaneChain = true;
  __device__ static uint32_t lane_chain(Scalars& sc, uint32_t& sqv, uint32_t myc, uint32_t k, const Win& w,
                                        uint32_t (*SNAP)[16], int lane, uint32_t& mvw, uint32_t (&scw)[kVary]) {
    reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;
    const uint64_t badm = __ballot((uint32_t)lane < k && (myc & replay::kTokBad));
    const uint32_t kplay = badm ? min(k, (uint32_t)__builtin_ctzll(badm)) : k;
    const bool live = (uint32_t)lane < kplay;
    const int from = (int)replay::tok_from(myc), to = (int)replay::tok_to(myc), promo = (int)replay::tok_piece(myc);
    const int us = (int)(sc.stm ^ ((uint32_t)lane & 1u));
    const int back = us == WHITE ? 0 : 56;
    const uint32_t start = (uint32_t)__shfl((int)sqv, from, 64);  // the first board's piece on from
    // writers table: rows 57-64 of this window's snapshot buffer (written
    // only by step 4, after their last use here)
    uint64_t* WR = reinterpret_cast<uint64_t*>(SNAP[57]);
    int w1 = to, w2 = 64;  // squares a move writes (64: none)
    // piece on from_j before move j (S) through the writers of step 1
    auto resolve = [&]() -> uint32_t {
      WR[lane] = 0;
      replay::lds_fence();
      if (live) {
        atomicOr(reinterpret_cast<unsigned long long*>(&WR[w1]), 1ull << lane);
        if (w2 < 64) atomicOr(reinterpret_cast<unsigned long long*>(&WR[w2]), 1ull << lane);
      }
      replay::lds_fence();
      const uint64_t m = WR[from] & ((1ull << lane) - 1);
      replay::lds_fence();  // the table's reads before a second pass clears it
      const int src = m ? 63 - __builtin_clzll(m) : 0;
      const int sw1 = __shfl(w1, src, 64), spr = __shfl(promo, src, 64);
      const int sus = (int)(sc.stm ^ ((uint32_t)src & 1u));
      bool known = true;
      uint32_t val = start;
      if (m) {
        if (sw1 != from) val = (uint32_t)make_piece_d(sus, ROOK);  // a castling move's rook square
        else if (spr) val = (uint32_t)make_piece_d(sus, spr);      // a promotion
        else known = false;                                         // that move's own piece
      }
      int link = src;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const uint32_t lv = (uint32_t)__shfl((int)val, link, 64);
        const int lk = __shfl((int)known, link, 64), ll = __shfl(link, link, 64);
        if (!known) {
          if (lk) {
            val = lv;
            known = true;
          } else {
            link = ll;
          }
        }
      }
      return val;
    };
    uint32_t pc = resolve();
    // castling: step()'s test with this move's rights
    auto castle_rook = [&](uint32_t p) -> int {
      int rsq = -1;
      if (live && !promo && (p & 7) == KING) {
        const uint32_t cr = rights(sc.cr0, sc.ksq, w.pre);
#pragma unroll
        for (int side = 0; side < 2; ++side) {
          const int r = sc_cr(cr, us, side);
          if (rsq < 0 && r >= 0 && (to == r || (!sc.c960 && to == back + (side == 0 ? 6 : 2)))) rsq = r;
        }
      }
      return rsq;
    };
    int rsq = castle_rook(pc);
    const bool castle = rsq >= 0;
    const bool king_side = rsq > from;
    const int kto = back + (king_side ? 6 : 2), rto = back + (king_side ? 5 : 3);
    if (__ballot(castle)) {
      w1 = castle ? kto : to;
      w2 = castle ? rto : 64;
      pc = resolve();
    }
    // en passant: the ep square before move j is the one move j - 1 left
    const bool king = (pc & 7) == KING, pawn = (pc & 7) == PAWN;
    const int new_ep = (!king && pawn && (from ^ to) == 16) ? (from + to) >> 1 : -1;
    const int prev_ep = __shfl_up(new_ep, 1, 64);
    const int ep = lane == 0 ? sc.ep : prev_ep;
    const int cap = (!king && pawn && to == ep && ((from ^ to) & 7)) ? to + (us == WHITE ? -8 : 8) : 64;
    const uint32_t placed = promo ? (uint32_t)make_piece_d(us, promo) : pc;
    // this move's effect: clear c1, c2; write v1 at s1, v2 at s2 (64: none)
    const int c1 = from, c2 = castle ? rsq : cap, s1 = castle ? kto : to, s2 = castle ? rto : 64;
    const uint32_t v1 = castle ? pc : placed, v2 = (uint32_t)make_piece_d(us, ROOK);
    const uint32_t pk = (uint32_t)c1 | (uint32_t)c2 << 7 | (uint32_t)s1 << 14 | (uint32_t)s2 << 21;
    const uint32_t pv = v1 | v2 << 4;
    mvw = live ? (castle ? ((uint32_t)from | ((uint32_t)rsq << 6) | (1u << 15))
                         : ((uint32_t)from | ((uint32_t)to << 6) | ((uint32_t)promo << 12)))
               : 0u;
    scw[0] = live ? (uint32_t)new_ep : 0u;
    replay::lds_fence();
    uint32_t v = sqv;
    for (uint32_t j = 0; j < kplay; ++j) {
      const uint32_t a = replay::lane_value(pk, (int)j), b = replay::lane_value(pv, (int)j);
      const uint32_t l = (uint32_t)lane;
      v = (l == (a & 127u) || l == ((a >> 7) & 127u)) ? 0u : v;
      v = l == ((a >> 14) & 127u) ? (b & 15u) : v;
      v = l == ((a >> 21) & 127u) ? (b >> 4) : v;
      reinterpret_cast<uint8_t*>(SNAP[j + 1])[lane] = (uint8_t)v;
    }
    sqv = v;
    if (kplay) {
      sc.ep = (int32_t)replay::lane_value((uint32_t)new_ep, (int)kplay - 1);
      sc.stm ^= kplay & 1u;
    }
    replay::lds_fence();
    return kplay;
  }
  __device__ static uint32_t pack_move(const DMove& m) {
    return (uint32_t)m.from | ((uint32_t)m.to << 6) | ((uint32_t)m.promo << 12) | ((uint32_t)m.castle << 15);
  }
  __device__ static DMove unpack_move(uint32_t w) {
    return DMove{(int)(w & 63), (int)((w >> 6) & 63), (int)((w >> 12) & 7), (int)((w >> 15) & 1)};
  }
  // A snapshot's bytes (piece codes) as bitboards: bit k of a code is bitboard
  // plane k (type bits 0-2: P=1 N=2 B=3 R=4 Q=5 K=6; bit 3 black).
  __device__ static DBoard board_from(const uint32_t (&w)[16], const Scalars& sc) {
    const uint64_t p0 = replay::byte_plane(w, 0), p1 = replay::byte_plane(w, 1), p2 = replay::byte_plane(w, 2);
    const uint64_t p3 = replay::byte_plane(w, 3);
    const uint64_t occ = p0 | p1 | p2;
    DBoard b;
    b.bc[WHITE] = occ & ~p3;
    b.bc[BLACK] = occ & p3;
    b.bt[0] = 0;
    b.bt[PAWN] = p0 & ~p1 & ~p2;
    b.bt[KNIGHT] = ~p0 & p1 & ~p2;
    b.bt[BISHOP] = p0 & p1 & ~p2;
    b.bt[ROOK] = ~p0 & ~p1 & p2;
    b.bt[QUEEN] = p0 & ~p1 & p2;
    b.bt[KING] = ~p0 & p1 & p2;
    b.cr = sc.cr;
    b.ep = sc.ep;
    b.stm = sc.stm;
    b.c960 = sc.c960;
    return b;
  }
  __device__ static fnnue_pos pack_from(const uint32_t (&w)[16], const Scalars& sc) {
    uint32_t q[9];
    uint32_t nib[8];
    replay::pack_nibbles(w, nib);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = nib[i];
    q[8] = sc.stm;
    fnnue_pos p;
    memcpy(&p, q, sizeof(p));
    return p;
  }
  // interpret() built m from the token; the host builder accepts the token iff
  // a legal move prints as it, and that move can only be m (a castling move's
  // destination holds the own rook or lies two files from the unmoved king,
  // where no other move goes): so the token is accepted iff m is legal.
  __device__ static bool verify(const DBoard& b, const DMove& m) { return pseudo_member(b, m) && legal(b, m); }
  __device__ static fnnue_pos pack(const DBoard& b) { return fnnue::pack(b); }
  __device__ static bool any_legal_from(const DBoard& b, int sq, bool) {
    if (!((colour(b, b.stm) >> sq) & 1)) return false;
    bool any = false;
    const DBoard c = b;  // the generator takes its board by reference: a copy, so the chain's board stays in registers
    for_each_legal(c, [&](const DMove&) -> bool {
      any = true;
      return false;
    }, 1ull << sq);
    return any;
  }
  __device__ static uint8_t end_flags(const DBoard& b, bool any) {
    const int k = king_sq(b, b.stm);
    const bool check = k >= 0 && attacked(b, k, b.stm ^ 1, b.bc[0] | b.bc[1]);
    return (uint8_t)((any ? 0 : kFinalNoMoves) | (check ? kFinalCheck : 0));
  }
};

// ---- kernels ----
// text layout of game g: FEN in [fen_off[g], mv_off[g]), moves in [mv_off[g], fen_off[g + 1]).
__global__ void count_plies_kernel(const char* __restrict__ text, const uint32_t* __restrict__ fen_off,
                                   const uint32_t* __restrict__ mv_off, uint32_t ngames, uint32_t* __restrict__ plies) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngames) return;
  plies[g] = 1u + (uint32_t)count_tokens(text, mv_off[g], fen_off[g + 1]);
}

__global__ void count_children_kernel(const DBoard* __restrict__ states, uint32_t n, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DBoard b = states[i];
  uint32_t c = 0;
  for_each_legal(b, [&](const DMove&) -> bool {
    ++c;
    return true;
  });
  cnt[i] = 1u + c;
}

__global__ void write_children_kernel(const DBoard* __restrict__ states, uint32_t n, const uint32_t* __restrict__ off,
                                      fnnue_pos* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DBoard b = states[i];
  uint32_t o = off[i];
  out[o++] = pack(b);
  for_each_legal(b, [&](const DMove& m) -> bool {
    DBoard c = b;
    do_move(c, m);
    out[o++] = pack(c);
    return true;
  });
}

template <int D>
__device__ uint64_t perft_dev(const DBoard& b) {
  uint64_t n = 0;
  for_each_legal(b, [&](const DMove& m) -> bool {
    if constexpr (D <= 1) {
      ++n;
    } else {
      DBoard c = b;
      do_move(c, m);
      n += perft_dev<D - 1>(c);
    }
    return true;
  });
  return n;
}

template <int D>
__global__ void perft_kernel(const DBoard* __restrict__ states, uint32_t n, unsigned long long* __restrict__ total) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(total, (unsigned long long)perft_dev<D>(states[i]));
}

}  // namespace

hipError_t BuilderScratch::get(int slot, size_t want, void** out) {
  if (want > bytes[slot]) {
    if (p[slot]) (void)hipFree(p[slot]);
    p[slot] = nullptr;
    bytes[slot] = 0;
    const size_t n = want + want / 4 + 256;
    const hipError_t e = hipMalloc(&p[slot], n);
    if (e != hipSuccess) return e;
    bytes[slot] = n;
  }
  *out = p[slot];
  return hipSuccess;
}

void BuilderScratch::release() {
  for (int i = 0; i < kSlots; ++i) {
    if (p[i]) (void)hipFree(p[i]);
    p[i] = nullptr;
    bytes[i] = 0;
  }
}

// Exclusive scan of cnt[0..n) into off[0..n], off[n] = total (hipcub).
hipError_t builder_exclusive_scan(const uint32_t* cnt, uint32_t* off, uint32_t n, hipStream_t s, BuilderScratch& ws) {
  size_t tmp_bytes = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, (int)n + 1, s);
  if (e != hipSuccess) return e;
  void* tmp = nullptr;
  if ((e = ws.get(BuilderScratch::kScan, tmp_bytes, &tmp)) != hipSuccess) return e;
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, (int)n + 1, s);
}

DBoard to_dboard(const Board& h) {
  DBoard b{};
  b.bc[0] = h.byColor[0];
  b.bc[1] = h.byColor[1];
  for (int t = 0; t < 7; ++t) b.bt[t] = t ? h.byType[t] : 0;
  for (int c = 0; c < 2; ++c)
    for (int side = 0; side < 2; ++side) {
      const int sq = h.castle_rook[c][side];
      const int sh = 8 * (2 * c + side);
      b.cr = (b.cr & ~(0xFFu << sh)) | ((uint32_t)(sq < 0 ? 0xFF : sq) << sh);
    }
  b.ep = h.ep;
  b.stm = (uint32_t)h.stm;
  b.c960 = h.chess960 ? 1 : 0;
  return b;
}

namespace {

hipError_t launch_chess_replay(const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                               const uint32_t* d_ply_off, uint32_t ngames, fnnue_pos* d_out, DBoard* d_states,
                               uint8_t* d_final, uint32_t* d_err, hipStream_t s) {
  return replay::launch_replay<ChessRules>((int)kVariantChess, d_text, d_fen_off, d_mv_off, ngames, d_ply_off, d_out,
                                           d_states, d_err, d_final, s);
}

}  // namespace

hipError_t replay_games_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                               const uint32_t* d_ply_off, uint32_t ngames, void* d_out, uint8_t* d_final,
                               uint32_t* d_err, hipStream_t s) {
  if (variant != kVariantChess)
    return replay_vgames_device(variant, d_text, d_fen_off, d_mv_off, d_ply_off, ngames,
                                static_cast<fnnue_vpos*>(d_out), nullptr, d_final, d_err, s);
  return launch_chess_replay(d_text, d_fen_off, d_mv_off, d_ply_off, ngames, static_cast<fnnue_pos*>(d_out), nullptr,
                             d_final, d_err, s);
}

BuildResult build_batch_device(const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                               uint32_t ngames, bool children, fnnue_pos* d_out, size_t cap, uint32_t* d_group_off,
                               size_t off_cap, hipStream_t s, BuilderScratch& ws, uint8_t* d_final) {
  BuildResult R;
  auto fail = [&](hipError_t e) {
    R.hip = e;
    return R;
  };
  hipError_t e;
  uint32_t *plies = nullptr, *ply_off = nullptr, *err = nullptr, *cnt = nullptr, *coff = nullptr;
  DBoard* states = nullptr;
  using W = BuilderScratch;
  if ((e = ws.get(W::kPlies, (size_t)(ngames + 1) * 4, (void**)&plies)) != hipSuccess) return fail(e);
  if ((e = ws.get(W::kPlyOff, (size_t)(ngames + 1) * 4, (void**)&ply_off)) != hipSuccess) return fail(e);
  if ((e = ws.get(W::kErr, 16, (void**)&err)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(err, 0, 16, s)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(plies + ngames, 0, 4, s)) != hipSuccess) return fail(e);
  const uint32_t bs = 64;
  hipLaunchKernelGGL(count_plies_kernel, dim3((ngames + bs - 1) / bs), dim3(bs), 0, s, d_text, d_fen_off, d_mv_off,
                     ngames, plies);
  if ((e = hipGetLastError()) != hipSuccess) return fail(e);
  if ((e = builder_exclusive_scan(plies, ply_off, ngames, s, ws)) != hipSuccess) return fail(e);
  uint32_t total_plies = 0;
  if ((e = hipMemcpyAsync(&total_plies, ply_off + ngames, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(e);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(e);
  if (!children) {
    R.n_out = total_plies;
    R.n_groups = ngames;
    if (cap < total_plies || off_cap < (size_t)ngames + 1 || !d_out || !d_group_off) {
      R.capacity = true;
      return R;
    }
    if ((e = launch_chess_replay(d_text, d_fen_off, d_mv_off, ply_off, ngames, d_out, nullptr, d_final, err, s)) !=
        hipSuccess)
      return fail(e);
    if ((e = hipMemcpyAsync(d_group_off, ply_off, (size_t)(ngames + 1) * 4, hipMemcpyDeviceToDevice, s)) !=
        hipSuccess)
      return fail(e);
  } else {
    if ((e = ws.get(W::kStates, (size_t)total_plies * sizeof(DBoard), (void**)&states)) != hipSuccess) return fail(e);
    if ((e = ws.get(W::kCnt, (size_t)(total_plies + 1) * 4, (void**)&cnt)) != hipSuccess) return fail(e);
    if ((e = ws.get(W::kCoff, (size_t)(total_plies + 1) * 4, (void**)&coff)) != hipSuccess) return fail(e);
    if ((e = launch_chess_replay(d_text, d_fen_off, d_mv_off, ply_off, ngames, nullptr, states, d_final, err, s)) !=
        hipSuccess)
      return fail(e);
    uint32_t herr[4];
    if ((e = hipMemcpyAsync(herr, err, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(e);
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(e);
    if (herr[0]) {
      R.err_code = herr[0];
      R.err_game = herr[1];
      R.err_ply = herr[2];
      return R;
    }
    if ((e = hipMemsetAsync(cnt + total_plies, 0, 4, s)) != hipSuccess) return fail(e);
    hipLaunchKernelGGL(count_children_kernel, dim3((total_plies + bs - 1) / bs), dim3(bs), 0, s, states,
                       total_plies, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return fail(e);
    if ((e = builder_exclusive_scan(cnt, coff, total_plies, s, ws)) != hipSuccess) return fail(e);
    uint32_t total = 0;
    if ((e = hipMemcpyAsync(&total, coff + total_plies, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(e);
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(e);
    R.n_out = total;
    R.n_groups = total_plies;
    if (cap < total || off_cap < (size_t)total_plies + 1 || !d_out || !d_group_off) {
      R.capacity = true;
      return R;
    }
    hipLaunchKernelGGL(write_children_kernel, dim3((total_plies + bs - 1) / bs), dim3(bs), 0, s, states,
                       total_plies, coff, d_out);
    if ((e = hipGetLastError()) != hipSuccess) return fail(e);
    if ((e = hipMemcpyAsync(d_group_off, coff, (size_t)(total_plies + 1) * 4, hipMemcpyDeviceToDevice, s)) !=
        hipSuccess)
      return fail(e);
  }
  uint32_t herr[4];
  if ((e = hipMemcpyAsync(herr, err, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(e);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(e);
  R.err_code = herr[0];
  R.err_game = herr[1];
  R.err_ply = herr[2];
  return R;
}

hipError_t perft_device(const std::vector<DBoard>& frontier, int depth, uint64_t* nodes) {
  *nodes = 0;
  if (frontier.empty()) return hipSuccess;
  if (depth < 1 || depth > 3) return hipErrorInvalidValue;
  DBoard* d = nullptr;
  unsigned long long* tot = nullptr;
  hipError_t e = hipMalloc(&d, frontier.size() * sizeof(DBoard));
  if (e != hipSuccess) return e;
  if ((e = hipMalloc(&tot, 8)) == hipSuccess && (e = hipMemset(tot, 0, 8)) == hipSuccess &&
      (e = hipMemcpy(d, frontier.data(), frontier.size() * sizeof(DBoard), hipMemcpyHostToDevice)) == hipSuccess) {
    const uint32_t n = (uint32_t)frontier.size(), bs = 64;
    if (depth == 1) hipLaunchKernelGGL(perft_kernel<1>, dim3((n + bs - 1) / bs), dim3(bs), 0, 0, d, n, tot);
    else if (depth == 2) hipLaunchKernelGGL(perft_kernel<2>, dim3((n + bs - 1) / bs), dim3(bs), 0, 0, d, n, tot);
    else hipLaunchKernelGGL(perft_kernel<3>, dim3((n + bs - 1) / bs), dim3(bs), 0, 0, d, n, tot);
    if ((e = hipGetLastError()) == hipSuccess) {
      unsigned long long h = 0;
      e = hipMemcpy(&h, tot, 8, hipMemcpyDeviceToHost);
      *nodes = h;
    }
  }
  (void)hipFree(d);
  if (tot) (void)hipFree(tot);
  return e;
}

}  // namespace fnnue
