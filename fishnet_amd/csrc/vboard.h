// vboard.h — crazyhouse and atomic rules on bitboards, one source for the host
// (fnnue_game_vpositions, fnnue_vperft) and the device batch builder
// (vbuilder.hip): FEN with holdings and promoted marks, legal moves including
// drops, do_move with pockets (crazyhouse) or explosions (atomic), packing to
// fnnue_vpos.
//
// Replaces, for the variants the reference sends to Fairy-Stockfish
// ([ref] src/queue.rs:524-552: VariantPosition::from_setup with the batch's
// variant, Uci::to_move legality, play_unchecked; flavour routing :530-539),
// what shakmaty 0.23.0 does there.  The rules (as published; the move
// generator is pinned by perft known answers in tests/test_vbuilder.py):
//  * crazyhouse: chess moves plus drops of pocket pieces on empty squares
//    (pawns not on the first or last rank); a capture puts the captured piece
//    in the capturer's pocket, as a pawn if it was promoted; a drop may not
//    leave the own king attacked, like any move.
//  * atomic: a capture removes the capturer, the captured piece and every
//    non-pawn piece on the 8 squares around the capture square (en passant:
//    around the destination); kings never capture; a move is illegal if it
//    explodes the own king, legal if it explodes the other king, and otherwise
//    legal iff the own king is not attacked afterwards, where kings standing
//    next to each other never attack (a capture next to the capturer's own
//    king would explode it).  Castling needs the king's path unattacked in
//    that sense.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/fnnue.h"

namespace fnnue {
namespace vb {

#define FNNUE_HD __host__ __device__ __forceinline__

constexpr int kCrazyhouse = FNNUE_VARIANT_CRAZYHOUSE, kAtomic = FNNUE_VARIANT_ATOMIC;
constexpr int PAWN = 1, KNIGHT = 2, BISHOP = 3, ROOK = 4, QUEEN = 5, KING = 6;
constexpr uint64_t kNotA = 0xFEFEFEFEFEFEFEFEull, kNotH = 0x7F7F7F7F7F7F7F7Full;
constexpr uint64_t kNotAB = 0xFCFCFCFCFCFCFCFCull, kNotGH = 0x3F3F3F3F3F3F3F3Full;
constexpr uint64_t kRank1 = 0xFFull, kRank8 = 0xFF00000000000000ull;

struct VBoard {
  uint64_t bc[2];     // by colour
  uint64_t bt[7];     // by piece type 1..6
  uint64_t promoted;  // crazyhouse: promoted pieces (go to the pocket as pawns)
  uint64_t pocket[2]; // pockets: byte t - 1 of pocket[c] = colour c's pieces of type t (P N B R Q)
  int8_t cr[2][2];    // castling rook squares [colour][0 king side, 1 queen side], -1 none
  int8_t ep;          // en-passant target square or -1
  uint8_t stm;
  uint8_t variant;    // kCrazyhouse / kAtomic
  uint8_t c960;       // castling needs Chess960 (king-takes-rook) notation
};

// kind: 0 move, 1 castling (to = the rook's square), 2 drop (from = -1,
// piece = the dropped type); piece = the promotion type for moves.
struct VMove {
  int8_t from, to, piece, kind;
};

FNNUE_HD int vlsb(uint64_t b) { return __builtin_ctzll(b); }
FNNUE_HD int imin(int a, int b) { return a < b ? a : b; }
FNNUE_HD int imax(int a, int b) { return a > b ? a : b; }
FNNUE_HD int vpopcnt(uint64_t b) { return __builtin_popcountll(b); }
FNNUE_HD int mkpc(int c, int t) { return (c << 3) | t; }

FNNUE_HD uint64_t knight_att(int s) {
  const uint64_t b = 1ull << s;
  return ((b << 17) & kNotA) | ((b << 15) & kNotH) | ((b << 10) & kNotAB) | ((b << 6) & kNotGH) |
         ((b >> 17) & kNotH) | ((b >> 15) & kNotA) | ((b >> 10) & kNotGH) | ((b >> 6) & kNotAB);
}
FNNUE_HD uint64_t king_att(int s) {
  const uint64_t b = 1ull << s;
  return ((b << 1) & kNotA) | ((b >> 1) & kNotH) | (b << 8) | (b >> 8) | ((b << 9) & kNotA) | ((b << 7) & kNotH) |
         ((b >> 7) & kNotA) | ((b >> 9) & kNotH);
}
FNNUE_HD uint64_t pawn_att(int c, int s) {  // squares a pawn of colour c on s attacks
  const uint64_t b = 1ull << s;
  return c == 0 ? ((b << 9) & kNotA) | ((b << 7) & kNotH) : ((b >> 7) & kNotA) | ((b >> 9) & kNotH);
}
// Sliding attacks by occluded fill (Kogge-Stone): a fixed instruction
// sequence, so device lanes holding different boards never diverge.  SH > 0
// shifts left; `mask` removes squares that wrapped around a board edge.
template <int SH>
FNNUE_HD uint64_t shl(uint64_t b) {
  if constexpr (SH > 0) return b << SH;
  else return b >> -SH;
}
template <int SH>
FNNUE_HD uint64_t fill(uint64_t gen, uint64_t empty, uint64_t mask) {
  uint64_t pro = empty & mask;
  gen |= pro & shl<SH>(gen);
  pro &= shl<SH>(pro);
  gen |= pro & shl<2 * SH>(gen);
  pro &= shl<2 * SH>(pro);
  gen |= pro & shl<4 * SH>(gen);
  return shl<SH>(gen) & mask;
}
FNNUE_HD uint64_t bishop_att(int s, uint64_t occ) {
  const uint64_t g = 1ull << s, e = ~occ;
  return fill<9>(g, e, kNotA) | fill<7>(g, e, kNotH) | fill<-7>(g, e, kNotA) | fill<-9>(g, e, kNotH);
}
FNNUE_HD uint64_t rook_att(int s, uint64_t occ) {
  const uint64_t g = 1ull << s, e = ~occ;
  return fill<8>(g, e, ~0ull) | fill<-8>(g, e, ~0ull) | fill<1>(g, e, kNotA) | fill<-1>(g, e, kNotH);
}

// Board fields by a colour / piece type known only at run time: selects and
// shifts, never a run-time array index (on the device an indexed register
// array lives in scratch memory).
FNNUE_HD uint64_t colour(const VBoard& b, int c) { return c ? b.bc[1] : b.bc[0]; }
FNNUE_HD int in_hand(const VBoard& b, int c, int t) {  // t = PAWN..QUEEN
  return (int)(((c ? b.pocket[1] : b.pocket[0]) >> (8 * (t - 1))) & 255u);
}
FNNUE_HD void hand_add(VBoard& b, int c, int t, int d) {  // the count stays within 0..255
  const uint64_t delta = (uint64_t)(int64_t)d << (8 * (t - 1));
  if (c) b.pocket[1] += delta;
  else b.pocket[0] += delta;
}
FNNUE_HD int cr_get(const VBoard& b, int c, int side) {
  return c ? (side ? b.cr[1][1] : b.cr[1][0]) : (side ? b.cr[0][1] : b.cr[0][0]);
}
FNNUE_HD void cr_set(VBoard& b, int c, int side, int v) {
  if (c) {
    if (side) b.cr[1][1] = (int8_t)v;
    else b.cr[1][0] = (int8_t)v;
  } else {
    if (side) b.cr[0][1] = (int8_t)v;
    else b.cr[0][0] = (int8_t)v;
  }
}
FNNUE_HD void cr_clear(VBoard& b, int c) {
  cr_set(b, c, 0, -1);
  cr_set(b, c, 1, -1);
}

FNNUE_HD uint64_t occupied(const VBoard& b) { return b.bc[0] | b.bc[1]; }

FNNUE_HD int type_at(const VBoard& b, uint64_t m) {  // 0: empty
  int t = 0;
  for (int k = 1; k <= KING; ++k) t = (b.bt[k] & m) ? k : t;
  return t;
}
FNNUE_HD int piece_at(const VBoard& b, int s) {
  const uint64_t m = 1ull << s;
  const int t = type_at(b, m);
  return t ? mkpc((b.bc[1] & m) ? 1 : 0, t) : 0;
}
FNNUE_HD void put(VBoard& b, int s, int pc) {
  const uint64_t m = 1ull << s;
  const int c = pc >> 3, t = pc & 7;
  b.bc[0] |= c ? 0ull : m;
  b.bc[1] |= c ? m : 0ull;
  for (int k = 1; k <= KING; ++k) b.bt[k] |= k == t ? m : 0ull;
}
FNNUE_HD void remove_sq(VBoard& b, int s) {
  const uint64_t m = ~(1ull << s);
  b.bc[0] &= m;
  b.bc[1] &= m;
  for (int t = 1; t < 7; ++t) b.bt[t] &= m;
  b.promoted &= m;
}
FNNUE_HD int king_sq(const VBoard& b, int c) {
  const uint64_t k = b.bt[KING] & colour(b, c);
  return k ? vlsb(k) : -1;
}

// Is square s attacked by colour `by` (occupancy occ)?  Plain chess attacks.
FNNUE_HD bool attacked(const VBoard& b, int s, int by, uint64_t occ) {
  const uint64_t them = colour(b, by);
  return ((pawn_att(by ^ 1, s) & b.bt[PAWN]) | (knight_att(s) & b.bt[KNIGHT]) | (king_att(s) & b.bt[KING]) |
          (bishop_att(s, occ) & (b.bt[BISHOP] | b.bt[QUEEN])) | (rook_att(s, occ) & (b.bt[ROOK] | b.bt[QUEEN]))) &
         them;
}

// Would the side to move's king be in danger on square s?  Atomic: a king
// next to the other king cannot be captured (the capture would explode the
// capturer's king), and the other king itself never captures.
FNNUE_HD bool king_danger(const VBoard& b, int s, int us, uint64_t occ) {
  const int them = us ^ 1;
  if (b.variant == kAtomic) {
    const int kt = king_sq(b, them);
    if (kt >= 0 && (king_att(s) & (1ull << kt))) return false;
    VBoard c = b;
    c.bt[KING] &= ~colour(b, them);  // kings do not capture in atomic
    return attacked(c, s, them, occ);
  }
  return attacked(b, s, them, occ);
}

FNNUE_HD void do_move(VBoard& b, const VMove& m) {
  const int us = b.stm, them = us ^ 1;
  int new_ep = -1;
  if (m.kind == 2) {
    put(b, m.to, mkpc(us, m.piece));
    hand_add(b, us, m.piece, -1);
  } else if (m.kind == 1) {
    const int back = us == 0 ? 0 : 56;
    const bool king_side = m.to > m.from;
    const int kto = back + (king_side ? 6 : 2), rto = back + (king_side ? 5 : 3);
    const bool rook_promoted = (b.promoted >> m.to) & 1;
    remove_sq(b, m.from);
    remove_sq(b, m.to);
    put(b, kto, mkpc(us, KING));
    put(b, rto, mkpc(us, ROOK));
    if (rook_promoted) b.promoted |= 1ull << rto;
    cr_clear(b, us);
  } else {
    const int pc = piece_at(b, m.from);
    int cap_sq = m.to;
    if ((pc & 7) == PAWN && m.to == b.ep && ((m.from ^ m.to) & 7) && !(occupied(b) & (1ull << m.to)))
      cap_sq = m.to + (us == 0 ? -8 : 8);
    const int cap = piece_at(b, cap_sq);
    const bool cap_promoted = (b.promoted >> cap_sq) & 1;
    const bool was_promoted = (b.promoted >> m.from) & 1;
    if (cap) {
      if (b.variant == kCrazyhouse) {
        const int t = cap_promoted ? PAWN : (cap & 7);
        if (in_hand(b, us, t) < 255) hand_add(b, us, t, 1);
      }
      remove_sq(b, cap_sq);
    }
    remove_sq(b, m.from);
    put(b, m.to, m.piece ? mkpc(us, m.piece) : pc);
    if (b.variant == kCrazyhouse && (m.piece || was_promoted)) b.promoted |= 1ull << m.to;
    if (cap && b.variant == kAtomic) {
      remove_sq(b, m.to);  // the capturer explodes with its victim
      for (uint64_t nb = king_att(m.to) & occupied(b) & ~b.bt[PAWN]; nb; nb &= nb - 1) remove_sq(b, vlsb(nb));
    }
    if ((pc & 7) == PAWN && (m.from ^ m.to) == 16) new_ep = (m.from + m.to) / 2;
    if ((pc & 7) == KING) cr_clear(b, us);
  }
  // castling rights end with the rook (moved, captured, exploded) or the king
  for (int c = 0; c < 2; ++c) {
    if (king_sq(b, c) < 0) cr_clear(b, c);
    for (int side = 0; side < 2; ++side) {
      const int r = b.cr[c][side];
      if (r >= 0 && piece_at(b, r) != mkpc(c, ROOK)) b.cr[c][side] = -1;
    }
  }
  (void)them;
  b.ep = (int8_t)new_ep;
  b.stm = (uint8_t)(us ^ 1);
}

FNNUE_HD bool legal_after(const VBoard& before, const VBoard& after) {
  const int us = before.stm, them = us ^ 1;
  const int ku = king_sq(after, us);
  if (ku < 0) return false;  // own king exploded (atomic) or captured
  if (before.variant == kAtomic) {
    const int kt = king_sq(after, them);
    if (kt < 0) return true;  // the other king exploded: the game ends here
  }
  // `after` has the other side to move: ask whether `us`'s king is in danger there
  VBoard a = after;
  a.stm = (uint8_t)us;
  return !king_danger(a, ku, us, occupied(a));
}

// Castling conditions for the rook on rsq (side 0 king side, 1 queen side):
// rook in place, the squares between and the destinations empty, the king not
// in danger on its square or on any square it passes (the king lifted off
// its square for the latter).
FNNUE_HD bool castle_ok(const VBoard& b, int ksq, int rsq, int side) {
  const int us = b.stm;
  const int back = us == 0 ? 0 : 56;
  const uint64_t occ = occupied(b);
  if (rsq < 0 || piece_at(b, rsq) != mkpc(us, ROOK)) return false;
  const int kto = back + (side == 0 ? 6 : 2), rto = back + (side == 0 ? 5 : 3);
  const int lo = imin(imin(ksq, rsq), imin(kto, rto)), hi = imax(imax(ksq, rsq), imax(kto, rto));
  const uint64_t span = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
  if (occ & span & ~(1ull << ksq) & ~(1ull << rsq)) return false;
  if (king_danger(b, ksq, us, occ)) return false;
  const int step = kto > ksq ? 1 : -1;
  const uint64_t occ2 = occ & ~(1ull << ksq);
  bool ok = true;
  for (int t = ksq; t != kto && ok;) {
    t += step;
    if (king_danger(b, t, us, occ2)) ok = false;
  }
  return ok;
}

// Is m one of for_each_legal's candidate moves (before the legal_after
// filter)?  Drops: a pocket piece on an empty square (pawns not on the first
// or last rank); moves: as the generator makes them (atomic kings never
// capture, en passant onto an empty square only, castling by castle_ok).
FNNUE_HD bool pseudo_member(const VBoard& b, const VMove& m) {
  const int us = b.stm, them = us ^ 1;
  const uint64_t occ = occupied(b), own = colour(b, us), opp = colour(b, them);
  const uint64_t tm = 1ull << m.to;
  if (m.kind == 2) {
    if (b.variant != kCrazyhouse || m.piece < PAWN || m.piece > QUEEN || !in_hand(b, us, m.piece)) return false;
    uint64_t empty = ~occ;
    if (m.piece == PAWN) empty &= ~(kRank1 | kRank8);
    return (empty & tm) != 0;
  }
  const uint64_t fm = 1ull << m.from;
  if (!(own & fm)) return false;
  if (m.kind == 1) {
    const int ksq = king_sq(b, us), back = us == 0 ? 0 : 56;
    if (m.piece || m.from != ksq || (ksq & 56) != back) return false;
    const int side = cr_get(b, us, 0) == m.to ? 0 : cr_get(b, us, 1) == m.to ? 1 : -1;
    return side >= 0 && castle_ok(b, ksq, m.to, side);
  }
  const int t = type_at(b, fm);
  if (t == PAWN) {
    const int r = m.from >> 3, up = us == 0 ? 8 : -8;
    const bool promo_ok = r == (us == 0 ? 6 : 1) ? m.piece != 0 : m.piece == 0;
    const int t1 = m.from + up, t2 = t1 + up;
    bool ok = false;
    if (!(occ & (1ull << t1))) {
      ok = m.to == t1 && promo_ok;
      ok = ok || (m.to == t2 && r == (us == 0 ? 1 : 6) && !(occ & (1ull << t2)) && m.piece == 0);
    }
    const uint64_t pa = pawn_att(us, m.from);
    ok = ok || ((pa & opp & tm) && promo_ok);
    ok = ok || (b.ep >= 0 && m.to == b.ep && (pa & tm) && !(occ & tm) && m.piece == 0);
    return ok;
  }
  uint64_t targets;
  if (t == KNIGHT) targets = knight_att(m.from);
  else if (t == BISHOP) targets = bishop_att(m.from, occ);
  else if (t == ROOK) targets = rook_att(m.from, occ);
  else if (t == QUEEN) targets = bishop_att(m.from, occ) | rook_att(m.from, occ);
  else targets = king_att(m.from) & (b.variant == kAtomic ? ~opp : ~0ull);  // atomic kings never capture
  return m.piece == 0 && (targets & ~own & tm) != 0;
}

// Legal moves: pieces by square (pawn pushes with promotions Q R B N, double
// push, captures, en passant), castling king side then queen side, then drops
// (crazyhouse: piece types P N B R Q, squares a1..h8).  f(move) returns false to
// stop early.  from_mask limits the moving pieces; want_moves / want_drops
// select the two kinds.
template <class F>
__host__ __device__ void for_each_legal(const VBoard& b, F&& f, uint64_t from_mask = ~0ull, bool want_moves = true,
                                        bool want_drops = true) {
  const int us = b.stm, them = us ^ 1;
  const uint64_t occ = occupied(b), own = colour(b, us), opp = colour(b, them);
  const bool atomic = b.variant == kAtomic;
  auto emit = [&](int from, int to, int piece, int kind) -> bool {
    const VMove m{(int8_t)from, (int8_t)to, (int8_t)piece, (int8_t)kind};
    VBoard c = b;
    do_move(c, m);
    return !legal_after(b, c) || f(m);
  };
  if (want_moves) {
    const int up = us == 0 ? 8 : -8;
    const int rank7 = us == 0 ? 6 : 1, rank2 = us == 0 ? 1 : 6;
    for (uint64_t pcs = own & from_mask; pcs; pcs &= pcs - 1) {
      const int s = vlsb(pcs);
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
          if (!pawn_to(vlsb(a))) return;
        if (b.ep >= 0 && (pawn_att(us, s) & (1ull << b.ep)) && !(occ & (1ull << b.ep)) && !emit(s, b.ep, 0, 0))
          return;
        continue;
      }
      uint64_t targets;
      if (b.bt[KNIGHT] & sm) targets = knight_att(s);
      else if (b.bt[BISHOP] & sm) targets = bishop_att(s, occ);
      else if (b.bt[ROOK] & sm) targets = rook_att(s, occ);
      else if (b.bt[QUEEN] & sm) targets = bishop_att(s, occ) | rook_att(s, occ);
      else targets = king_att(s) & (atomic ? ~opp : ~0ull);  // atomic kings never capture
      for (uint64_t t = targets & ~own; t; t &= t - 1)
        if (!emit(s, vlsb(t), 0, 0)) return;
    }
    const int ksq = king_sq(b, us);
    const int back = us == 0 ? 0 : 56;
    if (ksq >= 0 && (ksq & 56) == back && ((from_mask >> ksq) & 1)) {
      for (int side = 0; side < 2; ++side) {
        const int rsq = cr_get(b, us, side);
        if (castle_ok(b, ksq, rsq, side) && !emit(ksq, rsq, 0, 1)) return;
      }
    }
  }
  if (want_drops && b.variant == kCrazyhouse) {
    for (int pt = PAWN; pt <= QUEEN; ++pt) {
      if (!in_hand(b, us, pt)) continue;
      uint64_t empty = ~occ;
      if (pt == PAWN) empty &= ~(kRank1 | kRank8);
      for (uint64_t t = empty; t; t &= t - 1)
        if (!emit(-1, vlsb(t), pt, 2)) return;
    }
  }
}

// Game-end flags of a position (builder.h kFinal*): no legal move (bit 0),
// the side to move's king attacked (bit 1), its king exploded (bit 2, atomic).
FNNUE_HD uint8_t final_state(const VBoard& b) {
  bool any = false;
  for_each_legal(b, [&](const VMove&) -> bool {
    any = true;
    return false;
  });
  const int us = b.stm, k = king_sq(b, us);
  const bool check = k >= 0 && king_danger(b, k, us, occupied(b));
  return (uint8_t)((any ? 0 : 1) | (check ? 2 : 0) | (k < 0 ? 4 : 0));
}

FNNUE_HD fnnue_vpos pack(const VBoard& b) {
  fnnue_vpos p;
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = 0;
  for (uint64_t o = occupied(b); o; o &= o - 1) {
    const int s = vlsb(o);
    w[s >> 3] |= (uint32_t)piece_at(b, s) << (4 * (s & 7));
  }
  uint8_t* d = reinterpret_cast<uint8_t*>(&p);
  for (int i = 0; i < 48; ++i) d[i] = 0;
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 4; ++k) d[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
  d[32] = b.stm;
  for (int c = 0; c < 2; ++c)
    for (int t = 0; t < 5; ++t) d[33 + 5 * c + t] = (uint8_t)(b.pocket[c] >> (8 * t));
  return p;
}

FNNUE_HD bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// Next whitespace-separated token of text[p, end): its length (0 = none).
FNNUE_HD int next_token(const char* text, uint32_t& p, uint32_t end, uint32_t& start) {
  while (p < end && is_space(text[p])) ++p;
  start = p;
  while (p < end && !is_space(text[p])) ++p;
  return (int)(p - start);
}

FNNUE_HD int piece_type_of(char ch) {
  switch (ch | 32) {
    case 'p': return PAWN;
    case 'n': return KNIGHT;
    case 'b': return BISHOP;
    case 'r': return ROOK;
    case 'q': return QUEEN;
    case 'k': return KING;
    default: return 0;
  }
}

// FEN of a variant position: placement (a '~' after a piece marks it
// promoted), crazyhouse holdings as "[...]" after the placement or as a ninth
// placement field ("/..."), then side to move, castling (KQkq, Shredder or
// X-FEN), en passant.  Returns false on malformed input.
FNNUE_HD bool parse_fen(const char* text, uint32_t p, uint32_t end, int variant, VBoard& b) {
  for (int i = 0; i < 2; ++i) b.bc[i] = 0;
  for (int i = 0; i < 7; ++i) b.bt[i] = 0;
  b.promoted = 0;
  b.pocket[0] = b.pocket[1] = 0;
  b.cr[0][0] = b.cr[0][1] = b.cr[1][0] = b.cr[1][1] = -1;
  b.ep = -1;
  b.stm = 0;
  b.variant = (uint8_t)variant;
  b.c960 = 0;
  uint32_t st;
  int len = next_token(text, p, end, st);
  if (len == 0) return false;
  int r = 7, f = 0, last = -1;
  bool holdings = false;
  for (uint32_t i = st; i < st + (uint32_t)len; ++i) {
    const char ch = text[i];
    if (holdings) {
      if (ch == ']') break;
      if (ch == '-') continue;
      const int t = piece_type_of(ch);
      if (!t || t == KING || variant != kCrazyhouse) return false;
      const int col = (ch >= 'a' && ch <= 'z') ? 1 : 0;
      if (in_hand(b, col, t) == 255) return false;
      hand_add(b, col, t, 1);
      continue;
    }
    if (ch == '[') {
      if (r != 0 || f != 8) return false;
      holdings = true;
      continue;
    }
    if (ch == '~') {
      if (last < 0) return false;
      b.promoted |= 1ull << last;
      continue;
    }
    if (ch == '/') {
      if (f != 8) return false;
      if (r == 0) {  // a ninth field: holdings
        holdings = true;
        continue;
      }
      --r;
      f = 0;
      continue;
    }
    if (ch >= '1' && ch <= '8') {
      f += ch - '0';
      if (f > 8) return false;
      last = -1;
      continue;
    }
    const int t = piece_type_of(ch);
    if (!t || r < 0 || f > 7 || !((ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z'))) return false;
    last = r * 8 + f;
    put(b, last, mkpc((ch >= 'a' && ch <= 'z') ? 1 : 0, t));
    ++f;
  }
  if (!holdings && (r != 0 || f != 8)) return false;
  len = next_token(text, p, end, st);
  if (len != 1 || (text[st] != 'w' && text[st] != 'b')) return false;
  b.stm = text[st] == 'w' ? 0 : 1;
  if (vpopcnt(b.bt[KING] & b.bc[0]) != 1 || vpopcnt(b.bt[KING] & b.bc[1]) != 1) return false;
  uint32_t cst;
  const int clen = next_token(text, p, end, cst);
  if (clen > 0 && !(clen == 1 && text[cst] == '-')) {
    for (uint32_t i = cst; i < cst + (uint32_t)clen; ++i) {
      const char ch = text[i];
      const int col = (ch >= 'a' && ch <= 'z') ? 1 : 0;
      const char lc = (char)(ch | 32);
      const int back = col == 0 ? 0 : 56;
      const int k = king_sq(b, col);
      const int rook = mkpc(col, ROOK);
      int rsq = -1, side = -1;
      if ((k & 56) != back) continue;
      if (lc == 'k') side = 0;
      else if (lc == 'q') side = 1;
      else if (lc >= 'a' && lc <= 'h') side = 2;
      else return false;
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
      if (rsq >= 0 && ((k & 7) != 4 || (rsq & 7) != (side == 0 ? 7 : 0))) b.c960 = 1;
    }
  }
  uint32_t est;
  const int elen = next_token(text, p, end, est);
  if (elen == 2 && text[est] >= 'a' && text[est] <= 'h' && text[est + 1] >= '1' && text[est + 1] <= '8')
    b.ep = (int8_t)((text[est + 1] - '1') * 8 + (text[est] - 'a'));
  return true;
}

// The legal move a decoded token names: a drop of `piece` on `to` (drop), or
// the move from `from` to `to` with promotion `piece` (0 none), castling as
// king-takes-rook or (standard positions) the king's two-square step.
FNNUE_HD bool match_decoded(const VBoard& b, int from, int to, int piece, bool drop, VMove& out) {
  bool found = false;
  if (drop) {
    for_each_legal(b, [&](const VMove& m) -> bool {
      if (m.piece == piece && m.to == to) {
        out = m;
        found = true;
        return false;
      }
      return true;
    }, 0ull, false, true);
    return found;
  }
  for_each_legal(b, [&](const VMove& m) -> bool {
    if (m.from != from || (m.kind != 1 && m.piece != piece) || (m.kind == 1 && piece)) return true;
    const bool hit = m.to == to || (m.kind == 1 && !b.c960 && to == (m.from & 56) + (m.to > m.from ? 6 : 2));
    if (hit) {
      out = m;
      found = true;
    }
    return !hit;
  }, 1ull << from, true, false);
  return found;
}

// The legal move whose UCI text equals the token: "e2e4", "e7e8q", castling as
// king-takes-rook or (standard positions) the king's two-square step, drops
// as "P@e4" (either case).
FNNUE_HD bool match_uci(const VBoard& b, const char* tok, int len, VMove& out) {
  auto sqr = [&](int i) -> int {
    const char f = tok[i], r = tok[i + 1];
    return (f >= 'a' && f <= 'h' && r >= '1' && r <= '8') ? (r - '1') * 8 + (f - 'a') : -1;
  };
  if (len == 4 && tok[1] == '@') {
    const int pt = piece_type_of(tok[0]), to = sqr(2);
    if (!pt || pt == KING || to < 0) return false;
    return match_decoded(b, -1, to, pt, true, out);
  }
  if (len != 4 && len != 5) return false;
  const int from = sqr(0), to = sqr(2);
  if (from < 0 || to < 0) return false;
  int promo = 0;
  if (len == 5) {
    promo = piece_type_of(tok[4]);
    if (!promo || promo == PAWN || promo == KING) return false;
  }
  return match_decoded(b, from, to, promo, false, out);
}

#undef FNNUE_HD

// UCI text of a legal move (host): drops "N@f3", castling king-takes-rook in
// Chess960 positions and the king's two-square step otherwise, promotions
// "e7e8q".
inline std::string vuci(const VBoard& b, const VMove& m) {
  auto sq = [](int s) { return std::string{(char)('a' + (s & 7)), (char)('1' + (s >> 3))}; };
  if (m.kind == 2) return std::string(1, "PNBRQ"[m.piece - 1]) + "@" + sq(m.to);
  int to = m.to;
  if (m.kind == 1 && !b.c960) to = (m.from & 56) + (m.to > m.from ? 6 : 2);
  std::string u = sq(m.from) + sq(to);
  if (m.kind == 0 && m.piece) u += "nbrq"[m.piece - 2];
  return u;
}

}  // namespace vb
}  // namespace fnnue
