// board.cpp — legal move generation and FEN/UCI handling for the batch builder.
// Semantics follow the reference's batch expansion (src/queue.rs:524-606,
// shakmaty CastlingMode::Chess960) and Stockfish's Position::set/do_move for
// what the NNUE features see (piece placement + side to move).
#include "board.h"

#include <cstring>
#include <sstream>

namespace fnnue {

namespace {

uint64_t KNIGHT_ATT[64], KING_ATT[64], PAWN_ATT[2][64];
const int ROOK_DIRS[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
const int BISHOP_DIRS[4][2] = {{1, 1}, {1, -1}, {-1, 1}, {-1, -1}};

struct TableInit {
  TableInit() {
    for (int s = 0; s < 64; ++s) {
      int r = s >> 3, f = s & 7;
      uint64_t n = 0, k = 0;
      static const int kn[8][2] = {{1, 2}, {2, 1}, {2, -1}, {1, -2}, {-1, -2}, {-2, -1}, {-2, 1}, {-1, 2}};
      for (auto& d : kn) {
        int rr = r + d[0], ff = f + d[1];
        if (rr >= 0 && rr < 8 && ff >= 0 && ff < 8) n |= 1ull << (rr * 8 + ff);
      }
      for (int dr = -1; dr <= 1; ++dr)
        for (int df = -1; df <= 1; ++df) {
          if (!dr && !df) continue;
          int rr = r + dr, ff = f + df;
          if (rr >= 0 && rr < 8 && ff >= 0 && ff < 8) k |= 1ull << (rr * 8 + ff);
        }
      KNIGHT_ATT[s] = n;
      KING_ATT[s] = k;
      uint64_t pw = 0, pb = 0;
      if (r < 7) { if (f > 0) pw |= 1ull << (s + 7); if (f < 7) pw |= 1ull << (s + 9); }
      if (r > 0) { if (f > 0) pb |= 1ull << (s - 9); if (f < 7) pb |= 1ull << (s - 7); }
      PAWN_ATT[WHITE][s] = pw;
      PAWN_ATT[BLACK][s] = pb;
    }
  }
} table_init;

uint64_t slide(int s, const int dirs[4][2], uint64_t occ) {
  uint64_t a = 0;
  int r0 = s >> 3, f0 = s & 7;
  for (int d = 0; d < 4; ++d) {
    int r = r0 + dirs[d][0], f = f0 + dirs[d][1];
    while (r >= 0 && r < 8 && f >= 0 && f < 8) {
      int t = r * 8 + f;
      a |= 1ull << t;
      if (occ & (1ull << t)) break;
      r += dirs[d][0];
      f += dirs[d][1];
    }
  }
  return a;
}

inline int lsb(uint64_t b) { return __builtin_ctzll(b); }

}  // namespace

void Board::clear() {
  std::memset(sq, 0, sizeof(sq));
  byColor[0] = byColor[1] = 0;
  for (auto& t : byType) t = 0;
  stm = WHITE;
  ep = -1;
  castle_rook[0][0] = castle_rook[0][1] = castle_rook[1][0] = castle_rook[1][1] = -1;
  halfmove = 0;
  fullmove = 1;
  chess960 = false;
}

void Board::put(int s, int pc) {
  sq[s] = (uint8_t)pc;
  byColor[color_of(pc)] |= 1ull << s;
  byType[type_of(pc)] |= 1ull << s;
  byType[0] |= 1ull << s;
}

void Board::remove(int s) {
  int pc = sq[s];
  if (!pc) return;
  sq[s] = 0;
  byColor[color_of(pc)] &= ~(1ull << s);
  byType[type_of(pc)] &= ~(1ull << s);
  byType[0] &= ~(1ull << s);
}

int Board::king_sq(int c) const {
  uint64_t k = byType[KING] & byColor[c];
  return k ? lsb(k) : -1;
}

bool Board::attacked(int s, int by, uint64_t occ) const {
  const uint64_t them = byColor[by];
  if (PAWN_ATT[by ^ 1][s] & byType[PAWN] & them) return true;
  if (KNIGHT_ATT[s] & byType[KNIGHT] & them) return true;
  if (KING_ATT[s] & byType[KING] & them) return true;
  if (slide(s, BISHOP_DIRS, occ) & (byType[BISHOP] | byType[QUEEN]) & them) return true;
  if (slide(s, ROOK_DIRS, occ) & (byType[ROOK] | byType[QUEEN]) & them) return true;
  return false;
}

void Board::do_move(const Move& m) {
  const int us = stm, them = us ^ 1;
  const int pc = sq[m.from];
  const int back = us == WHITE ? 0 : 56;
  int new_ep = -1;
  bool reset50 = false;
  if (m.castle) {
    const int rook_sq = m.to;
    const bool king_side = rook_sq > m.from;
    const int kto = back + (king_side ? 6 : 2), rto = back + (king_side ? 5 : 3);
    const int rook = sq[rook_sq];
    remove(m.from);
    remove(rook_sq);
    put(kto, pc);
    put(rto, rook);
    castle_rook[us][0] = castle_rook[us][1] = -1;
  } else {
    if (sq[m.to]) { remove(m.to); reset50 = true; }
    if (type_of(pc) == PAWN) {
      reset50 = true;
      if (m.to == ep && (m.from & 7) != (m.to & 7)) remove(m.to + (us == WHITE ? -8 : 8));
      if ((m.from ^ m.to) == 16) new_ep = (m.from + m.to) / 2;
    }
    remove(m.from);
    put(m.to, m.promo ? make_piece(us, m.promo) : pc);
    if (type_of(pc) == KING) castle_rook[us][0] = castle_rook[us][1] = -1;
    for (int c = 0; c < 2; ++c)
      for (int side = 0; side < 2; ++side)
        if (castle_rook[c][side] == m.from || castle_rook[c][side] == m.to) castle_rook[c][side] = -1;
  }
  (void)them;
  ep = new_ep;
  halfmove = reset50 ? 0 : halfmove + 1;
  if (us == BLACK) ++fullmove;
  stm = them;
}

int Board::pseudo_moves(Move* buf) const {
  const int us = stm, them = us ^ 1;
  const uint64_t occ = occupied(), own = byColor[us], opp = byColor[them];
  int nm = 0;
  auto add = [&](int f, int t, int promo, int castle) { buf[nm++] = Move{(uint8_t)f, (uint8_t)t, (uint8_t)promo, (uint8_t)castle}; };
  const int up = us == WHITE ? 8 : -8;
  const int rank7 = us == WHITE ? 6 : 1, rank2 = us == WHITE ? 1 : 6;
  for (uint64_t b = own; b; b &= b - 1) {
    const int s = lsb(b), pt = type_of(sq[s]);
    uint64_t targets = 0;
    switch (pt) {
      case PAWN: {
        const int r = s >> 3;
        auto add_pawn = [&](int t) {
          if (r == rank7) for (int p = QUEEN; p >= KNIGHT; --p) add(s, t, p, 0);
          else add(s, t, 0, 0);
        };
        const int t1 = s + up;
        if (!(occ & (1ull << t1))) {
          add_pawn(t1);
          const int t2 = t1 + up;
          if (r == rank2 && !(occ & (1ull << t2))) add(s, t2, 0, 0);
        }
        for (uint64_t a = PAWN_ATT[us][s] & opp; a; a &= a - 1) add_pawn(lsb(a));
        if (ep >= 0 && (PAWN_ATT[us][s] & (1ull << ep))) add(s, ep, 0, 0);
        continue;
      }
      case KNIGHT: targets = KNIGHT_ATT[s]; break;
      case BISHOP: targets = slide(s, BISHOP_DIRS, occ); break;
      case ROOK: targets = slide(s, ROOK_DIRS, occ); break;
      case QUEEN: targets = slide(s, BISHOP_DIRS, occ) | slide(s, ROOK_DIRS, occ); break;
      case KING: targets = KING_ATT[s]; break;
    }
    for (uint64_t t = targets & ~own; t; t &= t - 1) add(s, lsb(t), 0, 0);
  }
  // Castling (Chess960 rules; standard chess is the special case).
  const int ksq = king_sq(us);
  const int back = us == WHITE ? 0 : 56;
  if (ksq >= 0 && (ksq & 56) == back) {
    for (int side = 0; side < 2; ++side) {
      const int rsq = castle_rook[us][side];
      if (rsq < 0 || sq[rsq] != make_piece(us, ROOK)) continue;
      const int kto = back + (side == 0 ? 6 : 2), rto = back + (side == 0 ? 5 : 3);
      int lo = ksq, hi = ksq;
      for (int x : {rsq, kto, rto}) { lo = x < lo ? x : lo; hi = x > hi ? x : hi; }
      bool ok = true;
      for (int t = lo; t <= hi && ok; ++t)
        if (t != ksq && t != rsq && sq[t]) ok = false;
      if (!ok) continue;
      if (attacked(ksq, them, occ)) continue;
      const int step = kto > ksq ? 1 : -1;
      for (int t = ksq; t != kto && ok; ) { t += step; if (attacked(t, them, occ)) ok = false; }
      if (ok) add(ksq, rsq, 0, 1);
    }
  }
  return nm;
}

bool Board::is_legal(const Move& m) const {
  Board c = *this;
  c.do_move(m);
  const int k = c.king_sq(stm);
  return k >= 0 && !c.attacked(k, stm ^ 1, c.occupied());
}

void Board::legal_moves(std::vector<Move>& out) const {
  out.clear();
  Move buf[256];
  const int nm = pseudo_moves(buf);
  for (int i = 0; i < nm; ++i)
    if (is_legal(buf[i])) out.push_back(buf[i]);
}

bool Board::random_legal_move(uint64_t& rng, Move& out) const {
  Move buf[256];
  int nm = pseudo_moves(buf);
  while (nm > 0) {
    const int i = (int)(splitmix64(rng) % (uint64_t)nm);
    if (is_legal(buf[i])) { out = buf[i]; return true; }
    buf[i] = buf[--nm];
  }
  return false;
}

static std::string sqname(int s) {
  std::string r;
  r += char('a' + (s & 7));
  r += char('1' + (s >> 3));
  return r;
}

std::string Board::uci(const Move& m, bool chess960_castling) const {
  int to = m.to;
  if (m.castle && !chess960_castling) to = (m.from & 56) + (m.to > m.from ? 6 : 2);
  std::string s = sqname(m.from) + sqname(to);
  if (m.promo) s += " pnbrqk"[m.promo];
  return s;
}

fnnue_pos Board::pack() const {
  fnnue_pos p;
  std::memset(&p, 0, sizeof(p));
  for (int s = 0; s < 64; ++s) p.sq[s >> 1] |= (uint8_t)(sq[s] << (4 * (s & 1)));
  p.stm = (uint8_t)stm;
  return p;
}

std::string Board::fen() const {
  std::ostringstream o;
  for (int r = 7; r >= 0; --r) {
    int empty = 0;
    for (int f = 0; f < 8; ++f) {
      int pc = sq[r * 8 + f];
      if (!pc) { ++empty; continue; }
      if (empty) { o << empty; empty = 0; }
      o << (color_of(pc) == WHITE ? " PNBRQK"[type_of(pc)] : " pnbrqk"[type_of(pc)]);
    }
    if (empty) o << empty;
    if (r) o << '/';
  }
  o << (stm == WHITE ? " w " : " b ");
  std::string c;
  for (int col = 0; col < 2; ++col)
    for (int side = 0; side < 2; ++side) {
      int r = castle_rook[col][side];
      if (r < 0) continue;
      char ch = chess960 ? char('a' + (r & 7)) : (side == 0 ? 'k' : 'q');
      c += col == WHITE ? char(ch - 32) : ch;
    }
  o << (c.empty() ? "-" : c) << ' ' << (ep >= 0 ? sqname(ep) : "-") << ' ' << halfmove << ' ' << fullmove;
  return o.str();
}

bool board_from_fen(const char* fen, Board& b, std::string* err) {
  b.clear();
  std::istringstream in(fen ? fen : "");
  std::string place, side, castle = "-", eps = "-";
  int hm = 0, fm = 1;
  if (!(in >> place >> side)) { if (err) *err = "FEN needs placement and side to move"; return false; }
  in >> castle >> eps;
  if (!(in >> hm)) hm = 0;
  if (!(in >> fm)) fm = 1;
  int r = 7, f = 0;
  for (char ch : place) {
    if (ch == '/') { if (f != 8) { if (err) *err = "FEN rank length"; return false; } --r; f = 0; continue; }
    if (ch >= '1' && ch <= '8') { f += ch - '0'; if (f > 8) { if (err) *err = "FEN rank overflow"; return false; } continue; }
    const char* w = "PNBRQK";
    const char* bl = "pnbrqk";
    int pc = 0;
    for (int i = 0; i < 6; ++i) { if (ch == w[i]) pc = make_piece(WHITE, i + 1); if (ch == bl[i]) pc = make_piece(BLACK, i + 1); }
    if (!pc || r < 0 || f > 7) { if (err) *err = std::string("FEN bad piece char '") + ch + "'"; return false; }
    b.put(r * 8 + f, pc);
    ++f;
  }
  if (r != 0 || f != 8) { if (err) *err = "FEN must have 8 ranks"; return false; }
  if (side == "w") b.stm = WHITE;
  else if (side == "b") b.stm = BLACK;
  else { if (err) *err = "FEN side to move"; return false; }
  if (__builtin_popcountll(b.byType[KING] & b.byColor[WHITE]) != 1 ||
      __builtin_popcountll(b.byType[KING] & b.byColor[BLACK]) != 1) {
    if (err) *err = "FEN needs exactly one king per side";
    return false;
  }
  if (castle != "-") {
    for (char ch : castle) {
      const int col = (ch >= 'a' && ch <= 'z') ? BLACK : WHITE;
      const char lc = (char)(ch | 32);
      const int back = col == WHITE ? 0 : 56;
      const int k = b.king_sq(col);
      if ((k & 56) != back) continue;
      const int rook = make_piece(col, ROOK);
      int rsq = -1, side = -1;
      if (lc == 'k') {
        for (int x = back + 7; x > k; --x) if (b.sq[x] == rook) { rsq = x; break; }
        side = 0;
      } else if (lc == 'q') {
        for (int x = back; x < k; ++x) if (b.sq[x] == rook) { rsq = x; break; }
        side = 1;
      } else if (lc >= 'a' && lc <= 'h') {
        rsq = back + (lc - 'a');
        if (b.sq[rsq] != rook) rsq = -1;
        side = rsq > k ? 0 : 1;
        b.chess960 = true;
      } else {
        if (err) *err = "FEN castling field";
        return false;
      }
      if (rsq >= 0) b.castle_rook[col][side] = rsq;
    }
  }
  for (int col = 0; col < 2; ++col) {
    const int k = b.king_sq(col);
    for (int side = 0; side < 2; ++side) {
      const int rsq = b.castle_rook[col][side];
      if (rsq < 0) continue;
      if ((k & 7) != 4 || ((rsq & 7) != (side == 0 ? 7 : 0))) b.chess960 = true;
    }
  }
  if (eps != "-" && eps.size() == 2 && eps[0] >= 'a' && eps[0] <= 'h' && eps[1] >= '1' && eps[1] <= '8')
    b.ep = (eps[1] - '1') * 8 + (eps[0] - 'a');
  b.halfmove = hm;
  b.fullmove = fm;
  return true;
}

// The first legal move that prints as the token (either castling notation
// outside Chess960).  Every move prints its own from-square first, so only
// the pseudo-legal moves from the token's first square are checked for
// legality and printed: the same first match as scanning every legal move.
bool parse_uci(const Board& b, const char* uci, Move& out) {
  const std::string u(uci ? uci : "");
  if (u.size() < 4 || u[0] < 'a' || u[0] > 'h' || u[1] < '1' || u[1] > '8') return false;
  const int from = (u[1] - '1') * 8 + (u[0] - 'a');
  Move buf[256];
  const int nm = b.pseudo_moves(buf);
  for (int i = 0; i < nm; ++i) {
    const Move& m = buf[i];
    if (m.from != from || !b.is_legal(m)) continue;
    if (b.uci(m, true) == u || (!b.chess960 && b.uci(m, false) == u)) { out = m; return true; }
  }
  return false;
}

bool Board::has_legal_move() const {
  Move buf[256];
  const int nm = pseudo_moves(buf);
  for (int i = 0; i < nm; ++i)
    if (is_legal(buf[i])) return true;
  return false;
}

uint64_t perft(const Board& b, int depth) {
  std::vector<Move> moves;
  b.legal_moves(moves);
  if (depth <= 1) return depth == 1 ? moves.size() : 1;
  uint64_t n = 0;
  for (const Move& m : moves) {
    Board c = b;
    c.do_move(m);
    n += perft(c, depth - 1);
  }
  return n;
}

}  // namespace fnnue
