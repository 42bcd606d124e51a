// board.h — host-side batch builder: FEN / UCI (standard + Chess960) / legal
// move generation / random playouts, producing packed fnnue_pos records.
//
// Replaces the role shakmaty 0.23.0 plays in the reference's batch expansion
// (src/queue.rs:524-606: VariantPosition::from_setup, Uci::to_move,
// play_unchecked) and Stockfish's Position::set / do_move (upstream
// src/position.cpp) as far as the NNUE path needs them.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fnnue.h"

namespace fnnue {

enum Color : int { WHITE = 0, BLACK = 1 };
// Stockfish Piece codes (upstream src/types.h): W_PAWN=1..W_KING=6, B_PAWN=9..B_KING=14.
enum PieceType : int { PAWN = 1, KNIGHT, BISHOP, ROOK, QUEEN, KING };
inline int make_piece(int c, int pt) { return (c << 3) | pt; }
inline int type_of(int pc) { return pc & 7; }
inline int color_of(int pc) { return pc >> 3; }

struct Move {
  uint8_t from, to;     // castling: to = rook square (king-takes-rook, internal)
  uint8_t promo;        // piece type or 0
  uint8_t castle;       // 1 if castling
};

struct Board {
  uint8_t sq[64];       // piece code per square, 0 = empty
  uint64_t byColor[2];
  uint64_t byType[7];   // index by piece type, [0] = all
  int stm = WHITE;
  int ep = -1;          // en-passant target square or -1
  int castle_rook[2][2];// [color][0=king side,1=queen side] rook square or -1
  int halfmove = 0, fullmove = 1;
  bool chess960 = false;

  void clear();
  void put(int s, int pc);
  void remove(int s);
  int king_sq(int c) const;
  uint64_t occupied() const { return byColor[0] | byColor[1]; }
  bool attacked(int s, int by, uint64_t occ) const;
  bool in_check() const { return attacked(king_sq(stm), stm ^ 1, occupied()); }
  // Pseudo-legal moves (castling already fully checked); returns the count.
  int pseudo_moves(Move* buf) const;
  bool is_legal(const Move& m) const;
  // All legal moves.
  void legal_moves(std::vector<Move>& out) const;
  bool has_legal_move() const;  // legal_moves non-empty, stopping at the first
  // Uniformly random legal move by rejection sampling over the pseudo-legal
  // list; false if there is none.  rng is a splitmix64 state.
  bool random_legal_move(uint64_t& rng, Move& out) const;
  void do_move(const Move& m);
  std::string fen() const;
  std::string uci(const Move& m, bool chess960_castling) const;
  fnnue_pos pack() const;
};

// Parses a FEN (X-FEN/Shredder castling accepted). Returns false on malformed input.
bool board_from_fen(const char* fen, Board& b, std::string* err);
// Finds the legal move matching a UCI string (standard "e1g1" or Chess960
// king-takes-rook castling). Returns false if not legal.
bool parse_uci(const Board& b, const char* uci, Move& out);

uint64_t perft(const Board& b, int depth);

// splitmix64 (also used by the synthetic net generator and the bench).
inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace fnnue
