// builder.h — device-side batch builder (builder.hip): FEN parse, UCI replay
// and legal children on the GPU.  Same semantics as the host builder
// (board.h / board.cpp), which the tests hold it to record for record.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/fnnue.h"
#include "board.h"

namespace fnnue {

__host__ __device__ inline int make_piece_d(int c, int pt) { return (c << 3) | pt; }

// Board state a ply needs for move generation: bitboards, castling rooks,
// en-passant square, side to move.  The small fields are whole 32-bit words
// (the replay's board chain runs on the scalar unit, which has no 8- or
// 16-bit compares): castling rook of [colour c][side s] (0 king side, 1 queen
// side) in byte 2c + s of `cr`, 0xFF none (accessors in builder.hip).
struct DBoard {
  uint64_t bc[2];   // by colour
  uint64_t bt[7];   // by piece type (1..6), [0] unused
  uint32_t cr;
  int32_t ep;
  uint32_t stm;
  uint32_t c960;    // castling rights need Chess960 notation (non-standard rook/king files)
};

DBoard to_dboard(const Board& b);

// kBuildErrCount: a game's move tokens differ from the count its offsets were
// sized for (the host's count; never for offsets from the builder's own count).
constexpr uint32_t kBuildErrFen = 1, kBuildErrMove = 2, kBuildErrCount = 3;

// State of a game's last position (optional builder output, one byte per
// game): a game that ended on the board ends there, since no move can follow.
// The engine answers such a root with `bestmove (none)` and `score mate 0`
// (checkmated, or atomic: its king exploded) or `score cp 0` (stalemate)
// ([ref] src/stockfish.rs:359-376 parses them to Score::Mate(0) / Cp(0)).
constexpr uint8_t kFinalNoMoves = 1, kFinalCheck = 2, kFinalExtinct = 4;
// A game the replay rejected: kFinalFailed | its kBuildErr* code (replay_games_device).
constexpr uint8_t kFinalFailed = 0x80;

struct BuildResult {
  hipError_t hip = hipSuccess;
  bool capacity = false;   // outputs too small: n_out / n_groups say what is needed
  size_t n_out = 0, n_groups = 0;
  uint32_t err_code = 0, err_game = 0, err_ply = 0;  // kBuildErr*: first failing game, ply (1-based move)
};

// Grow-only device scratch of the batch builder (one per context, one per
// backend): per-game ply counts and offsets, the error word, the scan's
// temporary storage, per-ply boards and children counts.  A steady stream of
// batches allocates nothing; buffers are freed by release() only.
struct BuilderScratch {
  enum { kPlies, kPlyOff, kErr, kScan, kStates, kCnt, kCoff, kSlots };
  void* p[kSlots] = {};
  size_t bytes[kSlots] = {};
  // p[slot] with at least `want` bytes (grows by a quarter beyond the request)
  hipError_t get(int slot, size_t want, void** out);
  void release();
};

// text: game g's FEN in [fen_off[g], mv_off[g]), its space-separated UCI moves
// in [mv_off[g], fen_off[g + 1]).  children = false: every ply of every game,
// group g = game g; children = true: one group per ply = the ply's position
// followed by its legal children (Board::legal_moves order).  d_final
// (optional, ngames bytes): kFinal* flags of each game's last position.
// Sizes the outputs on the device and reads the sizes back: synchronises `s`.
BuildResult build_batch_device(const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                               uint32_t ngames, bool children, fnnue_pos* d_out, size_t cap, uint32_t* d_group_off,
                               size_t off_cap, hipStream_t s, BuilderScratch& ws, uint8_t* d_final = nullptr);

// Exclusive scan of cnt[0..n) into off[0..n], off[n] = total (hipcub, temporary
// storage from ws); stream-ordered, no host sync.
hipError_t builder_exclusive_scan(const uint32_t* cnt, uint32_t* off, uint32_t n, hipStream_t s, BuilderScratch& ws);

// The same expansion for Fairy-Stockfish variants (vbuilder.hip, vboard.h):
// crazyhouse / atomic FENs and UCI moves (drops "P@e4"), fnnue_vpos records.
BuildResult build_vbatch_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                                uint32_t ngames, bool children, fnnue_vpos* d_out, size_t cap, uint32_t* d_group_off,
                                size_t off_cap, hipStream_t s, BuilderScratch& ws, uint8_t* d_final = nullptr);

// Every ply of every game with offsets the caller already knows (ply_off:
// ngames + 1 entries, ply_off[g + 1] - ply_off[g] = 1 + the game's move
// tokens, as fnnue_backend_batch_size counts them): one launch, no sizing
// pass, no allocation, no host sync.  variant = kVariantChess (d_out:
// fnnue_pos) or a variant (fnnue_vpos).  d_err: 4 words, zero before the
// launch; afterwards err[0] = kBuildErr* of a failing game (0: none), err[1]
// that game, err[2] its ply.  d_final: optional kFinal* per game.
hipError_t replay_games_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                               const uint32_t* d_ply_off, uint32_t ngames, void* d_out, uint8_t* d_final,
                               uint32_t* d_err, hipStream_t s);
// vbuilder.hip's launcher of the same (variants only).
hipError_t replay_vgames_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                                const uint32_t* d_ply_off, uint32_t ngames, fnnue_vpos* d_out, void* d_states,
                                uint8_t* d_final, uint32_t* d_err, hipStream_t s);

// Leaf count of perft(depth) summed over the frontier boards (1 <= depth <= 3).
hipError_t perft_device(const std::vector<DBoard>& frontier, int depth, uint64_t* nodes);

}  // namespace fnnue
