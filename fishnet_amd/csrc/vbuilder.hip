// vbuilder.hip — device batch builder for Fairy-Stockfish variants
// (crazyhouse, atomic): the variant half of IncomingBatch::from_acquired
// ([ref] src/queue.rs:524-552 with body.variant != Standard, routed to the
// MultiVariant engine at :530-539; variants from src/assets.rs:384-391).
//
// As builder.hip for chess: one wave per game (replay_wave.h) parses the FEN
// (holdings, promoted marks) and replays the UCI moves (drops "P@e4",
// pockets, explosions) with the rules of vboard.h — the same source the host replay
// (fnnue_game_vpositions) runs, which the tests hold it to record for record —
// writing one fnnue_vpos per ply; CHILDREN adds one thread per ply for its
// legal children (drops included).
#include <hip/hip_runtime.h>

#include <vector>

#include "builder.h"
#include "replay_wave.h"
#include "vboard.h"

namespace fnnue {

namespace {

__global__ void vcount_plies_kernel(const char* __restrict__ text, const uint32_t* __restrict__ fen_off,
                                    const uint32_t* __restrict__ mv_off, uint32_t ngames,
                                    uint32_t* __restrict__ plies) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngames) return;
  uint32_t p = mv_off[g], st, n = 1;
  const uint32_t end = fen_off[g + 1];
  while (vb::next_token(text, p, end, st) > 0) ++n;
  plies[g] = n;
}

// Variant rules of the wave replay (replay_wave.h), vboard.h's.
struct VariantRules {
  using Board = vb::VBoard;
  using Move = vb::VMove;
  using Pos = fnnue_vpos;
  // the board's non-square state: pockets, castling rooks (VBoard::cr bytes),
  // en passant, side to move, variant | c960 << 8
  struct Scalars {
    uint64_t pocket[2];
    uint32_t cr;
    int32_t ep;
    uint32_t stm;
    uint32_t vc;
  };
  // Along the chain the pockets, cr and ep change; stm alternates and the
  // variant word is fixed (the checking lanes derive those two).
  static constexpr int kVary = 6;
  static constexpr bool kLaneChain = false;  // drops and explosions: the sequential chain (replay::chain)
  struct Win {};
  __device__ static Win window(const Scalars&, uint32_t, uint32_t, int) { return Win{}; }
  __device__ static void advance(Scalars&, const Win&, uint32_t) {}
  __device__ static void fix(Scalars& s, const Scalars& s0, const Win&, uint32_t j, bool after) {
    s.stm = s0.stm ^ ((j + (after ? 1u : 0u)) & 1u);
    s.vc = s0.vc;
  }
  __device__ static Scalars scalars(const vb::VBoard& b) {
    Scalars s;
    s.pocket[0] = b.pocket[0];
    s.pocket[1] = b.pocket[1];
    uint32_t cr;
    __builtin_memcpy(&cr, b.cr, 4);
    s.cr = cr;
    s.ep = b.ep;
    s.stm = b.stm;
    s.vc = (uint32_t)b.variant | ((uint32_t)b.c960 << 8);
    return s;
  }
  __device__ static int sc_cr(uint32_t cr, int c, int side) {
    return (int)(int8_t)((cr >> (8 * (2 * c + side))) & 0xFFu);
  }
  __device__ static void sc_cr_set(uint32_t& cr, int c, int side, int v) {
    const int sh = 8 * (2 * c + side);
    cr = (cr & ~(0xFFu << sh)) | (((uint32_t)v & 0xFFu) << sh);
  }
  __device__ static int sc_hand(const Scalars& s, int c, int t) {
    return (int)(((c ? s.pocket[1] : s.pocket[0]) >> (8 * (t - 1))) & 255u);
  }
  __device__ static void sc_hand_add(Scalars& s, int c, int t, int d) {
    const uint64_t delta = (uint64_t)(int64_t)d << (8 * (t - 1));
    if (c) s.pocket[1] += delta;
    else s.pocket[0] += delta;
  }
  __device__ static bool parse_fen(const char* t, uint32_t p, uint32_t e, int variant, vb::VBoard& b) {
    return vb::parse_fen(t, p, e, variant, b);
  }
  __device__ static const char* start_fen(int variant) {
    return variant == vb::kCrazyhouse ? "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1"
                                      : "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1";
  }
  __device__ static uint32_t start_fen_len(int variant) { return variant == vb::kCrazyhouse ? 58 : 56; }
  __device__ static vb::VBoard start_board(int variant) {
    vb::VBoard b;
    b.bc[0] = 0x000000000000FFFFull;
    b.bc[1] = 0xFFFF000000000000ull;
    b.bt[0] = 0;
    b.bt[vb::PAWN] = 0x00FF00000000FF00ull;
    b.bt[vb::KNIGHT] = 0x4200000000000042ull;
    b.bt[vb::BISHOP] = 0x2400000000000024ull;
    b.bt[vb::ROOK] = 0x8100000000000081ull;
    b.bt[vb::QUEEN] = 0x0800000000000008ull;
    b.bt[vb::KING] = 0x1000000000000010ull;
    b.promoted = 0;
    b.pocket[0] = b.pocket[1] = 0;
    b.cr[0][0] = 7;
    b.cr[0][1] = 0;
    b.cr[1][0] = 63;
    b.cr[1][1] = 56;
    b.ep = -1;
    b.stm = 0;
    b.variant = (uint8_t)variant;
    b.c960 = 0;
    return b;
  }
  // vb::match_uci's token rules: drops "P@e4" (piece letter either case, no
  // king), moves "e2e4" / "e7e8q" (promotion letter either case, N B R Q)
  __device__ static uint32_t encode(const char* c, int len) {
    if (len == 4 && c[1] == '@') {
      const int pt = vb::piece_type_of(c[0]), to = replay::tok_sq(c[2], c[3]);
      if (!pt || pt == vb::KING || to < 0) return replay::kTokBad;
      return ((uint32_t)to << 6) | ((uint32_t)pt << 12) | replay::kTokDrop;
    }
    const int from = replay::tok_sq(c[0], c[1]), to = replay::tok_sq(c[2], c[3]);
    if (from < 0 || to < 0) return replay::kTokBad;
    int promo = 0;
    if (len == 5) {
      promo = vb::piece_type_of(c[4]);
      if (!promo || promo == vb::PAWN || promo == vb::KING) return replay::kTokBad;
    }
    return (uint32_t)from | ((uint32_t)to << 6) | ((uint32_t)promo << 12);
  }
  __device__ static bool interpret(const Scalars& b, uint32_t code, vb::VMove& m, uint32_t sqv) {
    const int to = (int)replay::tok_to(code), pc = (int)replay::tok_piece(code);
    if (code & replay::kTokDrop) {
      m = vb::VMove{-1, (int8_t)to, (int8_t)pc, 2};
      return true;
    }
    const int from = (int)replay::tok_from(code);
    const uint32_t own = replay::lane_value(sqv, from) & 15u;
    if (!own || (int)(own >> 3) != (int)b.stm) return false;
    m = vb::VMove{(int8_t)from, (int8_t)to, (int8_t)pc, 0};
    if ((own & 7u) == (uint32_t)vb::KING && !pc) {
      const int back = b.stm == 0 ? 0 : 56;
      const bool c960 = (b.vc >> 8) & 1;
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int rsq = sc_cr(b.cr, b.stm, side);
        if (rsq >= 0 && (to == rsq || (!c960 && to == back + (side == 0 ? 6 : 2)))) {
          m = vb::VMove{(int8_t)from, (int8_t)rsq, 0, 1};
          return true;
        }
      }
    }
    return true;
  }
  // lane byte: piece code, bit 4 = promoted (crazyhouse)
  __device__ static uint32_t lane_square(const vb::VBoard& b, int sq) {
    return (uint32_t)vb::piece_at(b, sq) | ((uint32_t)((b.promoted >> sq) & 1) << 4);
  }
  // vb::do_move with lane l holding square l (see ChessRules::play): drops,
  // castling (the rook keeps its promoted mark), captures to the pocket (a
  // promoted piece as a pawn), atomic explosions as one select per lane.
  __device__ static void play(Scalars& b, const vb::VMove& m, uint32_t& sqv, int lane) {
    using vb::mkpc;
    constexpr int PAWN = vb::PAWN, ROOK = vb::ROOK, KING = vb::KING;
    const int us = b.stm;
    const int variant = (int)(b.vc & 255u);
    uint32_t v = sqv;
    int new_ep = -1;
    if (m.kind == 2) {
      v = lane == m.to ? (uint32_t)mkpc(us, m.piece) : v;
      sc_hand_add(b, us, m.piece, -1);
    } else if (m.kind == 1) {
      const int back = us == 0 ? 0 : 56;
      const bool king_side = m.to > m.from;
      const int kto = back + (king_side ? 6 : 2), rto = back + (king_side ? 5 : 3);
      const uint32_t rook_flag = replay::lane_value(v, m.to) & 16u;
      v = (lane == m.from || lane == m.to) ? 0u : v;
      v = lane == kto ? (uint32_t)mkpc(us, KING) : v;
      v = lane == rto ? ((uint32_t)mkpc(us, ROOK) | rook_flag) : v;
      sc_cr_set(b.cr, us, 0, -1);
      sc_cr_set(b.cr, us, 1, -1);
    } else {
      const uint32_t moved = replay::lane_value(v, m.from);
      const int pc = (int)(moved & 15u);
      int cap_sq = m.to;
      if ((pc & 7) == PAWN && m.to == b.ep && ((m.from ^ m.to) & 7) && !(replay::lane_value(v, m.to) & 15u))
        cap_sq = m.to + (us == 0 ? -8 : 8);
      const uint32_t capv = replay::lane_value(v, cap_sq);
      const int cap = (int)(capv & 15u);
      const bool zh = variant == vb::kCrazyhouse;
      if (cap && zh) {
        const int t = (capv & 16u) ? PAWN : (cap & 7);
        if (sc_hand(b, us, t) < 255) sc_hand_add(b, us, t, 1);
      }
      const uint32_t flag = (zh && (m.piece || (moved & 16u))) ? 16u : 0u;
      v = (lane == m.from || (cap && lane == cap_sq)) ? 0u : v;
      v = lane == m.to ? ((uint32_t)(m.piece ? mkpc(us, m.piece) : pc) | flag) : v;
      if (cap && variant == vb::kAtomic) {
        // the capturer explodes with its victim, and every non-pawn around
        const bool near = (vb::king_att(m.to) >> lane) & 1;
        v = (lane == m.to || (near && v != 0 && (v & 7u) != (uint32_t)PAWN)) ? 0u : v;
      }
      if ((pc & 7) == PAWN && (m.from ^ m.to) == 16) new_ep = (m.from + m.to) / 2;
      if ((pc & 7) == KING) {
        sc_cr_set(b.cr, us, 0, -1);
        sc_cr_set(b.cr, us, 1, -1);
      }
    }
    sqv = v;
    // castling rights end with the rook (moved, captured, exploded) or the king
    const uint64_t kings = __ballot((v & 7u) == (uint32_t)KING);
    const uint64_t black = __ballot((v & 15u) >= 8);
    for (int c = 0; c < 2; ++c) {
      if (!(kings & (c ? black : ~black))) {
        sc_cr_set(b.cr, c, 0, -1);
        sc_cr_set(b.cr, c, 1, -1);
      }
      for (int side = 0; side < 2; ++side) {
        const int r = sc_cr(b.cr, c, side);
        if (r >= 0 && (replay::lane_value(v, r) & 15u) != (uint32_t)mkpc(c, ROOK)) sc_cr_set(b.cr, c, side, -1);
      }
    }
    b.ep = new_ep;
    b.stm = (uint32_t)(us ^ 1);
  }
  // One chain step: interpret the code on the current board and play it;
  // false: it names no move of the side to move (the game's replay ends).
  __device__ __forceinline__ static bool step(Scalars& b, const Win&, uint32_t, uint32_t code, uint32_t& sqv, int lane,
                                              uint32_t& mv) {
    vb::VMove m;
    if (!interpret(b, code, m, sqv)) return false;
    play(b, m, sqv, lane);
    mv = pack_move(m);
    return true;
  }
  __device__ static uint32_t pack_move(const vb::VMove& m) {
    uint32_t w;
    __builtin_memcpy(&w, &m, 4);
    return w;
  }
  __device__ static vb::VMove unpack_move(uint32_t w) {
    vb::VMove m;
    __builtin_memcpy(&m, &w, 4);
    return m;
  }
  // A snapshot's bytes as bitboards (bit k of a code = plane k; bit 4 promoted).
  __device__ static vb::VBoard board_from(const uint32_t (&w)[16], const Scalars& sc) {
    const uint64_t p0 = replay::byte_plane(w, 0), p1 = replay::byte_plane(w, 1), p2 = replay::byte_plane(w, 2);
    const uint64_t p3 = replay::byte_plane(w, 3), p4 = replay::byte_plane(w, 4);
    const uint64_t occ = p0 | p1 | p2;
    vb::VBoard b;
    b.bc[0] = occ & ~p3;
    b.bc[1] = occ & p3;
    b.bt[0] = 0;
    b.bt[vb::PAWN] = p0 & ~p1 & ~p2;
    b.bt[vb::KNIGHT] = ~p0 & p1 & ~p2;
    b.bt[vb::BISHOP] = p0 & p1 & ~p2;
    b.bt[vb::ROOK] = ~p0 & ~p1 & p2;
    b.bt[vb::QUEEN] = p0 & ~p1 & p2;
    b.bt[vb::KING] = ~p0 & p1 & p2;
    b.promoted = p4;
    b.pocket[0] = sc.pocket[0];
    b.pocket[1] = sc.pocket[1];
    __builtin_memcpy(b.cr, &sc.cr, 4);
    b.ep = (int8_t)sc.ep;
    b.stm = (uint8_t)sc.stm;
    b.variant = (uint8_t)(sc.vc & 255u);
    b.c960 = (uint8_t)((sc.vc >> 8) & 255u);
    return b;
  }
  __device__ static fnnue_vpos pack_from(const uint32_t (&w)[16], const Scalars& sc) {
    uint32_t q[12];
    uint32_t nib[8];
    replay::pack_nibbles(w, nib);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = nib[i];
    // byte 32 stm, bytes 33..42 the pockets (white P N B R Q, black P N B R Q)
    const uint64_t wp = sc.pocket[0], bp = sc.pocket[1];
    q[8] = sc.stm | ((uint32_t)(wp & 0xFFFFFFu) << 8);
    q[9] = (uint32_t)((wp >> 24) & 0xFFFFu) | ((uint32_t)(bp & 0xFFFFu) << 16);
    q[10] = (uint32_t)((bp >> 16) & 0xFFFFFFu);
    q[11] = 0;
    fnnue_vpos p;
    memcpy(&p, q, sizeof(p));
    return p;
  }
  // As for chess (builder.hip ChessRules::verify): the token is accepted iff
  // the move interpret() built from it is legal.
  __device__ static bool verify(const vb::VBoard& b, const vb::VMove& m) {
    if (!vb::pseudo_member(b, m)) return false;
    vb::VBoard c = b;
    vb::do_move(c, m);
    return vb::legal_after(b, c);
  }
  __device__ static fnnue_vpos pack(const vb::VBoard& b) { return vb::pack(b); }
  __device__ static bool any_legal_from(const vb::VBoard& b, int sq, bool drops) {
    const bool own = (vb::colour(b, b.stm) >> sq) & 1;
    if (!own && !drops) return false;
    bool any = false;
    const vb::VBoard c = b;  // a copy for the by-reference generator: the chain's board stays in registers
    vb::for_each_legal(c, [&](const vb::VMove&) -> bool {
      any = true;
      return false;
    }, own ? 1ull << sq : 0ull, own, drops);
    return any;
  }
  __device__ static uint8_t end_flags(const vb::VBoard& b, bool any) {
    const int us = b.stm, k = vb::king_sq(b, us);
    const bool check = k >= 0 && vb::king_danger(b, k, us, vb::occupied(b));
    return (uint8_t)((any ? 0 : kFinalNoMoves) | (check ? kFinalCheck : 0) | (k < 0 ? kFinalExtinct : 0));
  }
};

__global__ void vcount_children_kernel(const vb::VBoard* __restrict__ states, uint32_t n, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const vb::VBoard b = states[i];
  uint32_t c = 0;
  vb::for_each_legal(b, [&](const vb::VMove&) -> bool {
    ++c;
    return true;
  });
  cnt[i] = 1u + c;
}

__global__ void vwrite_children_kernel(const vb::VBoard* __restrict__ states, uint32_t n,
                                       const uint32_t* __restrict__ off, fnnue_vpos* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const vb::VBoard b = states[i];
  uint32_t o = off[i];
  out[o++] = vb::pack(b);
  vb::for_each_legal(b, [&](const vb::VMove& m) -> bool {
    vb::VBoard c = b;
    vb::do_move(c, m);
    out[o++] = vb::pack(c);
    return true;
  });
}

}  // namespace

hipError_t replay_vgames_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                                const uint32_t* d_ply_off, uint32_t ngames, fnnue_vpos* d_out, void* d_states,
                                uint8_t* d_final, uint32_t* d_err, hipStream_t s) {
  return replay::launch_replay<VariantRules>(variant, d_text, d_fen_off, d_mv_off, ngames, d_ply_off, d_out,
                                             static_cast<vb::VBoard*>(d_states), d_err, d_final, s);
}

BuildResult build_vbatch_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                                uint32_t ngames, bool children, fnnue_vpos* d_out, size_t cap, uint32_t* d_group_off,
                                size_t off_cap, hipStream_t s, BuilderScratch& ws, uint8_t* d_final) {
  BuildResult R;
  auto fail = [&](hipError_t e) {
    R.hip = e;
    return R;
  };
  hipError_t e;
  uint32_t *plies = nullptr, *ply_off = nullptr, *err = nullptr, *cnt = nullptr, *coff = nullptr;
  vb::VBoard* states = nullptr;
  using W = BuilderScratch;
  if ((e = ws.get(W::kPlies, (size_t)(ngames + 1) * 4, (void**)&plies)) != hipSuccess) return fail(e);
  if ((e = ws.get(W::kPlyOff, (size_t)(ngames + 1) * 4, (void**)&ply_off)) != hipSuccess) return fail(e);
  if ((e = ws.get(W::kErr, 16, (void**)&err)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(err, 0, 16, s)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(plies + ngames, 0, 4, s)) != hipSuccess) return fail(e);
  const uint32_t bs = 64;
  hipLaunchKernelGGL(vcount_plies_kernel, dim3((ngames + bs - 1) / bs), dim3(bs), 0, s, d_text, d_fen_off, d_mv_off,
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
    if ((e = replay_vgames_device(variant, d_text, d_fen_off, d_mv_off, ply_off, ngames, d_out, nullptr, d_final, err,
                                  s)) != hipSuccess)
      return fail(e);
    if ((e = hipMemcpyAsync(d_group_off, ply_off, (size_t)(ngames + 1) * 4, hipMemcpyDeviceToDevice, s)) !=
        hipSuccess)
      return fail(e);
  } else {
    if ((e = ws.get(W::kStates, (size_t)total_plies * sizeof(vb::VBoard), (void**)&states)) != hipSuccess)
      return fail(e);
    if ((e = ws.get(W::kCnt, (size_t)(total_plies + 1) * 4, (void**)&cnt)) != hipSuccess) return fail(e);
    if ((e = ws.get(W::kCoff, (size_t)(total_plies + 1) * 4, (void**)&coff)) != hipSuccess) return fail(e);
    if ((e = replay_vgames_device(variant, d_text, d_fen_off, d_mv_off, ply_off, ngames, nullptr, states, d_final,
                                  err, s)) != hipSuccess)
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
    hipLaunchKernelGGL(vcount_children_kernel, dim3((total_plies + bs - 1) / bs), dim3(bs), 0, s, states,
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
    hipLaunchKernelGGL(vwrite_children_kernel, dim3((total_plies + bs - 1) / bs), dim3(bs), 0, s, states,
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

}  // namespace fnnue
