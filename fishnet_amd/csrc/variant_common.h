// variant_common.h — Fairy-Stockfish "HalfKAv2 variants" feature set on the
// device (net.h; restated in oracle/variant_oracle.c, parity unpinned):
// lane-per-position decode of fnnue_vpos, king blocks, planes and the
// per-perspective feature lists, shared by the from-scratch plan
// (variant.hip) and the incremental segments (ft_segments.hip).
#pragma once
#include "sliced_common.h"

namespace fnnue {
namespace {

struct VariantBoard {
  LaneBoard b;        // board part (fnnue_vpos starts like fnnue_pos)
  uint32_t hand[10];  // white P N B R Q, black P N B R Q
  int nfeat;          // pieces on board + in hand (= list length + 1 per perspective)
  bool ok;
  bool over;          // atomic game over: one king exploded (no NNUE eval, not an error)
};

template <bool kOcc = true>
__device__ __forceinline__ VariantBoard vdecode(const fnnue_vpos* p, bool pockets) {
  VariantBoard v;
  v.b = lane_decode<kOcc>(reinterpret_cast<const fnnue_pos*>(p));
  const uint8_t* h = reinterpret_cast<const uint8_t*>(p) + 33;
  int tot = 0;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    v.hand[i] = h[i];
    tot += h[i];
    bad |= h[i] > (uint32_t)kVHandSlots || (!pockets && h[i] != 0);
  }
  v.b.stm = reinterpret_cast<const uint8_t*>(p)[32];
  v.nfeat = v.b.cnt + tot;
  v.ok = v.b.ok && v.b.stm <= 1 && !bad && v.nfeat <= 32;
  // Atomic: a capture next to a king explodes it and ends the game; the
  // position after it (exactly one king left) is a terminal record the
  // evaluator answers with (0, 0) without latching an error.  Only variants
  // without pockets here (crazyhouse kings are never removed).
  v.over = !pockets && v.b.sane && !bad && v.nfeat <= 32 && v.b.nwk + v.b.nbk == 1;
  return v;
}

__device__ __forceinline__ int vblock(int persp, int ksq) { return persp ? ksq ^ 56 : ksq; }

__device__ __forceinline__ int vplane(int persp, int pc) {
  const int type = pc & 7;
  return type == 6 ? 10 : 2 * (type - 1) + ((pc >> 3) != persp);
}

// Perspective `persp`'s list: every feature but the own king, as 16 * row
// (row relative to the king block), padded with the zero row R; rows of parity
// pp first (the bank pairing of ft_slices, see write_rows).  The entries are
// gathered in the thread's own LDS row (`mine`, 68-B stride: a wave's rows
// start in 32 different banks) because their count per source is data
// dependent — a register array indexed by a divergent k costs a waterfall loop
// per entry — then read back as 16 words with static indices.
constexpr int kVListStrideWords = 17;

// Row (within the perspective's king block) of a board piece pc on square s.
__device__ __forceinline__ uint32_t vboard_row(int persp, int s, int pc) {
  return (uint32_t)(vblock(persp, s) + 64 * vplane(persp, pc));
}
// Row of the k-th piece (k = 0, 1, ...) of hand slot i (owner i >= 5, type i % 5).
__device__ __forceinline__ uint32_t vhand_row(int persp, int i, uint32_t k) {
  return kVBoardRows + kVHandSlots * (2 * (i % 5) + ((i >= 5) != persp)) + k;
}

template <int R>
__device__ __forceinline__ void vwrite_rows(const VariantBoard& v, int persp, uint32_t it, uint32_t pp,
                                            uint32_t* __restrict__ mine, uint16_t* __restrict__ flist) {
  const int ksq = persp ? v.b.bk : v.b.wk;
  const uint64_t occ = v.b.occ & ~(1ull << ksq);
  constexpr uint64_t kEvenFiles = 0x5555555555555555ull;
  uint16_t* L = reinterpret_cast<uint16_t*>(mine);
  int k = 0;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const uint32_t want = pass == 0 ? pp : pp ^ 1u;  // row parity = file parity (rank flip keeps files)
    for (uint64_t m = occ & (want ? ~kEvenFiles : kEvenFiles); m; m &= m - 1) {
      const int s = __builtin_ctzll(m);
      L[k++] = (uint16_t)(16u * (uint32_t)(vblock(persp, s) + 64 * vplane(persp, nibble_at(v.b.w, s))));
    }
    if (R > kVBoardRows) {
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int owner = i >= 5, pt = i % 5;
        const uint32_t base = kVBoardRows + kVHandSlots * (2 * pt + (owner != persp));
        for (uint32_t c = want; c < v.hand[i]; c += 2) L[k++] = (uint16_t)(16u * (base + c));  // row parity = c & 1
      }
    }
  }
  for (; k < 32; ++k) L[k] = (uint16_t)(16u * R);
  uint32_t E[16];
#pragma unroll
  for (int j = 0; j < 16; ++j)  // this thread's own LDS writes (same type: no aliasing reorder), in order
    E[j] = (uint32_t)L[2 * j] | (uint32_t)L[2 * j + 1] << 16;
  uint4* dst = reinterpret_cast<uint4*>(flist + (size_t)it * 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[q] = make_uint4(E[4 * q], E[4 * q + 1], E[4 * q + 2], E[4 * q + 3]);
}

}  // namespace
}  // namespace fnnue
