// ft_segments.hip — incremental feature transformer on LDS tiles, for grouped
// positions (CHAIN: a game's plies in order; STAR: a parent and its
// children), BASELINE configs 3 and 4.
//
// Upstream Stockfish updates an accumulator incrementally along the
// StateInfo chain (nnue_feature_transformer.h update_accumulator: subtract the
// removed feature rows, add the added ones) and refreshes it when the
// perspective's own king moved (HalfKAv2_hm::requires_refresh).  While a
// perspective's own king stays put its features all live in one king block,
// i.e. in one LDS tile of the sliced layout (ft_sliced.hip).  So a *segment*
// = a refresh position and the positions derived from it without another
// refresh (CHAIN: the following plies; STAR: the parent's children) is
// processed by the 8 lanes of one item inside the (king block, slice)
// workgroup that holds the tile: the refresh position sums its full feature
// list, every further position applies <= 2 removed and <= 2 added rows to
// the previous accumulator (CHAIN) or to the parent's (STAR).  int16 add/sub
// wrap is a group, so results equal a refresh bit for bit.
//
// Plan (all on the device):
//   group_span    once per call: per position its group's {first, end}
//                 (wave per group); checks the device-only offsets
// then per chunk of <= 2^20 positions (cut at fixed positions, not at group
// boundaries, so no offset ever comes to the host; a group cut by a chunk
// boundary restarts with a refresh there, group_range):
//   seg_delta     per (position, perspective): refresh flag or the delta
//                 record {slot, half, bucket, 2 removed, 2 added rows};
//                 zeroes the counters
//   scan          exclusive scan of refresh flags -> item index per refresh:
//                 block counts in seg_delta, seg_scan_blocks, then local
//                 scans in seg_items_scan, which also maps item k -> its
//                 root position
//   seg_place     segment length per refresh (next refresh / group parent)
//                 and the item histogram; delta records placed at root +
//                 rank (a segment's plies contiguous)
//   plan_scan / seg_scatter   counting sort of items by
//                 (king block, length bin), unit table cut every
//                 kSegUnitPlies (16384) positions of work per king block,
//                 full lists (write_rows)
//   ft_segments   (unit, slice) workgroups, XCD-aware, tile in LDS
// then stack_kernel over x / bucket / psqt_part in position order.
//
// The same machinery runs the Fairy-Stockfish variant feature sets (64 king
// blocks, crazyhouse pocket rows): a feature set Fs supplies the position
// record, its decode, king blocks, feature rows and the tile geometry.  A
// variant ply's delta also carries its pocket changes as row adds / removes
// (a capture adds the captured piece's next hand row, a drop removes the
// dropped piece's last one); atomic explosions exceed two removed rows and
// refresh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "variant_common.h"

namespace fnnue {

namespace {

constexpr uint32_t kSlotMask = 0xFFFFFF;  // item record x: slot | half << 24 | bucket << 25
constexpr uint32_t kRowMask = 0x1FFFFFF;  // delta record x: (2 * slot + half) | bucket << 25
// A segment item is a whole run of positions walked serially, so units are
// cut by positions (kSegUnitPlies, plan_scan_kernel_t) rather than by items.

// Feature sets.  Dec: the lane decode (board b, list length + 1 = nfeat, ok).
// kNone: 16 * the tile's first zero row (unused delta slots, sentinel).
struct ChessFs {
  using Pos = fnnue_pos;
  using G = ChessGeom;
  static constexpr int KB = 32;
  static constexpr int kClasses = 4;  // list-length classes per length bin (seg_count_class)
  static constexpr bool kHand = false;
  static constexpr uint32_t kNone = 16u * G::kRows;
  struct Dec {
    LaneBoard b;
    uint32_t hand[10];
    int nfeat;
    bool ok;
    bool over;  // never for chess (variant_common.h: atomic game over)
  };
  template <bool kOcc = true>
  __device__ static __forceinline__ Dec decode(const Pos* p) {
    Dec d;
    d.b = lane_decode<kOcc>(p);
    d.nfeat = d.b.cnt;
    d.ok = d.b.ok;
    d.over = false;
    return d;
  }
  // The base of a delta: its board words, with validity and king squares
  // from an earlier decode (seg_info).
  __device__ static __forceinline__ Dec load_base(const Pos* p, uint32_t info) {
    Dec d;
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int k = 0; k < 8; ++k) d.b.w[k] = pw[k];
    d.ok = (info & 1u) != 0;
    d.b.wk = (int)((info >> 1) & 63u);
    d.b.bk = (int)((info >> 7) & 63u);
    return d;
  }
  __device__ static __forceinline__ int block(int c, int ksq) { return king_block(c, ksq); }
  // 16 * (make_index(c, s, pc, ksq) - 704 * kb): the oriented square plus
  // 64 * the plane (nibble table), the king block cancels
  __device__ static __forceinline__ uint32_t board_entry(int c, int s, int pc, int ksq, int) {
    const uint32_t flip = (c ? 56u : 0u) ^ ((ksq & 7) < 4 ? 7u : 0u);
    const uint64_t ptab = c ? plane_table(1) : plane_table(0);
    return 16u * (((uint32_t)s ^ flip) + 64u * (uint32_t)((ptab >> (4 * pc)) & 15u));
  }
  __device__ static __forceinline__ void write_list(const Dec& d, int c, uint32_t it, uint32_t pp, uint32_t* mine,
                                                    uint16_t* flist) {
    write_rows(d.b, c, c ? d.b.bk : d.b.wk, it, pp, mine, flist);
  }
};

template <int V>  // kVariantCrazyhouse / kVariantAtomic
struct VariantFs {
  using Pos = fnnue_vpos;
  static constexpr int R = (int)variant_rows(V);
  using G = VariantGeom<R>;
  static constexpr int KB = 64;
  static constexpr bool kHand = V == kVariantCrazyhouse;
  static constexpr int kClasses = kHand ? 1 : 4;
  static constexpr uint32_t kNone = 16u * R;
  using Dec = VariantBoard;
  template <bool kOcc = true>
  __device__ static __forceinline__ Dec decode(const Pos* p) { return vdecode<kOcc>(p, kHand); }
  __device__ static __forceinline__ Dec load_base(const Pos* p, uint32_t info) {
    Dec d;
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int k = 0; k < 8; ++k) d.b.w[k] = pw[k];
    const uint8_t* h = reinterpret_cast<const uint8_t*>(p) + 33;
#pragma unroll
    for (int j = 0; j < 10; ++j) d.hand[j] = h[j];
    d.ok = (info & 1u) != 0;
    d.b.wk = (int)((info >> 1) & 63u);
    d.b.bk = (int)((info >> 7) & 63u);
    return d;
  }
  __device__ static __forceinline__ int block(int c, int ksq) { return vblock(c, ksq); }
  __device__ static __forceinline__ uint32_t board_entry(int c, int s, int pc, int, int) {
    return 16u * vboard_row(c, s, pc);
  }
  __device__ static __forceinline__ void write_list(const Dec& d, int c, uint32_t it, uint32_t pp, uint32_t* mine,
                                                    uint16_t* flist) {
    vwrite_rows<R>(d, c, it, pp, mine, flist);
  }
};

// Counter layout of a feature set's plan (plan_scan_kernel_t<KB>).
template <class Fs>
struct SegCtr {
  static constexpr int kNB = 33 * Fs::kClasses;  // bins per king block
  static constexpr int kIB = Fs::KB * kNB, kB = kIB + kPosBins, kOff = kB, kCur = 2 * kB, kNUnits = 3 * kB;
  static constexpr size_t kWords = 3 * kB + 16;
};

// Each position's group span {first, end}, absolute positions of the whole
// call, written once per call by group_span_kernel (one wave per group fills
// its members, coalesced) so the plan kernels of every chunk read one word
// pair instead of binary-searching the offsets.  With check set it also checks
// the offsets (non-decreasing, off[0] = 0, off[ngroups] = npos; else error bit
// 2, FNNUE_E_ARG): the offsets of a *_device call never come to the host.
// span == nullptr: check only (the gather path).
// A group longer than kSpanChunk (one long CHAIN, or a whole batch sent as one
// group) is not filled by its one wave, which would walk it serially (ADVICE
// r03): the wave fills it up to the next kSpanChunk-aligned position and
// writes the span at every aligned position inside it; group_span_big_kernel
// (one workgroup per aligned chunk of positions) then fills the rest of each
// chunk whose first entry names such a group.  Every aligned position's entry
// is written by the first kernel (by its small group, or as a big group's
// marker), so the second kernel never reads a stale entry.
constexpr uint32_t kSpanChunk = 4096;
// group g's span entries, by one wave (lane)
__device__ __forceinline__ void group_span_one(const uint32_t* __restrict__ off, uint32_t ngroups, uint32_t npos,
                                               uint2* __restrict__ span, int check, uint32_t* __restrict__ err,
                                               uint32_t g, uint32_t lane) {
  if (check && lane == 0) {
    bool bad = off[g + 1] < off[g];
    if (g == 0) bad |= off[0] != 0 || off[ngroups] != npos;
    if (bad) atomicOr(err, 2u);
  }
  if (!span) return;
  const uint32_t a = min(off[g], npos), b = min(max(off[g + 1], a), npos);
  const uint2 v = make_uint2(a, b);
  if (b - a <= kSpanChunk) {
    for (uint32_t i = a + lane; i < b; i += 64) span[i] = v;
    return;
  }
  const uint32_t a1 = (a + kSpanChunk - 1) / kSpanChunk * kSpanChunk;  // < b: the group is longer than a chunk
  for (uint32_t i = a + lane; i < a1; i += 64) span[i] = v;
  for (uint32_t i = a1 + lane * kSpanChunk; i < b; i += 64 * kSpanChunk) span[i] = v;
}

__global__ __launch_bounds__(256) void group_span_kernel(const uint32_t* __restrict__ off, uint32_t ngroups,
                                                         uint32_t npos, uint2* __restrict__ span, int check,
                                                         uint32_t* __restrict__ err) {
  const uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= ngroups) return;
  group_span_one(off, ngroups, npos, span, check, err, g, threadIdx.x & 63);
}

__global__ __launch_bounds__(256) void group_span_big_kernel(uint32_t npos, uint2* __restrict__ span) {
  const uint32_t c0 = blockIdx.x * kSpanChunk;
  const uint2 v = span[c0];
  if (v.y - v.x <= kSpanChunk) return;  // a small group's entry: the chunk is filled
  const uint32_t e = min(c0 + kSpanChunk, min(v.y, npos));
  for (uint32_t i = c0 + 1 + threadIdx.x; i < e; i += 256) span[i] = v;
}

// The group of chunk position i (absolute position sbase + i), in chunk
// coordinates and clamped to first <= i < end <= n.  A group that starts
// before the chunk starts at the chunk's first position there (its first
// in-chunk position is refreshed: a CHAIN continues from it, a STAR's
// remaining children derive from it); one that ends after the chunk ends at
// the chunk's end.  With malformed offsets (gaps leave span entries
// unwritten) every access stays inside the chunk.  Grouping never affects
// results: deltas are diffs of the two boards, a refresh otherwise.
__device__ __forceinline__ uint2 group_range(const uint2* __restrict__ span, uint32_t i, uint32_t n, uint32_t sbase) {
  const uint2 v = span[i];
  const uint32_t a = v.x > sbase ? v.x - sbase : 0u, b = v.y > sbase ? v.y - sbase : 0u;
  return make_uint2(min(a, i), min(max(b, i + 1), n));
}

// Validity and king squares of a decoded position, for the next position's
// delta (seg_delta_kernel shares them through LDS).
template <class Dec>
__device__ __forceinline__ uint32_t seg_info(const Dec& d) {
  return (d.ok ? 1u : 0u) | (uint32_t)d.b.wk << 1 | (uint32_t)d.b.bk << 7;
}

// Refresh flags r0 / r1 and delta records of position i (both perspectives),
// B = its decode.  The base's validity and king squares come from `info`
// (the block's positions i0 .. i0 + 255) when it lies in this block: the
// base of a CHAIN ply is the previous position, so only a wave's first lane
// decodes a second board (a wave with any such lane pays the whole decode).
template <class Fs>
__device__ __forceinline__ void seg_delta_one(const typename Fs::Pos* __restrict__ pos, uint32_t n,
                                              const uint2* __restrict__ span, uint32_t sbase, int star,
                                              uint32_t* __restrict__ ref,
                                              uint4* __restrict__ dtmp, uint8_t* __restrict__ bucket,
                                              uint32_t* __restrict__ err, uint32_t i, uint32_t i0,
                                              const uint32_t* info, const typename Fs::Dec& B, uint32_t& r0,
                                              uint32_t& r1) {
  using Dec = typename Fs::Dec;
  if (!B.ok) {
    // no item, no accumulator; counted as a refresh so that STAR ranks skip it
    bucket[i] = 0xFF;
    ref[i] = ref[n + i] = 1;
    r0 = r1 = 1;
    if (!B.over) atomicOr(err, 1u);  // an exploded king (atomic) is a result (0, 0), not an error
    return;
  }
  const uint32_t bk = (uint32_t)(B.b.cnt - 1) >> 2;  // board pieces
  bucket[i] = (uint8_t)bk;
  const uint32_t first = group_range(span, i, n, sbase).x;
  const bool has_base = i > first;
  Dec A;
  bool base_ok = false;
  const uint32_t bi = star ? first : i - 1;  // the base, when has_base
  if (has_base) {
    const uint32_t ai = bi >= i0 ? info[bi - i0] : seg_info(Fs::template decode<false>(pos + bi));
    A = Fs::load_base(pos + bi, ai);
    base_ok = A.ok;
  }
  // Changed squares as a 64-bit mask, then at most four of them, one uniform
  // step each (a loop per board word ran a step for every word in which any
  // lane of the wave had a change: eight steps for a wave's moves).  The
  // nibbles are read back as bytes of the two records, both just loaded (a
  // register array indexed by a lane-varying square would live in scratch).
  uint64_t ch = 0;
  if (has_base) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      ch |= (uint64_t)nibble_bits(~zero_nibbles(A.b.w[k] ^ B.b.w[k]) & 0x88888888u) << (8 * k);
  }
  const int nch = __popcll(ch);
  // Removed / added entries of both perspectives in named slots (a register
  // array indexed by the running count would live in scratch as well); the
  // counts are the same for both perspectives.
  const int ks0 = B.b.wk, ks1 = B.b.bk;
  const int kb0 = Fs::block(0, ks0), kb1 = Fs::block(1, ks1);
  uint32_t r00 = Fs::kNone, r01 = Fs::kNone, r10 = Fs::kNone, r11 = Fs::kNone;
  uint32_t a00 = Fs::kNone, a01 = Fs::kNone, a10 = Fs::kNone, a11 = Fs::kNone;
  auto put = [](uint32_t& x0, uint32_t& x1, int cnt, uint32_t e) {
    x0 = cnt == 0 ? e : x0;
    x1 = cnt == 1 ? e : x1;
  };
  int nr = 0, na = 0;
  if (base_ok && nch <= 4) {
    const uint8_t* pa = reinterpret_cast<const uint8_t*>(pos + bi);
    const uint8_t* pb = reinterpret_cast<const uint8_t*>(pos + i);
    for (uint64_t m = ch; m; m &= m - 1) {
      const int s = __builtin_ctzll(m), sh = 4 * (s & 1);
      const int was = (pa[s >> 1] >> sh) & 15, now = (pb[s >> 1] >> sh) & 15;
      if (was) {
        put(r00, r01, nr, Fs::board_entry(0, s, was, ks0, kb0));
        put(r10, r11, nr, Fs::board_entry(1, s, was, ks1, kb1));
        ++nr;
      }
      if (now) {
        put(a00, a01, na, Fs::board_entry(0, s, now, ks0, kb0));
        put(a10, a11, na, Fs::board_entry(1, s, now, ks1, kb1));
        ++na;
      }
    }
    if constexpr (Fs::kHand) {
      // pocket slot j holding `was` pieces before and `now` after: the rows
      // of its pieces was .. now - 1 are added, now .. was - 1 removed
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const uint32_t was = A.hand[j], now = B.hand[j];
        for (uint32_t k = now; k < was && nr <= 2; ++k) {
          put(r00, r01, nr, 16u * vhand_row(0, j, k));
          put(r10, r11, nr, 16u * vhand_row(1, j, k));
          ++nr;
        }
        for (uint32_t k = was; k < now && na <= 2; ++k) {
          put(a00, a01, na, 16u * vhand_row(0, j, k));
          put(a10, a11, na, 16u * vhand_row(1, j, k));
          ++na;
        }
      }
    }
  }
  // refresh: own king moved, invalid base, > 4 changed squares, or more than
  // two removed / added rows (never for a legal chess move; explosions and
  // arbitrary groups refresh)
  const bool common = !base_ok || nch > 4 || nr > 2 || na > 2;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const bool refresh = common || (c ? A.b.bk != ks1 : A.b.wk != ks0);
    // a refresh carries its king block and count class for the item
    // histogram (seg_place)
    ref[c * n + i] = refresh ? 1u | (uint32_t)(c ? kb1 : kb0) << 8 | seg_count_class<Fs::kClasses>((uint32_t)B.nfeat) << 16 : 0u;
    (c ? r1 : r0) = refresh ? 1u : 0u;
    if (!refresh) {
      const uint32_t half = B.b.stm == c ? 0u : 1u;
      const uint32_t rm = c ? r10 | r11 << 16 : r00 | r01 << 16, ad = c ? a10 | a11 << 16 : a00 | a01 << 16;
      dtmp[c * n + i] = make_uint4((2u * i + half) | bk << 25, rm, ad, 0u);
    }
  }
}

// The first kernel of a chunk's plan: block 0 also zeroes the counter block
// (read by seg_place / plan_scan / seg_scatter) instead of a memset launch.
template <class Fs>
__global__ __launch_bounds__(256) void seg_delta_kernel(const typename Fs::Pos* __restrict__ pos, uint32_t n,
                                                        const uint2* __restrict__ span, uint32_t sbase, int star,
                                                        uint32_t* __restrict__ ref,
                                                        uint4* __restrict__ dtmp, uint8_t* __restrict__ bucket,
                                                        uint32_t* __restrict__ err, uint32_t* __restrict__ bsum,
                                                        uint32_t* __restrict__ ctr, uint32_t ctr_words) {
  __shared__ uint32_t info[256];
  if (blockIdx.x == 0)
    for (uint32_t k = threadIdx.x; k < ctr_words; k += blockDim.x) ctr[k] = 0;
  const uint32_t i0 = blockIdx.x * 256, i = i0 + threadIdx.x;
  typename Fs::Dec B;
  B.ok = B.over = false;
  B.b.wk = B.b.bk = 0;
  if (i < n) B = Fs::template decode<false>(pos + i);
  info[threadIdx.x] = seg_info(B);
  __syncthreads();
  uint32_t r0 = 0, r1 = 0;
  if (i < n) seg_delta_one<Fs>(pos, n, span, sbase, star, ref, dtmp, bucket, err, i, i0, info, B, r0, r1);
  // refresh counts of this block's 256 positions, per perspective (seg_scan_blocks)
  const int c0 = __syncthreads_count((int)r0), c1 = __syncthreads_count((int)r1);
  if (threadIdx.x == 0) {
    bsum[blockIdx.x] = (uint32_t)c0;
    bsum[gridDim.x + blockIdx.x] = (uint32_t)c1;
  }
}

// Exclusive scan of the per-block refresh counts (2 * nb of them, perspective
// 0's blocks first, as ref is laid out) into block offsets, and cref[2n] =
// the item count.  One workgroup; nb <= kMaxScanBlocks.
constexpr uint32_t kMaxScanBlocks = 8192;
__global__ __launch_bounds__(1024) void seg_scan_blocks_kernel(uint32_t* __restrict__ bsum, uint32_t nb, uint32_t n,
                                                               uint32_t* __restrict__ cref) {
  __shared__ uint32_t part[16];
  const uint32_t m = 2 * nb, per = (m + 1023) / 1024, t = threadIdx.x;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; ++k) sum += t * per + k < m ? bsum[t * per + k] : 0u;
  // per-thread sums scanned inside each wave by shuffles, then over the 16
  // wave totals
  const uint32_t lane = t & 63, wv = t >> 6;
  uint32_t incl = sum;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) part[wv] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
  for (uint32_t w = 0; w < wv; ++w) run += part[w];
  for (uint32_t k = 0; k < per; ++k)
    if (t * per + k < m) {
      const uint32_t v = bsum[t * per + k];
      bsum[t * per + k] = run;
      run += v;
    }
  if (t == 1023) cref[2 * n] = run;  // the total
}

// cref[j] (exclusive scan of ref) from the block offsets and a block-local
// scan; item k = cref[j] of each refresh j gets its position (ipos).
// Grid (nb, 2): block (b, c) covers positions 256 b .. +255 of perspective c.
__global__ __launch_bounds__(256) void seg_items_scan_kernel(uint32_t n, const uint32_t* __restrict__ ref,
                                                             const uint32_t* __restrict__ boff,
                                                             uint32_t* __restrict__ cref, uint32_t* __restrict__ ipos) {
  __shared__ uint32_t wsum[4];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y, j = c * n + i;
  const uint32_t r = i < n ? ref[j] : 0u;
  const uint64_t bal = __ballot(r != 0);
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t below = (uint32_t)__popcll(bal & ((1ull << lane) - 1));
  if (lane == 0) wsum[wv] = (uint32_t)__popcll(bal);
  __syncthreads();
  uint32_t base = boff[c * gridDim.x + blockIdx.x];
  for (uint32_t w = 0; w < wv; ++w) base += wsum[w];
  if (i >= n) return;
  const uint32_t k = base + below;
  cref[j] = k;
  if (r) ipos[k] = i;
}


// One thread per (perspective, position) j (grid stride), after the scan and
// seg_items:
// * a valid refresh gets its segment length (0 at every other j) and counts
//   in the item histogram by (king block, length bin) — the king block rides
//   in its refresh flag (seg_delta), so no position is decoded here.  CHAIN:
//   up to the next refresh of the same perspective (the next item; groups
//   start with one).  STAR: the group's parent owns its children that are not
//   refreshes.
// * any other position places its delta record at root + rank, so that a
//   segment's records are contiguous.
// At most one workgroup per CU: the histogram merge costs one global atomic
// per non-empty bin per workgroup.
// (The body runs as workgroup `bid` of `nb`, on an LDS histogram h of
// SegCtr<Fs>::kIB words: seg_place_kernel, or a phase of seg_plan_small_kernel.)
template <class Fs>
__device__ __forceinline__ void seg_place_body(uint32_t n, const uint2* __restrict__ span, uint32_t sbase, int star,
                                               const uint8_t* __restrict__ bucket, const uint32_t* __restrict__ ref,
                                               const uint32_t* __restrict__ cref, const uint32_t* __restrict__ ipos,
                                               uint32_t* __restrict__ len, const uint4* __restrict__ dtmp,
                                               uint4* __restrict__ drec, uint32_t* __restrict__ ctr,
                                               uint32_t* __restrict__ h, uint32_t bid, uint32_t nb) {
  constexpr int kIB = SegCtr<Fs>::kIB;
  for (int t = threadIdx.x; t < kIB; t += blockDim.x) h[t] = 0;
  __syncthreads();
  // Record 2n, read by items past the end of their segment: no rows, x row 2n
  // and bucket 0, i.e. x and PSQT stores just past the launch's buffer ranges
  // (dropped by the hardware), so the walk needs no liveness masking.
  if (bid == 0 && threadIdx.x == 0)
    drec[2 * n] = make_uint4(2 * n, Fs::kNone | Fs::kNone << 16, Fs::kNone | Fs::kNone << 16, 0u);
  for (uint32_t j = bid * blockDim.x + threadIdx.x; j < 2 * n; j += nb * blockDim.x) {
    const uint32_t c = j >= n ? 1u : 0u, i = j - c * n;
    const uint32_t rf = ref[j];
    if (rf) {
      uint32_t L = 0;
      if (bucket[i] != 0xFF) {
        if (star) {
          const uint2 g = group_range(span, i, n, sbase);
          L = i != g.x ? 1u : (g.y - i) - (cref[c * n + g.y] - cref[j + 1]);
        } else {
          const uint32_t k = cref[j];
          L = (k + 1 < cref[(c + 1) * n] ? ipos[k + 1] : n) - i;
        }
      }
      len[j] = L;
      if (L) atomicAdd(&h[((rf >> 8) & 0xFFu) * SegCtr<Fs>::kNB + seg_len_bin(L) * Fs::kClasses + (rf >> 16)], 1u);
      continue;
    }
    len[j] = 0;
    uint32_t r, rank;
    if (star) {
      r = group_range(span, i, n, sbase).x;  // the parent: a refresh item of this perspective
      rank = (i - r) - (cref[j] - cref[c * n + r + 1]);
    } else {
      r = ipos[cref[j] - 1];  // the last refresh of this perspective before i (same game)
      rank = i - r;
    }
    drec[c * n + r + rank] = dtmp[j];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kIB; t += blockDim.x)
    if (h[t]) atomicAdd(&ctr[t], h[t]);
}

template <class Fs>
__global__ __launch_bounds__(1024) void seg_place_kernel(uint32_t n, const uint2* __restrict__ span, uint32_t sbase,
                                                         int star,
                                                         const uint8_t* __restrict__ bucket,
                                                         const uint32_t* __restrict__ ref,
                                                         const uint32_t* __restrict__ cref,
                                                         const uint32_t* __restrict__ ipos, uint32_t* __restrict__ len,
                                                         const uint4* __restrict__ dtmp, uint4* __restrict__ drec,
                                                         uint32_t* __restrict__ ctr) {
  __shared__ uint32_t h[SegCtr<Fs>::kIB];
  seg_place_body<Fs>(n, span, sbase, star, bucket, ref, cref, ipos, len, dtmp, drec, ctr, h, blockIdx.x, gridDim.x);
}

template <class Fs>
__device__ __forceinline__ uint32_t seg_key(const typename Fs::Dec& d, int c, uint32_t L) {
  return (uint32_t)Fs::block(c, c ? d.b.bk : d.b.wk) * SegCtr<Fs>::kNB + seg_len_bin(L) * Fs::kClasses +
         seg_count_class<Fs::kClasses>((uint32_t)d.nfeat);
}

// The sort kernel runs one thread per item k < cref[2n] (refresh of
// perspective k >= cref[n]); invalid positions are refreshes with len 0.
// Sorted item record: {root | half << 24 | bucket << 25, length, perspective,
// list length + 1}; full feature list of the root as in the sliced plan.
// (As workgroup bid of nb on LDS lcnt / lbase of SegCtr<Fs>::kIB words and
// lists of 1024 * kListStrideWords words.)
template <class Fs>
__device__ __forceinline__ void seg_scatter_body(const typename Fs::Pos* __restrict__ pos, uint32_t n,
                                                 const uint32_t* __restrict__ cref, const uint32_t* __restrict__ ipos,
                                                 const uint32_t* __restrict__ len, uint32_t* __restrict__ ctr,
                                                 uint4* __restrict__ items, uint16_t* __restrict__ flist,
                                                 uint32_t* __restrict__ lcnt, uint32_t* __restrict__ lbase,
                                                 uint32_t* __restrict__ lists, uint32_t bid, uint32_t nb) {
  constexpr int kIB = SegCtr<Fs>::kIB;
  const uint32_t K = cref[2 * n], K0 = cref[n];
  // Grid-stride over 1024-item blocks: the item count is known only here, and
  // a grid sized for 2n items launched mostly empty 103-KB workgroups.
  for (uint32_t b0 = bid * blockDim.x; b0 < K; b0 += nb * blockDim.x) {
    __syncthreads();  // the previous block's LDS counts are read
    for (int i = threadIdx.x; i < kIB; i += blockDim.x) lcnt[i] = 0;
    __syncthreads();
    const uint32_t k = b0 + threadIdx.x;
    const uint32_t c = k >= K0 ? 1u : 0u, i = k < K ? ipos[k] : 0u;
    const uint32_t L = k < K ? len[c * n + i] : 0u;
    const bool live = L != 0;
    typename Fs::Dec d;
    uint32_t key = 0, rk = 0;
    if (live) {
      d = Fs::decode(pos + i);
      key = seg_key<Fs>(d, (int)c, L);
      rk = atomicAdd(&lcnt[key], 1u);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < kIB; t += blockDim.x)
      lbase[t] = lcnt[t] ? atomicAdd(&ctr[SegCtr<Fs>::kCur + t], lcnt[t]) : 0;
    __syncthreads();
    if (live) {
      const uint32_t slot = lbase[key] + rk;
      const uint32_t half = d.b.stm == (int)c ? 0u : 1u, bk = (uint32_t)(d.b.cnt - 1) >> 2;
      items[slot] = make_uint4(i | half << 24 | bk << 25, L, c, (uint32_t)d.nfeat);
      const uint32_t pp = (slot - ctr[SegCtr<Fs>::kOff + (key / SegCtr<Fs>::kNB) * SegCtr<Fs>::kNB]) & 1u;  // parity in its king block
      Fs::write_list(d, (int)c, slot, pp, lists + threadIdx.x * kListStrideWords, flist);
    }
  }
}

template <class Fs>
__global__ __launch_bounds__(1024) void seg_scatter_kernel(const typename Fs::Pos* __restrict__ pos, uint32_t n,
                                                           const uint32_t* __restrict__ cref,
                                                           const uint32_t* __restrict__ ipos,
                                                           const uint32_t* __restrict__ len,
                                                           uint32_t* __restrict__ ctr, uint4* __restrict__ items,
                                                           uint16_t* __restrict__ flist) {
  constexpr int kIB = SegCtr<Fs>::kIB;
  __shared__ uint32_t lcnt[kIB];
  __shared__ uint32_t lbase[kIB];
  __shared__ uint32_t lists[1024 * kListStrideWords];  // list staging, one row per lane
  seg_scatter_body<Fs>(pos, n, cref, ipos, len, ctr, items, flist, lcnt, lbase, lists, blockIdx.x, gridDim.x);
}

// The whole plan of a small grouped call (npos <= kSegSmallPlan, one chunk)
// in ONE workgroup: group spans (and the offset check), deltas, the scan of
// refresh flags, segment placement, the unit table and the sorted items with
// their lists — the phases of group_span .. seg_scatter, separated by
// workgroup barriers instead of kernel boundaries (for a game or a few, each
// of those eight launches is mostly its launch-to-launch gap: ~45 µs in all,
// profiles/r05/backend/timeline_1batch.txt).  Global memory written by one
// phase is read by the next from the same CU, ordered by the barrier.
// Its one workgroup walks the positions in rounds of 1024, so past ~2k
// positions the eight-kernel chain is faster: engine-actor calls of 24 / 32 /
// 48 / 64 batches (2.4k-6.3k plies) took 0.192 / 0.203 / 0.238 / 0.267 ms with
// a limit of 8192 and 0.185 / 0.192 / 0.208 / 0.221 ms with 2048, calls of
// 1-16 batches the same (profiles/r05/small_plan/).
constexpr uint32_t kSegSmallPlan = 2048;
template <class Fs>
constexpr int seg_small_lds_words() {
  constexpr int kIB = SegCtr<Fs>::kIB;
  constexpr int scatter = 2 * kIB + 1024 * kListStrideWords;
  constexpr int scan = plan_scan_lds_words<Fs::KB, SegCtr<Fs>::kNB>();
  return scatter > scan ? scatter : scan;
}
template <class Fs>
__global__ __launch_bounds__(1024) void seg_plan_small_kernel(const typename Fs::Pos* __restrict__ pos, uint32_t n,
                                                              const uint32_t* __restrict__ off, uint32_t ngroups,
                                                              uint2* __restrict__ span, int star,
                                                              uint32_t* __restrict__ ref, uint4* __restrict__ dtmp,
                                                              uint8_t* __restrict__ bucket, uint32_t* __restrict__ err,
                                                              uint32_t* __restrict__ cref, uint32_t* __restrict__ ipos,
                                                              uint32_t* __restrict__ len, uint4* __restrict__ drec,
                                                              uint32_t* __restrict__ ctr, int4* __restrict__ units,
                                                              uint32_t seg_plies, uint4* __restrict__ items,
                                                              uint16_t* __restrict__ flist) {
  constexpr int kIB = SegCtr<Fs>::kIB;
  __shared__ uint32_t lds[seg_small_lds_words<Fs>()];
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // counters, then each group's span entries (one wave per group) and the
  // offset check; a group longer than kSpanChunk: its chunks' entries after
  for (uint32_t k = t; k < (uint32_t)SegCtr<Fs>::kWords; k += 1024) ctr[k] = 0;
  for (uint32_t g = wv; g < ngroups; g += 16) group_span_one(off, ngroups, n, span, 1, err, g, lane);
  __syncthreads();
  for (uint32_t c0 = 0; c0 < n; c0 += kSpanChunk) {
    const uint2 v = span[c0];
    if (v.y - v.x <= kSpanChunk) continue;
    const uint32_t e = min(c0 + kSpanChunk, min(v.y, n));
    for (uint32_t i = c0 + 1 + t; i < e; i += 1024) span[i] = v;
  }
  __syncthreads();
  // deltas and refresh flags, 1024 positions at a time (their decodes shared
  // through LDS as seg_delta_kernel's block of 256 does)
  for (uint32_t i0 = 0; i0 < n; i0 += 1024) {
    const uint32_t i = i0 + t;
    typename Fs::Dec B;
    B.ok = B.over = false;
    B.b.wk = B.b.bk = 0;
    if (i < n) B = Fs::template decode<false>(pos + i);
    lds[t] = seg_info(B);
    __syncthreads();
    uint32_t r0 = 0, r1 = 0;
    if (i < n) seg_delta_one<Fs>(pos, n, span, 0u, star, ref, dtmp, bucket, err, i, i0, lds, B, r0, r1);
    __syncthreads();
  }
  // cref = exclusive scan of the refresh flags over both perspectives (2n),
  // ipos[k] = the position of item k, cref[2n] = the item count
  uint32_t base = 0;
  for (uint32_t j0 = 0; j0 < 2 * n; j0 += 1024) {
    const uint32_t j = j0 + t;
    const uint32_t r = j < 2 * n ? ref[j] : 0u;
    const uint64_t bal = __ballot(r != 0);
    if (lane == 0) lds[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t below = (uint32_t)__popcll(bal & ((1ull << lane) - 1)), tot = 0;
    for (uint32_t w = 0; w < 16; ++w) {
      const uint32_t c = lds[w];
      below += w < wv ? c : 0u;
      tot += c;
    }
    if (j < 2 * n) {
      const uint32_t k = base + below;
      cref[j] = k;
      if (r) ipos[k] = j >= n ? j - n : j;
    }
    base += tot;
    __syncthreads();
  }
  if (t == 0) cref[2 * n] = base;
  __syncthreads();
  seg_place_body<Fs>(n, span, 0u, star, bucket, ref, cref, ipos, len, dtmp, drec, ctr, lds, 0u, 1u);
  __syncthreads();
  plan_scan_body<Fs::KB, SegCtr<Fs>::kNB>(ctr, units, 0u, seg_plies, nullptr, lds);
  __syncthreads();
  seg_scatter_body<Fs>(pos, n, cref, ipos, len, ctr, items, flist, lds, lds + kIB, lds + 2 * kIB, 0u, 1u);
}

struct SegFetch {
  uint4 rec;
  uint2 lst;
};

__device__ __forceinline__ SegFetch fetch_seg(__amdgpu_buffer_rsrc_t items, __amdgpu_buffer_rsrc_t flist,
                                              int pass_base, int last, int lane, int it_in_wave) {
  SegFetch f;
  const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(items, (uint32_t)min(pass_base + it_in_wave, last) * 16u, 0, 0);
  f.rec = make_uint4(r.x, r.y, r.z, r.w);
  const uint32_t li = (uint32_t)min(pass_base + (lane >> 3), last);
  const u32x2 l = __builtin_amdgcn_raw_buffer_load_b64(flist, li * 64u + 8u * (uint32_t)(lane & 7), 0, 0);
  f.lst = make_uint2(l.x, l.y);
  return f;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

// One delta position: cur = base -/+ the removed / added rows of record d.
// kAdd2 = false when no record of the batch has a second added piece (only
// the other side's castling has one), which skips that row.  kSwar: rows and
// accumulators are SWAR words (sliced_common.h), so each column pair costs
// 32-bit VOP2 adds / subtracts instead of VOP3P packed ones; every
// intermediate is a subset sum of one position's features, inside the bound
// that enabled SWAR.
template <bool kAdd2, bool kSwar>
__device__ __forceinline__ void apply_delta(const char* lbase, const uint4& d, u16x4 b_lo, u16x4 b_hi, u16x4& lo,
                                            u16x4& hi) {
  const u32x4 r0 = *row_addr(lbase, d.y, 0), r1 = *row_addr(lbase, d.y, 1);
  const u32x4 a0 = *row_addr(lbase, d.z, 0);
  auto lo2 = [](const u32x4& v) { return __builtin_shufflevector(v, v, 0, 1); };
  auto hi2 = [](const u32x4& v) { return __builtin_shufflevector(v, v, 2, 3); };
  if constexpr (kSwar) {
    u32x2 l = __builtin_bit_cast(u32x2, b_lo) - (lo2(r0) + lo2(r1)) + lo2(a0);
    u32x2 h = __builtin_bit_cast(u32x2, b_hi) - (hi2(r0) + hi2(r1)) + hi2(a0);
    if constexpr (kAdd2) {
      const u32x4 a1 = *row_addr(lbase, d.z, 1);
      l += lo2(a1);
      h += hi2(a1);
    }
    lo = __builtin_bit_cast(u16x4, l);
    hi = __builtin_bit_cast(u16x4, h);
  } else {
    auto c = [](u32x2 v) { return __builtin_bit_cast(u16x4, v); };
    lo = b_lo - c(lo2(r0)) - c(lo2(r1)) + c(lo2(a0));
    hi = b_hi - c(hi2(r0)) - c(hi2(r1)) + c(hi2(a0));
    if constexpr (kAdd2) {
      const u32x4 a1 = *row_addr(lbase, d.z, 1);
      lo += c(lo2(a1));
      hi += c(hi2(a1));
    }
  }
}

template <bool kAdd2>
__device__ __forceinline__ int32_t psqt_delta(const int32_t* ptile, const uint4& d, int q) {
  auto p = [&](uint32_t e) { return (uint32_t)ptile[(e >> 4) * kPsqtBuckets + q]; };
  const uint32_t a2 = kAdd2 ? p(d.z >> 16) : 0u;
  return (int32_t)(p(d.z & 0xFFFFu) + a2 - p(d.y & 0xFFFFu) - p(d.y >> 16));
}

// One pass = 8 segment items per wave.  Refresh position: as slice_pass
// (ft_sliced.hip) but the PSQT sum keeps all 8 buckets, one per lane q of the
// item, because the bucket changes along a segment (kPsqt: slice 0 only).
// Then the wave walks the longest segment of the pass; finished items turn
// their rows into the zero row and their stores out of range (dropped).
constexpr int kDbufStride = 9;  // records per item in the per-wave LDS buffer (8 + 1 padding)
// One LDS buffer per wave serves both the pass's feature lists (64 x 8 B) and
// the walk's delta records (8 items x kDbufStride x 16 B): a wave uses them
// one after the other and its LDS operations complete in order, so they share
// the bytes (the crazyhouse tile and its PSQT tile then still fit in 160 KB).
// may_alias types and compiler barriers keep the two views ordered.
constexpr int kWaveBufU4 = 8 * kDbufStride;
typedef uint2 lds_u2 __attribute__((may_alias));
typedef uint4 lds_u4 __attribute__((may_alias));

template <int HD, bool kStar, bool kPsqt, bool kSwar, uint32_t kNone>
__device__ __forceinline__ void seg_pass(const SegFetch& f, uint4* __restrict__ wbuf, int lane, int it_in_wave, int s,
                                         int q, uint32_t n, const char* lbase, u16x4 b_lo, u16x4 b_hi, int krow,
                                         const int32_t* ptile, __amdgpu_buffer_rsrc_t psqt_rsrc,
                                         __amdgpu_buffer_rsrc_t x_rsrc, __amdgpu_buffer_rsrc_t drec_rsrc) {
  const uint4 rec = f.rec;
  const uint32_t maxn = __builtin_amdgcn_readfirstlane(wave_max_u32(rec.w));
  const uint32_t maxL = __builtin_amdgcn_readfirstlane(wave_max_u32(rec.y));
  asm volatile("" ::: "memory");  // the previous pass's record reads come first
  reinterpret_cast<lds_u2*>(wbuf)[lane] = f.lst;
  uint32_t e[16];
  const lds_u4* my = reinterpret_cast<const lds_u4*>(wbuf) + 4 * it_in_wave;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint4 v = my[m];
    e[4 * m] = v.x;
    e[4 * m + 1] = v.y;
    e[4 * m + 2] = v.z;
    e[4 * m + 3] = v.w;
  }
  u16x4 lo = b_lo, hi = b_hi;
  rows_sum<kSwar>((int)maxn - 1, e, lbase, lo, hi);
  const uint32_t col = 32 * s + 4 * q;
  __builtin_amdgcn_raw_buffer_store_b32(kSwar ? transform4_swar(lo, hi) : transform4(lo, hi), x_rsrc,
                                        ((rec.x & kSlotMask) * 2 + ((rec.x >> 24) & 1)) * (HD / 2) + col, 0, 0);
  int32_t p = 0;
  auto psqt_off = [&](uint32_t x, bool live) {
    return (live && (int)(x >> 25) == q) ? ((x & kSlotMask) * 2 + ((x >> 24) & 1)) * 4u : kDroppedOffset;
  };
  if constexpr (kPsqt) {
    // the list is already in registers (e): entries 2j, 2j+1 in e[j]
    uint32_t acc = (uint32_t)ptile[krow * kPsqtBuckets + q];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc += (uint32_t)ptile[((e[j] & 0xFFFFu) >> 4) * kPsqtBuckets + q] +
             (uint32_t)ptile[(e[j] >> 20) * kPsqtBuckets + q];
    p = (int32_t)acc;
    __builtin_amdgcn_raw_buffer_store_b32(p, psqt_rsrc, psqt_off(rec.x, true), 0, 0);
  }
  if (maxL <= 1) return;
  // Delta positions k = 1 .. maxL-1, records at drec[c*n + root + k], in
  // batches of 8: lane q of an item loads record 8b+1+q (one 16-B load per
  // lane per 8 positions, the next batch prefetched) and spreads the batch
  // through the wave's LDS buffer; the 8 positions of a batch are straight-
  // line code, so their LDS reads issue ahead of the accumulator chain.
  // Finished items (k >= L) read the sentinel record 2n: zero rows, stores
  // past the buffer ranges (dropped).
  const uint32_t rbase = (rec.z * n + (rec.x & kSlotMask)) * 16u;
  auto fetch = [&](uint32_t k) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(drec_rsrc, k < rec.y ? rbase + 16u * k : 32u * n, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
  };
  // 9 records of stride per item (one padding record): the two items of a
  // ds_read_b96 lane group ({0-3,20-23}: items 0 and 1; banks (a/4) mod 32)
  // then read records 144 B apart, 4 banks, instead of 128 B = the same banks.
  asm volatile("" ::: "memory");  // this pass's list reads come first
  lds_u4* db = reinterpret_cast<lds_u4*>(wbuf) + kDbufStride * it_in_wave;
  const uint32_t nb = __builtin_amdgcn_readfirstlane((maxL - 1 + 7) / 8);  // batches, wave-uniform
  constexpr int kAhead = 1;  // batches of records in flight ahead of the current one (2: no gain, r01)
  uint4 next[kAhead];
#pragma unroll
  for (int a = 0; a < kAhead; ++a) next[a] = fetch(8 * a + 1 + q);
  u16x4 blo = lo, bhi = hi;
  int32_t pb = p;
  // Positions in the last batch (1..8, wave-uniform): the walk stops at the
  // pass's longest segment instead of rounding it up to whole batches (even
  // lengths dominate CHAIN segments in random games — a king moves every
  // other ply — and 23 % of the position steps of config 3 were past every
  // item's end).
  const uint32_t rest = maxL - 1 - 8 * (nb - 1);
  // The positions of a batch, straight-line; kAdd2 as in apply_delta; kLast:
  // only the first `rest` (uniform branches).
  auto run_batch = [&](auto add2, auto last) {
    constexpr bool kAdd2 = decltype(add2)::value, kLast = decltype(last)::value;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      if (kLast && jj > 0 && (uint32_t)jj >= rest) break;
      const uint4 d = db[jj];  // past the segment's end: the sentinel record (seg_place_kernel)
      apply_delta<kAdd2, kSwar>(lbase, d, blo, bhi, lo, hi);
      const uint32_t xo = (d.x & kRowMask) * (HD / 2) + col;
      __builtin_amdgcn_raw_buffer_store_b32(kSwar ? transform4_swar(lo, hi) : transform4(lo, hi), x_rsrc, xo, 0, 0);
      int32_t pc = 0;
      if constexpr (kPsqt) {
        pc = (int32_t)((uint32_t)pb + (uint32_t)psqt_delta<kAdd2>(ptile, d, q));
        const uint32_t po = (int)(d.x >> 25) == q ? (d.x & kRowMask) * 4u : kDroppedOffset;
        __builtin_amdgcn_raw_buffer_store_b32(pc, psqt_rsrc, po, 0, 0);
      }
      if constexpr (!kStar) {
        blo = lo;
        bhi = hi;
        pb = pc;
      }
    }
  };
  for (uint32_t b = 0; b < nb; ++b) {
    const uint4 batch = next[0];
#pragma unroll
    for (int a = 0; a + 1 < kAhead; ++a) next[a] = next[a + 1];
    next[kAhead - 1] = fetch(8 * (b + kAhead) + 1 + q);
    db[q] = batch;  // LDS ops of a wave complete in order: read below, overwritten next batch
    // lane q of an item holds record 8b+1+q: any with a second add?
    const bool add2 = __ballot((batch.z >> 16) != kNone) != 0;
    if (b + 1 < nb) {
      if (add2)
        run_batch(std::true_type{}, std::false_type{});
      else
        run_batch(std::false_type{}, std::false_type{});
    } else {
      if (add2)
        run_batch(std::true_type{}, std::true_type{});
      else
        run_batch(std::false_type{}, std::true_type{});
    }
  }
}

// One net's view for a (unit, slice) task: its LDS-tile image, bias, PSQT
// rows, and the buffer resources of its PSQT parts and x (the plan's items,
// lists and delta records are the same for every net of the feature set).
struct SegNet {
  const uint4* tiles;
  const int16_t* ftb;
  const int32_t* psqw;
  __amdgpu_buffer_rsrc_t psqt_rsrc, x_rsrc;
};

// Buffer ranges are the launch's exact extents (x: n rows of HD bytes, < 2^31;
// psqt_part: 2n words; drec: 2n + 1 records, the last the sentinel record 2n).
// Items past their segment's end read the sentinel, whose x row 2n and PSQT
// word 2n fall just past the x and psqt_part ranges, so the hardware drops
// those stores; other dropped stores use kDroppedOffset.  No record can reach
// beyond the launch's rows.
template <int HD>
__device__ __forceinline__ SegNet seg_net(const uint4* tiles, const int16_t* ftb, const int32_t* psqw,
                                          int32_t* psqt_part, uint8_t* x, uint32_t n) {
  return SegNet{tiles, ftb, psqw, __builtin_amdgcn_make_buffer_rsrc(psqt_part, 0, (int)(8 * n), kBufferFlags),
                __builtin_amdgcn_make_buffer_rsrc(x, 0, (int)min((uint64_t)n * HD, (uint64_t)kBufferRange),
                                                  kBufferFlags)};
}

// The LDS a task works in (declared by the kernel): the tile, the PSQT tile,
// one buffer per wave (a pass's lists, then its delta records) and the pass
// counter.
template <class Fs>
struct SegLds {
  uint4 img[Fs::G::kTileU4];
  int32_t ptile[Fs::G::kTileRows * kPsqtBuckets];
  uint4 wbufs[16][kWaveBufU4];
  uint32_t claim;  // next pass of the unit to hand out
};

// Column slice s (of the net's HD / 64) of `unit`: the tile to LDS, the own
// king into the bias, then the unit's passes, claimed longest first.
template <int HD, bool kStar, bool kSwar, class Fs>
__device__ __forceinline__ void seg_task(SegLds<Fs>& L, const SegNet& net, int s, const int4 u, uint32_t n,
                                         __amdgpu_buffer_rsrc_t items_rsrc, __amdgpu_buffer_rsrc_t flist_rsrc,
                                         __amdgpu_buffer_rsrc_t drec_rsrc) {
  constexpr int S = HD / 64;
  using G = typename Fs::G;
  constexpr int kTileU4 = G::kTileU4;
  constexpr int kTileLoads = (kTileU4 + 1023) / 1024;
  constexpr int kPtileU4 = G::kTileRows * kPsqtBuckets / 4, kPtileRealU4 = G::kRows * kPsqtBuckets / 4;
  static_assert(kPtileU4 <= 2048, "PSQT tile loads: two per thread");
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int it_in_wave, q;
  lane_item(lane, it_in_wave, q);
  uint4* wb = L.wbufs[wv];
  __syncthreads();  // the previous unit's tile reads are done before the reload
  if (threadIdx.x == 0) L.claim = 16;
  const uint4* src = net.tiles + ((size_t)u.x * S + s) * kTileU4;
  uint4 t[kTileLoads];
#pragma unroll
  for (int k = 0; k < kTileLoads; ++k) t[k] = src[min((int)threadIdx.x + 1024 * k, kTileU4 - 1)];
  uint4 pt[2];
  const uint4* psrc = reinterpret_cast<const uint4*>(net.psqw + (size_t)u.x * G::kRows * kPsqtBuckets);
  if (s == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) pt[k] = psrc[min((int)threadIdx.x + 1024 * k, kPtileRealU4 - 1)];
  }
  u16x4 b_lo = *reinterpret_cast<const u16x4*>(net.ftb + 32 * s + 4 * q);
  u16x4 b_hi = *reinterpret_cast<const u16x4*>(net.ftb + HD / 2 + 32 * s + 4 * q);
  const int krow = G::king_row(u.x);
  const char* lbase = reinterpret_cast<const char*>(L.img) + G::kPlaneBytes * q;
  const int last = u.z - 1;
  // Passes are handed out longest first (items are sorted by length bin, so
  // from the unit's end backwards), the next one claimed from an LDS counter
  // when the current one starts: waves finish within one pass of each other.
  const int npass = (u.z - u.y + 7) / 8;
  auto pass_base = [&](int k) { return k < npass ? u.y + (npass - 1 - k) * 8 : (int)u.z; };
  int kp = wv;
  int base = pass_base(kp);
  SegFetch fa = fetch_seg(items_rsrc, flist_rsrc, base, last, lane, it_in_wave);
#pragma unroll
  for (int k = 0; k < kTileLoads; ++k)
    if ((int)threadIdx.x + 1024 * k < kTileU4) {
      uint4 v = t[k];
      if constexpr (kSwar) v = swar_tile_words(v);
      L.img[threadIdx.x + 1024 * k] = v;
    }
  if (s == 0) {
    uint4* pdst = reinterpret_cast<uint4*>(L.ptile);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = (int)threadIdx.x + 1024 * k;
      if (i < kPtileU4) pdst[i] = i < kPtileRealU4 ? pt[k] : make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();
  {  // the own-king row (every item of the unit has it) joins the bias
    const u32x4 kv = *reinterpret_cast<const u32x4*>(lbase + 16 * krow);
    if constexpr (kSwar) {
      b_lo = swar_words(b_lo);
      b_hi = swar_words_hi(b_hi);
    }
    accum_row<kSwar>(kv, b_lo, b_hi);
    if constexpr (kSwar) {  // both halves of every word offset by 0x8000 (transform4_swar)
      b_lo = __builtin_bit_cast(u16x4, __builtin_bit_cast(u32x2, b_lo) + kSwarOffset);
      b_hi = __builtin_bit_cast(u16x4, __builtin_bit_cast(u32x2, b_hi) + kSwarOffset);
    }
  }
  while (base < u.z) {
    const SegFetch cur = fa;
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&L.claim, 1u);
    kp = __builtin_amdgcn_readfirstlane((int)c);
    const int next = pass_base(kp);
    fa = fetch_seg(items_rsrc, flist_rsrc, next, last, lane, it_in_wave);
    if (s == 0)
      seg_pass<HD, kStar, true, kSwar, Fs::kNone>(cur, wb, lane, it_in_wave, s, q, n, lbase, b_lo, b_hi, krow,
                                                  L.ptile, net.psqt_rsrc, net.x_rsrc, drec_rsrc);
    else
      seg_pass<HD, kStar, false, kSwar, Fs::kNone>(cur, wb, lane, it_in_wave, s, q, n, lbase, b_lo, b_hi, krow,
                                                   L.ptile, net.psqt_rsrc, net.x_rsrc, drec_rsrc);
    base = next;
  }
}

template <int HD, bool kStar, bool kSwar, class Fs>
__global__ __launch_bounds__(1024) void ft_segments_kernel(const uint4* __restrict__ tiles,
                                                           const int16_t* __restrict__ ftb,
                                                           const uint32_t* __restrict__ ctr,
                                                           const int4* __restrict__ units,
                                                           const uint4* __restrict__ items,
                                                           const uint16_t* __restrict__ flist,
                                                           const uint4* __restrict__ drec, uint32_t n,
                                                           const int32_t* __restrict__ psqw,
                                                           int32_t* __restrict__ psqt_part,
                                                           uint8_t* __restrict__ x) {
  constexpr int S = HD / 64;
  __shared__ SegLds<Fs> L;
  const SegNet net = seg_net<HD>(tiles, ftb, psqw, psqt_part, x, n);
  const __amdgpu_buffer_rsrc_t items_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(items), 0, kBufferAll, kBufferFlags);
  const __amdgpu_buffer_rsrc_t flist_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(flist), 0, kBufferAll, kBufferFlags);
  const __amdgpu_buffer_rsrc_t drec_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(drec), 0, (int)(32 * n + 16), kBufferFlags);
  // Grid-stride over (unit, slice) pairs: the unit count is known only on the
  // device and its bound (seg_max_units) is far above typical counts.  The
  // grid is a multiple of 8 * S, so every pair keeps its XCD-aware mapping.
  const uint32_t nunits = ctr[SegCtr<Fs>::kNUnits];
  for (uint32_t w = blockIdx.x;; w += gridDim.x) {
    const uint32_t j = w >> 3;
    const uint32_t unit = (j / S) * 8 + (w & 7);
    if (unit >= nunits) return;
    seg_task<HD, kStar, kSwar, Fs>(L, net, (int)(j % S), units[unit], n, items_rsrc, flist_rsrc, drec_rsrc);
  }
}

template <int HD, class Fs>
hipError_t ft_segments_t(const SegPlan& G, const SlicedPlan& P, const NetPtrs& net, uint32_t n, bool star,
                         uint8_t* x, uint32_t max_units, hipStream_t stream) {
  constexpr int S = HD / 64;
  // grid = 8 * S * G (see the kernel's grid stride); up to 8 * 64 units per sweep
  const uint32_t groups = min((max_units + 7) / 8, 64u);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(groups * 8 * S), dim3(1024), 0, stream, (const uint4*)P.tiles, net.ft_bias, P.ctr,
                       (const int4*)P.units, (const uint4*)G.items, P.flist, (const uint4*)G.drec, n, net.psqt_w,
                       P.psqt_part, x);
  };
  if (star)
    P.swar ? launch(ft_segments_kernel<HD, true, true, Fs>) : launch(ft_segments_kernel<HD, true, false, Fs>);
  else
    P.swar ? launch(ft_segments_kernel<HD, false, true, Fs>) : launch(ft_segments_kernel<HD, false, false, Fs>);
  return hipGetLastError();
}

// The plan of one chunk for feature set Fs (see the file comment), then the
// dispatch of the main kernel over the net width.
template <class Fs>
hipError_t seg_plan_t(const typename Fs::Pos* pos, uint32_t n, const uint2* sp, uint32_t sbase, bool star,
                      const SlicedPlan& P, const SegPlan& G, uint8_t* bucket, uint32_t* err, hipStream_t stream) {
  hipError_t e;
  const uint32_t bs = 256, g1 = (n + bs - 1) / bs;
  if (g1 > kMaxScanBlocks) return hipErrorInvalidValue;
  uint32_t* bsum = static_cast<uint32_t*>(G.scan_temp);
  hipLaunchKernelGGL(seg_delta_kernel<Fs>, dim3(g1), dim3(bs), 0, stream, pos, n, sp, sbase, star ? 1 : 0, G.ref,
                     (uint4*)G.dtmp, bucket, err, bsum, P.ctr, (uint32_t)SegCtr<Fs>::kWords);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // cref = exclusive scan of ref (reduce in seg_delta, scan of the block sums, local scans)
  hipLaunchKernelGGL(seg_scan_blocks_kernel, dim3(1), dim3(1024), 0, stream, bsum, g1, n, G.cref);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(seg_items_scan_kernel, dim3(g1, 2), dim3(256), 0, stream, n, G.ref, bsum, G.cref, G.ipos);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  uint32_t cb = (2 * n + 1023) / 1024;
  if (cb > 256) cb = 256;
  hipLaunchKernelGGL(seg_place_kernel<Fs>, dim3(cb), dim3(1024), 0, stream, n, sp, sbase, star ? 1 : 0, bucket, G.ref,
                     G.cref, G.ipos, G.len, (const uint4*)G.dtmp, (uint4*)G.drec, P.ctr);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((plan_scan_kernel_t<Fs::KB, SegCtr<Fs>::kNB>), dim3(1), dim3(1024), 0, stream, P.ctr, (int4*)P.units, 0u,
                     G.unit_plies);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(seg_scatter_kernel<Fs>, dim3(min((2 * n + 1023) / 1024, 512u)), dim3(1024), 0, stream, pos, n, G.cref,
                     G.ipos, G.len, P.ctr, (uint4*)G.items, P.flist);
  return hipGetLastError();
}

}  // namespace

// units close at unit_plies of work, an item weighing at most
// seg_bin_weight(32): a unit holding fewer than kSegUnitPlies / that many items
// is its king block's last
uint32_t seg_max_units(uint32_t chunk, uint32_t unit_plies) {
  const uint32_t per = (unit_plies ? unit_plies : std::min(kSegUnitPlies, kSegUnitPliesSmall)) / seg_bin_weight(32);
  return 64 + (2 * chunk + per - 1) / per;
}

uint32_t seg_unit_plies(uint32_t hd) { return seg_unit_plies_for(hd); }

size_t seg_ctr_words() {
  return std::max({SegCtr<ChessFs>::kWords, SegCtr<VariantFs<kVariantCrazyhouse>>::kWords,
                   SegCtr<VariantFs<kVariantAtomic>>::kWords});
}

// the per-block refresh counts of seg_delta, two perspectives
size_t seg_scan_temp_bytes(uint32_t chunk) { return (size_t)8 * ((chunk + 255) / 256 + 1); }

#define FNNUE_HD_DISPATCH(hd, CALL) \
  switch (hd) {                     \
    case 128: return CALL(128);     \
    case 256: return CALL(256);     \
    case 512: return CALL(512);     \
    case 1024: return CALL(1024);   \
    case 1536: return CALL(1536);   \
    case 2048: return CALL(2048);   \
    case 2560: return CALL(2560);   \
    case 3072: return CALL(3072);   \
    default: return hipErrorInvalidValue; \
  }

hipError_t launch_group_span(const uint32_t* off, uint32_t ngroups, uint32_t npos, void* span, bool check,
                             uint32_t* err, hipStream_t stream) {
  if (ngroups == 0) return hipSuccess;
  hipLaunchKernelGGL(group_span_kernel, dim3((ngroups + 3) / 4), dim3(256), 0, stream, off, ngroups, npos,
                     static_cast<uint2*>(span), check ? 1 : 0, err);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !span || npos == 0) return e;
  hipLaunchKernelGGL(group_span_big_kernel, dim3((npos + kSpanChunk - 1) / kSpanChunk), dim3(256), 0, stream, npos,
                     static_cast<uint2*>(span));
  return hipGetLastError();
}

hipError_t launch_seg_plan(int variant, const void* pos, uint32_t n, const void* span, uint32_t sbase, int mode,
                           const SlicedPlan& P, const SegPlan& G, uint8_t* bucket, uint32_t* err, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const bool star = mode == FNNUE_GROUP_STAR;
  const uint2* sp = static_cast<const uint2*>(span);
  if (variant == kVariantChess)
    return seg_plan_t<ChessFs>(static_cast<const fnnue_pos*>(pos), n, sp, sbase, star, P, G, bucket, err, stream);
  const fnnue_vpos* vp = static_cast<const fnnue_vpos*>(pos);
  if (variant == kVariantCrazyhouse)
    return seg_plan_t<VariantFs<kVariantCrazyhouse>>(vp, n, sp, sbase, star, P, G, bucket, err, stream);
  if (variant == kVariantAtomic)
    return seg_plan_t<VariantFs<kVariantAtomic>>(vp, n, sp, sbase, star, P, G, bucket, err, stream);
  return hipErrorInvalidValue;
}

uint32_t seg_small_plan_max() { return kSegSmallPlan; }

hipError_t launch_seg_plan_small(int variant, const void* pos, uint32_t n, const uint32_t* off, uint32_t ngroups,
                                 void* span, int mode, const SlicedPlan& P, const SegPlan& G, uint8_t* bucket,
                                 uint32_t* err, hipStream_t stream) {
  if (n == 0 || n > kSegSmallPlan) return hipErrorInvalidValue;
  const int star = mode == FNNUE_GROUP_STAR ? 1 : 0;
#define FNNUE_SMALL_PLAN(Fs, P_T)                                                                                  \
  hipLaunchKernelGGL(seg_plan_small_kernel<Fs>, dim3(1), dim3(1024), 0, stream, static_cast<const P_T*>(pos), n, off, \
                     ngroups, static_cast<uint2*>(span), star, G.ref, (uint4*)G.dtmp, bucket, err, G.cref, G.ipos,  \
                     G.len, (uint4*)G.drec, P.ctr, (int4*)P.units, G.unit_plies, (uint4*)G.items, P.flist);        \
  return hipGetLastError();
  if (variant == kVariantChess) { FNNUE_SMALL_PLAN(ChessFs, fnnue_pos) }
  if (variant == kVariantCrazyhouse) { FNNUE_SMALL_PLAN(VariantFs<kVariantCrazyhouse>, fnnue_vpos) }
  if (variant == kVariantAtomic) { FNNUE_SMALL_PLAN(VariantFs<kVariantAtomic>, fnnue_vpos) }
#undef FNNUE_SMALL_PLAN
  return hipErrorInvalidValue;
}

hipError_t launch_seg_units(int variant, const SlicedPlan& P, void* units, uint32_t* ctr_out, uint32_t unit_plies,
                            hipStream_t stream) {
#define FNNUE_SEG_UNITS(Fs)                                                                                       \
  hipLaunchKernelGGL((plan_scan_kernel_t<Fs::KB, SegCtr<Fs>::kNB>), dim3(1), dim3(1024), 0, stream, P.ctr,       \
                     static_cast<int4*>(units), 0u, unit_plies, ctr_out + SegCtr<Fs>::kNUnits);                   \
  return hipGetLastError();
  if (variant == kVariantChess) { FNNUE_SEG_UNITS(ChessFs) }
  if (variant == kVariantCrazyhouse) { FNNUE_SEG_UNITS(VariantFs<kVariantCrazyhouse>) }
  if (variant == kVariantAtomic) { FNNUE_SEG_UNITS(VariantFs<kVariantAtomic>) }
#undef FNNUE_SEG_UNITS
  return hipErrorInvalidValue;
}

hipError_t launch_seg_ft(uint32_t hd, int variant, uint32_t n, int mode, const NetPtrs& net, const SlicedPlan& P,
                         const SegPlan& G, uint8_t* x, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const bool star = mode == FNNUE_GROUP_STAR;
  const uint32_t mu = seg_max_units(n, G.unit_plies);
  if (variant == kVariantChess) {
#define CALL(H) ft_segments_t<H, ChessFs>(G, P, net, n, star, x, mu, stream)
    FNNUE_HD_DISPATCH(hd, CALL)
#undef CALL
  }
#define FNNUE_VSEG(V)                                                                    \
  {                                                                                      \
    using Fs = VariantFs<V>;                                                             \
    switch (hd) {                                                                        \
      case 256: return ft_segments_t<256, Fs>(G, P, net, n, star, x, mu, stream);        \
      case 512: return ft_segments_t<512, Fs>(G, P, net, n, star, x, mu, stream);        \
      case 1024: return ft_segments_t<1024, Fs>(G, P, net, n, star, x, mu, stream);      \
      default: return hipErrorInvalidValue;                                              \
    }                                                                                    \
  }
  if (variant == kVariantCrazyhouse) FNNUE_VSEG(kVariantCrazyhouse)
  if (variant == kVariantAtomic) FNNUE_VSEG(kVariantAtomic)
#undef FNNUE_VSEG
  return hipErrorInvalidValue;
}

hipError_t launch_ft_segments(uint32_t hd, int variant, const void* pos, uint32_t n, const void* span, uint32_t sbase,
                              int mode, const NetPtrs& net, const SlicedPlan& P, const SegPlan& G, uint8_t* x,
                              uint8_t* bucket, uint32_t* err, hipStream_t stream, hipEvent_t mid) {
  if (n == 0) return hipSuccess;
  hipError_t e = launch_seg_plan(variant, pos, n, span, sbase, mode, P, G, bucket, err, stream);
  if (e == hipSuccess && mid) e = hipEventRecord(mid, stream);
  return e != hipSuccess ? e : launch_seg_ft(hd, variant, n, mode, net, P, G, x, stream);
}

}  // namespace fnnue
