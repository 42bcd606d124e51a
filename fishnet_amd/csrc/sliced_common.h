// sliced_common.h — device pieces shared by the LDS-stationary feature
// transformer kernels (ft_sliced.hip: independent positions; ft_segments.hip:
// incremental segments of games): tile layout, lane-per-position decode,
// feature lists, the plan scan, transform and the pipelined row reads.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "kernels.h"
#include "net.h"

namespace fnnue {
namespace {

constexpr int kRowsPerBlock = 704;            // PS_NB: rows per king block
constexpr int kTileRows = kRowsPerBlock + 1;  // + one zero row
constexpr int kNoRow = kRowsPerBlock;         // the zero row
// Tile layout, in HBM and in LDS: 8 planes q (16-byte column chunks), each
// 705 rows x 16 B padded to kPlaneBytes = 11296 = 32 (mod 256).  Chunk q of row
// r then sits in banks 8q + 4r + [0,4) (mod 64): one row's 8 chunks are
// conflict-free and rows of opposite parity use complementary banks.
constexpr int kPlaneBytes = 11296;
constexpr int kPlaneU4 = kPlaneBytes / 16;    // 706
constexpr int kPlaneU4_ = kPlaneU4;
constexpr int kTileU4 = 8 * kPlaneU4;         // 5648 x 16 B = 90,368 B
// Feature-list entries are 16*row (u16), the byte offset of the row inside a
// plane: ft_slices forms the LDS address base_q + entry with one SDWA add.
constexpr uint32_t kNoEntry = 16 * kNoRow;
// Row (within king block kb) of the own-king feature: KingBuckets is a
// bijection between kb and the oriented king square o on files e-h, and the
// king plane is 10 (upstream half_ka_v2_hm.h), so every item of kb has it.
__host__ __device__ constexpr int king_row(int kb) { return 640 + 8 * (7 - (kb >> 2)) + (7 - (kb & 3)); }
constexpr int kItemBins = 32 * 33;            // key = kb * 33 + n
constexpr int kPosBins = 9;                   // bucket 0..7, 8 = invalid
constexpr int kBins = kItemBins + kPosBins;
#ifndef PLAN_WG
#define PLAN_WG 1024
#endif
constexpr int kScatterPositions = PLAN_WG;    // positions per plan_scatter workgroup (one per lane)

constexpr uint32_t kItemRowMask = 0x1FFFFF;  // item record bits 0..20: 2 * slot + half (ft_sliced.hip)

// Counter block layout (uint32 words).
constexpr int kCnt = 0, kOff = kBins, kCur = 2 * kBins, kNUnits = 3 * kBins;

// Tile geometry of a feature set, for ft_slices / relayout:
//   kRows      feature rows per own-king block (the rows a tile holds)
//   kPlaneU4   16-B entries per plane: rows + zero rows, kPlaneU4 * 16 = 32
//              (mod 256) so rows of opposite parity use complementary banks
//   kBlocks    own-king blocks; king_row(kb) = the own king's row in block
//              kb (the same for every item of kb: folded into the bias)
//   kNUnitsWord  counter word holding the unit count (plan layout)
struct ChessGeom {  // HalfKAv2_hm: 32 mirrored king buckets x 704 rows
  static constexpr int kRows = kRowsPerBlock, kPlaneU4 = kPlaneU4_, kBlocks = 32, kNUnitsWord = kNUnits;
  static constexpr int kTileRows = kRows + 1, kPlaneBytes = 16 * kPlaneU4, kTileU4 = 8 * kPlaneU4;
  __host__ __device__ static constexpr int king_row(int kb) { return fnnue::king_row(kb); }
};
// Fairy-Stockfish HalfKAv2 variants (net.h): 64 king squares x R rows, own
// king row 640 + oriented king square (= kb).  Counters: kVBins bins of
// (kb, list length) and 9 position bins, laid out as the chess block.
constexpr int kVItemBins = 64 * 33, kVBins = kVItemBins + kPosBins;
constexpr int kVCnt = 0, kVOff = kVBins, kVCur = 2 * kVBins, kVNUnits = 3 * kVBins;
template <int R>
struct VariantGeom {
  static_assert(R % 16 == 0, "plane stride must stay 32 mod 256");
  static constexpr int kRows = R, kPlaneU4 = R + 2, kBlocks = 64, kNUnitsWord = kVNUnits;
  static constexpr int kTileRows = kRows + 1, kPlaneBytes = 16 * kPlaneU4, kTileU4 = 8 * kPlaneU4;
  __host__ __device__ static constexpr int king_row(int kb) { return 640 + kb; }
};

// ds_read_b128 services a wave in four 16-lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32).  Give each group exactly two items of 8 lanes so
// a group touches two 128-B rows (at most a 2-way bank conflict).
__device__ __forceinline__ void lane_item(int lane, int& item, int& q) {
  const int l = lane & 31, hi = (lane >> 5) * 4;
  if (l < 4) { item = 0; q = l; }
  else if (l < 12) { item = 2; q = l - 4; }
  else if (l < 16) { item = 0; q = l - 8; }
  else if (l < 20) { item = 3; q = l - 16; }
  else if (l < 28) { item = 1; q = l - 20; }
  else { item = 3; q = l - 24; }
  item += hi;
}

// ---------------------------------------------------------------------------
// Lane-per-position decode of a packed position (64 nibbles in 8 words) with
// SWAR nibble tests: the plan kernels touch every position once, so they
// decode 64 positions per wave instead of one.
struct LaneBoard {
  uint32_t w[8];
  uint64_t occ;
  int stm, wk, bk, cnt;
  int nwk, nbk;  // kings of each colour (an atomic game ends with one exploded)
  bool sane;     // valid piece codes, <= 32 pieces, stm 0 / 1 (kings not counted)
  bool ok;       // sane and one king per side
};

// Bit 4k+3 set iff nibble k of y is zero.
__device__ __forceinline__ uint32_t zero_nibbles(uint32_t y) {
  return ~(((y & 0x77777777u) + 0x77777777u) | y) & 0x88888888u;
}

// Compresses bits 3, 7, ..., 31 into an 8-bit mask.
__device__ __forceinline__ uint32_t nibble_bits(uint32_t z) {
  uint32_t m = z >> 3;
  m = (m | (m >> 3)) & 0x03030303u;
  m = (m | (m >> 6)) & 0x000F000Fu;
  return (m | (m >> 12)) & 0xFFu;
}

// kOcc = false: the occupancy mask is not built (occ = 0; cnt still counts).
template <bool kOcc = true>
__device__ __forceinline__ LaneBoard lane_decode(const fnnue_pos* p) {
  LaneBoard b;
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) b.w[i] = pw[i];
  b.stm = (int)(pw[8] & 0xFF);
  b.occ = 0;
  int nwk = 0, nbk = 0, cnt = 0;
  uint32_t bad = 0;
  b.wk = b.bk = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t w = b.w[i];
    const uint32_t occb = ~zero_nibbles(w) & 0x88888888u;  // bit 4k + 3: square 8i + k occupied
    if constexpr (kOcc) b.occ |= (uint64_t)nibble_bits(occb) << (8 * i);
    cnt += __popc(occb);
    const uint32_t kw = zero_nibbles(w ^ 0x66666666u), kb = zero_nibbles(w ^ 0xEEEEEEEEu);
    nwk += __popc(kw);
    nbk += __popc(kb);
    if (kw) b.wk = 8 * i + (__builtin_ctz(kw) >> 2);
    if (kb) b.bk = 8 * i + (__builtin_ctz(kb) >> 2);
    // no piece codes 7, 15 (type 7: low three bits set) or 8 (black, no type)
    bad |= (w & (w >> 1) & (w >> 2) & 0x11111111u) | zero_nibbles(w ^ 0x88888888u);
  }
  b.cnt = cnt;
  b.nwk = nwk;
  b.nbk = nbk;
  b.sane = !bad && b.cnt <= 32 && b.stm <= 1;
  b.ok = b.sane && nwk == 1 && nbk == 1;
  return b;
}

__device__ __forceinline__ int nibble_at(const uint32_t (&w)[8], int s) {
  const int i = s >> 3;
  const uint32_t a = (i & 1) ? w[1] : w[0], c = (i & 1) ? w[3] : w[2];
  const uint32_t e = (i & 1) ? w[5] : w[4], g = (i & 1) ? w[7] : w[6];
  const uint32_t lo = (i & 2) ? c : a, hi = (i & 2) ? g : e;
  return (int)((((i & 4) ? hi : lo) >> (4 * (s & 7))) & 15u);
}

// Segment items (ft_segments.hip) are binned by length: bin = L - 1 for
// L <= 16, then 8 lengths per bin up to 144, then one bin for longer runs.
__host__ __device__ constexpr uint32_t seg_len_bin(uint32_t L) {
  return L <= 16 ? L - 1 : L <= 144 ? 16 + (L - 17) / 8 : 32;
}
// Segment units: contiguous item ranges of one king block holding about
// kSegUnitPlies of work (items are sorted by length bin).  An item costs its
// root refresh plus one delta step per further position: the refresh sums the
// root's whole list (~25 rows, ~100 VALU per lane against ~27 for a delta
// position), so an item weighs kSegRootCost + the bin's longest length.
// Counting positions alone (kSegRootCost 0) made units of short segments
// (king moves, STAR children that move the king: one refresh each) up to 3-6x
// the work of the others (task timeline, tools/diag/seg_timeline.py,
// profiles/r04g); weighing the refresh (4) evens the tasks out (longest 152 ->
// 71 us on config 3): config 3 1163M -> 1179M, config 4 1115M -> 1164M
// (profiles/r04q; an earlier A/B that called it neutral compared two identical
// builds, see tools/exp_build.sh).
#ifndef SEG_UNIT_PLIES
#define SEG_UNIT_PLIES 20480
#endif
#ifndef SEG_UNIT_PLIES_SMALL
#define SEG_UNIT_PLIES_SMALL 8192
#endif
#ifndef SEG_ROOT_COST
#define SEG_ROOT_COST 4
#endif
constexpr uint32_t kSegUnitPlies = SEG_UNIT_PLIES;
// Nets of at most 4 column slices (HD <= 256) get units of half the work: 2
// slices per unit leave ~250 tasks for 256 CUs at 16384, one round whose span
// is its longest task (config 3 at HD 128: ft_segments 0.144 -> 0.094 ms).
// (Big nets: 20480 against 16384 / 12288: config 3 +0.9 % / -1.9 %, config
// 4 ±0 / -0.5 %, profiles/r04n.)
constexpr uint32_t kSegUnitPliesSmall = SEG_UNIT_PLIES_SMALL;
__host__ __device__ constexpr uint32_t seg_unit_plies_for(uint32_t hd) {
  return hd <= 256 ? kSegUnitPliesSmall : kSegUnitPlies;
}
constexpr uint32_t kSegRootCost = SEG_ROOT_COST;
__host__ __device__ constexpr uint32_t seg_bin_longest(uint32_t bin) {
  return bin < 16 ? bin + 1 : bin < 32 ? 8 * bin - 104 : 160;
}
__host__ __device__ constexpr uint32_t seg_bin_weight(uint32_t bin) { return seg_bin_longest(bin) + kSegRootCost; }

// Segment item bins per king block: 33 length bins x C classes of the root's
// list length, so that the items of a pass, which all sum the pass's longest
// list, have similar lengths (C = 4 for chess and atomic; 1 for crazyhouse,
// whose lists count the pockets too and are nearly all full).
template <int C>
__host__ __device__ constexpr uint32_t seg_count_class(uint32_t nfeat) {
  return C == 1 ? 0u : nfeat > 29 ? 3u : nfeat > 25 ? 2u : nfeat > 20 ? 1u : 0u;
}

// One workgroup of 1024 threads.  unit_items = 0: segment units (see
// seg_plies of work) instead of fixed-size ones.  KB king blocks (32: chess; 64:
// the variant feature sets), counters laid out as KB * NB item bins + 9
// position bins, then offsets, cursors and the unit count (kCnt / kOff / kCur
// / kNUnits for KB = 32, kV* for 64, SegCtr for segments).  NB = 33: bin =
// list length (fixed-size units); NB = 33 C: bin = C * length bin + class.
// The body runs in any 1024-thread workgroup (plan_scan_kernel_t, or a phase of
// the one-workgroup segment plan) on LDS the caller provides:
// plan_scan_lds_words<KB, NB>() words.
template <int KB, int NB>
__host__ __device__ constexpr int plan_scan_lds_words() {
  return (KB * NB + kPosBins) + 16 + KB * NB + KB + 1;
}
template <int KB, int NB = 33>
__device__ __forceinline__ void plan_scan_body(uint32_t* __restrict__ ctr, int4* __restrict__ units,
                                               uint32_t unit_items, uint32_t seg_plies, uint32_t* __restrict__ nu_out,
                                               uint32_t* __restrict__ lds) {
  constexpr int kIB = KB * NB, kB = kIB + kPosBins, kO = kB, kC = 2 * kB, kNU = 3 * kB;
  auto len_bin = [](int i) { return (i % NB) / (NB / 33); };
  uint32_t* s = lds;             // [kB]
  uint32_t* part = lds + kB;     // [16]
  const int t = threadIdx.x;
  // Exclusive scan of the item bins and, separately, of the position bins.
  constexpr int per = (kB + 1023) / 1024;
  uint32_t local[per];
  uint32_t sum = 0;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    local[k] = (i < kIB) ? ctr[i] : 0;
    sum += local[k];
  }
  // scan of the per-thread sums: inside each wave by shuffles, then over the
  // 16 wave totals (one barrier instead of two per step of a block scan)
  const int lane = t & 63, wv = t >> 6;
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) part[wv] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
  for (int w = 0; w < wv; ++w) run += part[w];
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i < kIB) s[i] = run;
    run += local[k];
  }
  if (t == 0) {
    uint32_t r = 0;
    for (int b = 0; b < kPosBins; ++b) {
      s[kIB + b] = r;
      r += ctr[kIB + b];
    }
  }
  __syncthreads();
  // nu_out: a second unit table over a plan already scattered (another net's
  // unit size): offsets and cursors stay as they are, the count goes to nu_out
  if (!nu_out)
    for (int i = t; i < kB; i += 1024) {
      ctr[kO + i] = s[i];
      ctr[kC + i] = s[i];
    }
  // end of king block kb's items
  auto kb_end = [&](int kb) -> uint32_t { return kb == KB - 1 ? s[KB * NB - 1] + ctr[KB * NB - 1] : s[(kb + 1) * NB]; };
  if (unit_items == 0) {
    // Segment units: unit u of king block kb starts at the first item whose
    // cumulative work (a bin's items weighed seg_bin_weight) reaches
    // u * seg_plies.  Bins are contiguous in item order, so each
    // (kb, bin) thread places the unit starts falling inside its bin.
    uint32_t* pb = lds + kB + 16;           // [kIB] positions before bin i within its king block
    uint32_t* ubase = lds + kB + 16 + kIB;  // [KB + 1] first unit of each king block
    for (int k = 0; k < per; ++k) {     // local[k] = count of bin t*per + k
      const int i = t * per + k;
      if (i < kIB) pb[i] = local[k] * seg_bin_weight(len_bin(i));
    }
    __syncthreads();
    if (t < KB) {
      uint32_t run = 0;
      for (int b = 0; b < NB; ++b) {
        const uint32_t v = pb[t * NB + b];
        pb[t * NB + b] = run;
        run += v;
      }
      const uint32_t mine = (run + seg_plies - 1) / seg_plies;
      uint32_t incl = mine;
#pragma unroll
      for (int o = 1; o < KB; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, KB);
        if (t >= o) incl += v;
      }
      ubase[t] = incl - mine;
      if (t == KB - 1) {
        ubase[KB] = incl;
        if (nu_out) *nu_out = incl;
        else ctr[kNU] = incl;
      }
    }
    __syncthreads();
    for (int k = 0; k < per; ++k) {
      const int i = t * per + k;
      if (i >= kIB || local[k] == 0) continue;
      const int kb = i / NB;
      const uint32_t w = seg_bin_weight(len_bin(i)), p0 = pb[i], p1 = p0 + local[k] * w;
      for (uint32_t u = (p0 + seg_plies - 1) / seg_plies; u * seg_plies < p1; ++u)
        units[ubase[kb] + u] = make_int4(kb, (int)(s[i] + (u * seg_plies - p0 + w - 1) / w), 0, 0);
    }
    __syncthreads();  // the starts are visible to the whole workgroup
    // Ends: the next unit's start, or the block's end.  Only .z is written
    // here, so reading a neighbour's .y does not race.  (Unit 0 of a block
    // starts at its first non-empty bin's offset, i.e. the block's first item.)
    for (uint32_t v = t; v < ubase[KB]; v += 1024) {
      const int kb = units[v].x;
      units[v].z = v + 1 < ubase[kb + 1] ? units[v + 1].y : (int)kb_end(kb);
    }
  } else if (t < KB) {
    // Unit table: each king block's item range in chunks of <= unit_items;
    // lane kb counts its block's units, a wave prefix sum places them.
    const int kb = t;
    const uint32_t b = s[kb * NB];
    const uint32_t e = kb_end(kb);
    const uint32_t mine = (e - b + unit_items - 1) / unit_items;
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < KB; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, KB);
      if (kb >= o) incl += v;
    }
    uint32_t nu = incl - mine;
    for (uint32_t c = b; c < e; c += unit_items) units[nu++] = make_int4(kb, (int)c, (int)min(e, c + unit_items), 0);
    if (kb == KB - 1) ctr[kNU] = incl;
  }
}

template <int KB, int NB = 33>
__global__ __launch_bounds__(1024) __attribute__((unused)) void plan_scan_kernel_t(uint32_t* __restrict__ ctr,
                                                                                  int4* __restrict__ units,
                                                                                  uint32_t unit_items,
                                                                                  uint32_t seg_plies = 0,
                                                                                  uint32_t* __restrict__ nu_out = nullptr) {
  __shared__ uint32_t lds[plan_scan_lds_words<KB, NB>()];
  plan_scan_body<KB, NB>(ctr, units, unit_items, seg_plies, nu_out, lds);
}

constexpr int kListStrideWords = 17;  // words per lane of the list staging rows (68 B)

// Plane of piece code pc (0..15) seen from perspective p, one nibble per pc:
// 2 * (type - 1) + (colour != p), both kings plane 10 (upstream
// half_ka_v2_hm.h PieceSquareIndex / 64).
__host__ __device__ constexpr uint64_t plane_table(int persp) {
  uint64_t t = 0;
  for (int pc = 1; pc < 16; ++pc) {
    const int type = pc & 7;
    if (type < 1 || type > 6) continue;
    const int plane = type == 6 ? 10 : 2 * (type - 1) + ((pc >> 3) != persp);
    t |= (uint64_t)plane << (4 * pc);
  }
  return t;
}

// Writes item `it`'s 32 feature-list entries (rows relative to its king block,
// padded with the zero row): every piece except the perspective's own king,
// whose row is the same for the whole king block (king_row) and is added to
// the bias once per workgroup instead of once per item.  ft_slices pairs items 2k and 2k+1 of a pass on
// one ds_read_b128 lane group; a 128-B tile row r lies in bank half r & 1, so
// even-position items list their even rows first and odd-position items their
// odd rows first: the pair then mostly reads opposite bank halves.  A row's
// parity is (square ^ mirror) & 1 (orient() flips files when the king is on
// files a-d), and the sum is order-independent.
// The entries are gathered in the thread's own LDS row (`mine`,
// kListStrideWords words: the rows of a wave start in 32 different banks),
// pre-filled with the zero row, then one u16 store per piece at its slot
// (first-parity pieces from 0, the others from the count of the first), and
// read back as words.  The pieces are walked rank by rank straight from the
// packed nibbles (word i = squares 8i..8i+7, nibble j = square 8i+j): the
// square, piece code and plane come from the bit position and a 64-bit plane
// table instead of a 64-bit scan plus an 8-way word select per piece
// (38 -> 18 VALU per piece).
// pp = the item's parity within its king block's items, (it - first item of
// the block) & 1.
__device__ __forceinline__ void write_rows(const LaneBoard& b, int persp, int ksq, uint32_t it, uint32_t pp,
                                               uint32_t* __restrict__ mine, uint16_t* __restrict__ flist) {
  const uint32_t mirror = (ksq & 7) < 4 ? 1u : 0u;
  const uint32_t flip = (persp ? 56u : 0u) ^ (mirror ? 7u : 0u);
  const uint64_t ptab = persp ? plane_table(1) : plane_table(0);
  constexpr uint64_t kEvenFiles = 0x5555555555555555ull;
  const uint32_t fpar = pp ^ mirror;  // square parity listed first
  const uint64_t occ = b.occ & ~(1ull << ksq);
  uint32_t kf = 0, ks = (uint32_t)__popcll(occ & (fpar ? ~kEvenFiles : kEvenFiles));
  // the row is written as u16 and as words: may_alias types keep the
  // compiler from reordering (or dropping) one kind against the other
  typedef uint16_t u16_alias __attribute__((__may_alias__));
  typedef uint32_t u32_alias __attribute__((__may_alias__));
  u32_alias* M = reinterpret_cast<u32_alias*>(mine);
  u16_alias* L = reinterpret_cast<u16_alias*>(mine);
#pragma unroll
  for (int j = 0; j < 16; ++j) M[j] = kNoEntry | kNoEntry << 16;
  const uint32_t kw = (uint32_t)ksq >> 3, kbit = 1u << (4 * (ksq & 7));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t w = b.w[i];
    uint32_t nz = ((((w & 0x77777777u) + 0x77777777u) | w) >> 3) & 0x11111111u;  // bit 4j: square 8i+j occupied
    nz &= kw == (uint32_t)i ? ~kbit : ~0u;
    const uint32_t c16 = ((8u * (uint32_t)i) ^ flip) << 4;
    while (nz) {
      const uint32_t bit = (uint32_t)__builtin_ctz(nz);  // 4j
      nz &= nz - 1;
      const uint32_t plane = (uint32_t)(ptab >> (((w >> bit) & 15u) << 2)) & 15u;
      const uint32_t e = ((bit << 2) ^ c16) + (plane << 10);  // 16 * ((8i + j) ^ flip) + 1024 * plane
      const bool f = ((bit >> 2) & 1u) == fpar;
      L[f ? kf : ks] = (uint16_t)e;
      kf += f ? 1u : 0u;
      ks += f ? 0u : 1u;
    }
  }
  uint4* dst = reinterpret_cast<uint4*>(flist + (size_t)it * 32);
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[q] = make_uint4(M[4 * q], M[4 * q + 1], M[4 * q + 2], M[4 * q + 3]);
}

// Number of 16-byte entries of the tile image: 32 king blocks x hd/64 slices
// x 705 rows x 8 entries per row.  Single source of truth for the allocation
// (sliced_tiles_bytes) and the relayout kernel's extent.
__host__ __device__ constexpr size_t tile_uint4_count(uint32_t hd) { return (size_t)32 * (hd / 64) * kTileU4; }

// ---------------------------------------------------------------------------
// Tile image: tile(kb, s)[q][r] (16 B) = {ft_w[kb*R+r][32s+4q .. +3],
// ft_w[kb*R+r][HD/2+32s+4q .. +3]}; rows r >= R (the zero rows) are zero.
template <int HD, class G = ChessGeom>
__global__ __launch_bounds__(256) void relayout_kernel(const int16_t* __restrict__ ftw, uint4* __restrict__ tiles) {
  constexpr int S = HD / 64;
  constexpr size_t total = (size_t)G::kBlocks * S * G::kTileU4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i % G::kPlaneU4);
    const size_t t = i / G::kPlaneU4;
    const int q = (int)(t & 7);
    const size_t ks = t >> 3;
    const int s = (int)(ks % S), kb = (int)(ks / S);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < G::kRows) {
      const int16_t* row = ftw + (size_t)(kb * G::kRows + r) * HD;
      const uint2 lo = *reinterpret_cast<const uint2*>(row + 32 * s + 4 * q);
      const uint2 hi = *reinterpret_cast<const uint2*>(row + HD / 2 + 32 * s + 4 * q);
      v = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
    tiles[i] = v;
  }
}

// Raw buffer resources: num_records = 2^31 - 1 bytes, so any offset >= 2^31
// fails the bounds check and the store is dropped.  Word 3 = the gfx9-family
// raw-buffer format (32-bit data format, no swizzle).
constexpr int kBufferRange = 0x7FFFFFFF;
constexpr int kBufferFlags = 0x00020000;
constexpr int kBufferAll = -1;  // num_records = 2^32 - 1: no bounds check in practice
constexpr uint32_t kDroppedOffset = 0x80000000u;

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// out byte k = (clamp(lo_k, 0, 127) * clamp(hi_k, 0, 127)) >> 7 (upstream
// transform).  The doubled product (< 2^15) holds that value in its high byte,
// so one v_perm_b32 packs the four bytes.
__device__ __forceinline__ uint32_t transform4(u16x4 lo, u16x4 hi) {
  const s16x4 zero = (s16x4)0, top = (s16x4)127;
  const s16x4 a = __builtin_elementwise_min(__builtin_elementwise_max((s16x4)lo, zero), top);
  const s16x4 b = __builtin_elementwise_min(__builtin_elementwise_max((s16x4)hi, zero), top);
  const u16x4 pr = ((u16x4)a * (u16x4)b) << (u16x4)1;
  const u32x2 w = __builtin_bit_cast(u32x2, pr);
  return __builtin_amdgcn_perm(w.y, w.x, 0x07050301u);
}

// One pass's fetch from HBM/L2: this lane's item record, and 8 bytes of the
// pass's feature lists (lane l: entries 4(l&7) .. +3 of pass item l>>3), so
// each list byte is fetched once per slice; the lists are then spread to the
// 8 lanes of each item through a per-wave LDS buffer.  Indices are clamped into
// the unit so the loads are unconditional (hipcc then counts vmcnt instead of
// draining it); a clamped lane repeats the unit's last item.
struct PassFetch {
  uint32_t rec;
  uint2 lst;
};
__device__ __forceinline__ PassFetch fetch_pass(__amdgpu_buffer_rsrc_t items, __amdgpu_buffer_rsrc_t flist,
                                                int pass_base, int last, int lane, int it_in_wave) {
  PassFetch f;
  f.rec = __builtin_amdgcn_raw_buffer_load_b32(items, (uint32_t)min(pass_base + it_in_wave, last) * 4u, 0, 0);
  const uint32_t li = (uint32_t)min(pass_base + (lane >> 3), last);
  const u32x2 l = __builtin_amdgcn_raw_buffer_load_b64(flist, li * 64u + 8u * (uint32_t)(lane & 7), 0, 0);
  f.lst = make_uint2(l.x, l.y);
  return f;
}

// LDS byte address of this lane's chunk of the row named by the low / high u16
// entry of `word`: base (= plane q) + entry; hipcc emits one v_add_u32_sdwa.
__device__ __forceinline__ const u32x4* row_addr(const char* base, uint32_t word, int t) {
  const uint32_t entry = (t & 1) ? (word >> 16) : (word & 0xFFFFu);
  return static_cast<const u32x4*>(__builtin_assume_aligned(base + entry, 16));
}

#ifndef FT_DEPTH
#define FT_DEPTH 2
#endif
// Rows in flight per wave: the LDS queue stays fed and hipcc counts lgkmcnt
// instead of draining it (2 against 3: config 2 +0.2 %, config 3 +0.5 %;
// 4: -0.4 % / -5 %, profiles/r04n).
constexpr int kRowDepth = 4 * FT_DEPTH;

// SWAR rows (ft_slices when the net allows it, accumulator_bound in net.h):
// a 32-bit word holding the int16 columns (c, c+1) as l + 65536 * h with l
// SIGNED, so that 32-bit adds of such words sum both columns at once (one VOP2
// v_add_u32 per word instead of a VOP3P v_pk_add_u16, which issues at ~1.75x
// its cost).  The sum is exact mod 2^32; while the true sum of column c stays
// within int16 range its low half is that sum and the high half, after the
// low half's sign is taken back out (transform4_swar), is column c+1's sum
// mod 2^16 — the int16 wraparound of upstream's accumulator.
__device__ __forceinline__ uint32_t swar_word(uint32_t packed) { return packed - ((packed & 0x8000u) << 1); }
__device__ __forceinline__ u16x4 swar_words(u16x4 v) {
  const u32x2 w = __builtin_bit_cast(u32x2, v);
  return __builtin_bit_cast(u16x4, u32x2{swar_word(w.x), swar_word(w.y)});
}

// Transform straight from SWAR words.  The accumulator starts at the bias plus
// kSwarOffset (0x80008000 per word): a word w = l + 65536 h (l signed, the
// exact low column; h the high column mod 2^16) then holds l + 0x8000 in its
// low half (the 0x8000 carries out of the low half exactly when l < 0,
// restoring the borrow a negative l took from the high half) and h + 0x8000
// in its high half, both mod 2^16.  A saturating u16 subtract of 0x8000 is
// max(column, 0) on both halves at once, so no unpacking is needed.
//
// The second half's columns (the `hi` words, columns HD/2..HD-1) are kept
// DOUBLED in the tile and the bias (swar_word_hi): hi - 0x8000 saturated is
// max(2 col, 0), its min with 254 is 2 clamp(col, 0, 127), and a * that is
// already (a b) << 1, whose high byte is SF's (a b) >> 7 — one shift per pair
// fewer.  Exact while every reachable second-half column stays below 2^14 in
// magnitude (accumulator_bound counts it twice, net.cpp).
constexpr uint32_t kSwarOffset = 0x80008000u;
__device__ __forceinline__ uint32_t swar_word_hi(uint32_t packed) {
  return swar_word((packed << 1) & 0xFFFEFFFEu);
}
__device__ __forceinline__ u16x4 swar_words_hi(u16x4 v) {
  const u32x2 w = __builtin_bit_cast(u32x2, v);
  return __builtin_bit_cast(u16x4, u32x2{swar_word_hi(w.x), swar_word_hi(w.y)});
}
__device__ __forceinline__ uint4 swar_tile_words(uint4 v) {  // 16 B of a tile row: 4 lo columns, 4 hi columns
  return make_uint4(swar_word(v.x), swar_word(v.y), swar_word_hi(v.z), swar_word_hi(v.w));
}
__device__ __forceinline__ uint32_t transform4_swar(u16x4 lo, u16x4 hi) {
  const u16x4 off = (u16x4)0x8000, top = (u16x4)127, top2 = (u16x4)254;
  const u16x4 a = __builtin_elementwise_min(__builtin_elementwise_sub_sat(lo, off), top);
  const u16x4 b2 = __builtin_elementwise_min(__builtin_elementwise_sub_sat(hi, off), top2);
  const u32x2 w = __builtin_bit_cast(u32x2, a * b2);
  return __builtin_amdgcn_perm(w.y, w.x, 0x07050301u);
}

template <bool kSwar = false>
__device__ __forceinline__ void accum_row(const u32x4& v, u16x4& lo, u16x4& hi) {
  const u32x2 a = __builtin_shufflevector(v, v, 0, 1);
  const u32x2 b = __builtin_shufflevector(v, v, 2, 3);
  if constexpr (kSwar) {
    lo = __builtin_bit_cast(u16x4, __builtin_bit_cast(u32x2, lo) + a);
    hi = __builtin_bit_cast(u16x4, __builtin_bit_cast(u32x2, hi) + b);
  } else {
    lo += __builtin_bit_cast(u16x4, a);
    hi += __builtin_bit_cast(u16x4, b);
  }
}

template <int NR, int R = 0>
__device__ __forceinline__ void rows1_head(const uint32_t (&e)[16], const char* base, u32x4 (&v)[kRowDepth]) {
  if constexpr (R < NR && R < kRowDepth) {
    v[R] = *row_addr(base, e[R >> 1], R & 1);
    rows1_head<NR, R + 1>(e, base, v);
  }
}

template <int NR, bool kSwar, int R = 0>
__device__ __forceinline__ void rows1_step(const uint32_t (&e)[16], const char* base, u32x4 (&v)[kRowDepth],
                                           u16x4& lo, u16x4& hi) {
  if constexpr (R < NR) {
    accum_row<kSwar>(v[R % kRowDepth], lo, hi);
    if constexpr (R + kRowDepth < NR) v[R % kRowDepth] = *row_addr(base, e[(R + kRowDepth) >> 1], (R + kRowDepth) & 1);
    rows1_step<NR, kSwar, R + 1>(e, base, v, lo, hi);
  }
}

// Exactly NR rows (a pass's longest list, not rounded up: rounding to groups of
// 4 cost 7 % padding rows, 2 % of the kernel), kRowDepth rows in flight,
// branch-free straight-line code per row count.
template <int NR, bool kSwar>
__device__ __forceinline__ void rows_exact(const uint32_t (&e)[16], const char* base, u16x4& lo, u16x4& hi) {
  u32x4 v[kRowDepth];
  rows1_head<NR>(e, base, v);
  rows1_step<NR, kSwar>(e, base, v, lo, hi);
}

// Sums the first `nrows` (wave-uniform, <= 32) rows of the feature list e
// (kSwar: rows and accumulator in SWAR words, see swar_word).
template <bool kSwar = false>
__device__ __forceinline__ void rows_sum(int nrows, const uint32_t (&e)[16], const char* base, u16x4& lo, u16x4& hi) {
  switch (nrows) {
#define FNNUE_ROWS_CASE(k) \
  case k: rows_exact<k, kSwar>(e, base, lo, hi); break;
    FNNUE_ROWS_CASE(1) FNNUE_ROWS_CASE(2) FNNUE_ROWS_CASE(3) FNNUE_ROWS_CASE(4) FNNUE_ROWS_CASE(5)
    FNNUE_ROWS_CASE(6) FNNUE_ROWS_CASE(7) FNNUE_ROWS_CASE(8) FNNUE_ROWS_CASE(9) FNNUE_ROWS_CASE(10)
    FNNUE_ROWS_CASE(11) FNNUE_ROWS_CASE(12) FNNUE_ROWS_CASE(13) FNNUE_ROWS_CASE(14) FNNUE_ROWS_CASE(15)
    FNNUE_ROWS_CASE(16) FNNUE_ROWS_CASE(17) FNNUE_ROWS_CASE(18) FNNUE_ROWS_CASE(19) FNNUE_ROWS_CASE(20)
    FNNUE_ROWS_CASE(21) FNNUE_ROWS_CASE(22) FNNUE_ROWS_CASE(23) FNNUE_ROWS_CASE(24) FNNUE_ROWS_CASE(25)
    FNNUE_ROWS_CASE(26) FNNUE_ROWS_CASE(27) FNNUE_ROWS_CASE(28) FNNUE_ROWS_CASE(29) FNNUE_ROWS_CASE(30)
    FNNUE_ROWS_CASE(31) FNNUE_ROWS_CASE(32)
#undef FNNUE_ROWS_CASE
    default: break;
  }
}

}  // namespace
}  // namespace fnnue
