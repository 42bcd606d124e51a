// ft_sliced.hip — LDS-stationary feature transformer for batches of
// independent positions (BASELINE config 2, "from scratch").
//
// Why: a position's two accumulators need 2n rows of 2 KiB gathered from a
// 46 MB table (HD = 1024).  Gathered per position (ft_scratch_kernel) the rows
// come from L2 (~72 % hits) and the Infinity Cache at ~22 TB/s.  Here the
// table is instead split into (king block kb, slice s) tiles of 705 rows x
// 128 B (64 of the HD int16 columns: 32 from each half, so the pairwise
// product stays inside a tile); one 1024-thread workgroup holds one tile in
// LDS (90 KB of the CU's 160 KB) and streams every perspective-item whose
// king block is kb through it, reading rows with ds_read_b128.  HBM/L2 then
// see only the compact plan (feature lists) and the transformed output.
//
// Pipeline per chunk of positions (all on the caller's stream, no host sync):
//   plan_count    per-workgroup LDS histograms of item keys (kb, n) and of
//                 position buckets -> global counts
//   plan_scan     one workgroup: exclusive scans -> item / slot offsets, and
//                 the unit table (kb, item range of <= kUnitItems)
//   plan_scatter  counting-sort scatter: per item its 32 feature rows (u16,
//                 relative to kb, padded with the zero row) and its output
//                 slot; positions re-ordered by layer-stack bucket; PSQT term
//   ft_slices     (unit, slice) workgroups, XCD-aware: all slices of a unit
//                 run on one XCD so the unit's feature lists are read once
//                 into that XCD's L2
// then stack_kernel (kernels.hip) over the bucket-sorted slots.
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

// Counter block layout (uint32 words).
constexpr int kCnt = 0, kOff = kBins, kCur = 2 * kBins, kNUnits = 3 * kBins;

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
  bool ok;
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

__device__ __forceinline__ LaneBoard lane_decode(const fnnue_pos* p) {
  LaneBoard b;
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) b.w[i] = pw[i];
  b.stm = (int)(pw[8] & 0xFF);
  b.occ = 0;
  int nwk = 0, nbk = 0;
  uint32_t bad = 0;
  b.wk = b.bk = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t w = b.w[i];
    b.occ |= (uint64_t)nibble_bits(~zero_nibbles(w) & 0x88888888u) << (8 * i);
    const uint32_t kw = zero_nibbles(w ^ 0x66666666u), kb = zero_nibbles(w ^ 0xEEEEEEEEu);
    nwk += __popc(kw);
    nbk += __popc(kb);
    if (kw) b.wk = 8 * i + (__builtin_ctz(kw) >> 2);
    if (kb) b.bk = 8 * i + (__builtin_ctz(kb) >> 2);
    bad |= zero_nibbles(w ^ 0x77777777u) | zero_nibbles(w ^ 0x88888888u) | zero_nibbles(~w);
  }
  b.cnt = __popcll(b.occ);
  b.ok = !bad && nwk == 1 && nbk == 1 && b.cnt <= 32 && b.stm <= 1;
  return b;
}

__device__ __forceinline__ int nibble_at(const uint32_t (&w)[8], int s) {
  const int i = s >> 3;
  const uint32_t a = (i & 1) ? w[1] : w[0], c = (i & 1) ? w[3] : w[2];
  const uint32_t e = (i & 1) ? w[5] : w[4], g = (i & 1) ? w[7] : w[6];
  const uint32_t lo = (i & 2) ? c : a, hi = (i & 2) ? g : e;
  return (int)((((i & 4) ? hi : lo) >> (4 * (s & 7))) & 15u);
}

__global__ __launch_bounds__(1024) void plan_count_kernel(const fnnue_pos* __restrict__ pos, uint32_t n,
                                                         uint32_t* __restrict__ ctr, uint32_t* __restrict__ err) {
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    const LaneBoard b = lane_decode(pos + p);
    if (!b.ok) {
      bad = 1;
      atomicAdd(&h[kItemBins + 8], 1u);
    } else {
      atomicAdd(&h[king_block(0, b.wk) * 33 + b.cnt], 1u);
      atomicAdd(&h[king_block(1, b.bk) * 33 + b.cnt], 1u);
      atomicAdd(&h[kItemBins + ((b.cnt - 1) >> 2)], 1u);
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(err, 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += blockDim.x)
    if (h[i]) atomicAdd(&ctr[kCnt + i], h[i]);
}

// One workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void plan_scan_kernel(uint32_t* __restrict__ ctr, int4* __restrict__ units,
                                                         uint32_t unit_items) {
  __shared__ uint32_t s[kBins];
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  // Exclusive scan of the item bins and, separately, of the position bins.
  constexpr int per = (kBins + 1023) / 1024;
  uint32_t local[per];
  uint32_t sum = 0;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    local[k] = (i < kItemBins) ? ctr[kCnt + i] : 0;
    sum += local[k];
  }
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i < kItemBins) s[i] = run;
    run += local[k];
  }
  if (t == 0) {
    uint32_t r = 0;
    for (int b = 0; b < kPosBins; ++b) {
      s[kItemBins + b] = r;
      r += ctr[kCnt + kItemBins + b];
    }
  }
  __syncthreads();
  for (int i = t; i < kBins; i += 1024) {
    ctr[kOff + i] = s[i];
    ctr[kCur + i] = s[i];
  }
  if (t < 32) {
    // Unit table: each king block's item range in chunks of <= unit_items;
    // lane kb counts its block's units, a wave prefix sum places them.
    const int kb = t;
    const uint32_t b = s[kb * 33];
    const uint32_t e = kb == 31 ? s[31 * 33 + 32] + ctr[kCnt + 31 * 33 + 32] : s[(kb + 1) * 33];
    const uint32_t mine = (e - b + unit_items - 1) / unit_items;
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 32);
      if (kb >= o) incl += v;
    }
    uint32_t nu = incl - mine;
    for (uint32_t c = b; c < e; c += unit_items) units[nu++] = make_int4(kb, (int)c, (int)min(e, c + unit_items), 0);
    if (kb == 31) ctr[kNUnits] = incl;
  }
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
__device__ __forceinline__ void write_rows(const LaneBoard& b, int persp, int ksq, uint32_t it,
                                           const uint32_t* __restrict__ ctr, uint16_t* __restrict__ flist) {
  const int kbc = king_block(persp, ksq);
  const uint32_t pp = (it - ctr[kOff + kbc * 33]) & 1;
  const uint32_t mirror = (ksq & 7) < 4 ? 1u : 0u;
  constexpr uint64_t kEvenFiles = 0x5555555555555555ull;
  const uint64_t occ = b.occ & ~(1ull << ksq);  // own king: folded into the bias (king_row)
  uint64_t first = occ & ((pp ^ mirror) ? ~kEvenFiles : kEvenFiles);
  uint64_t second = occ & ~first;
  uint32_t E[16];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    uint32_t a = kNoEntry;
    if (first | second) {
      uint64_t& m = first ? first : second;
      const int sq = __builtin_ctzll(m);
      m &= m - 1;
      a = 16u * (uint32_t)(make_index(persp, sq, nibble_at(b.w, sq), ksq) - kRowsPerBlock * kbc);
    }
    if (k & 1) E[k >> 1] |= a << 16;
    else E[k >> 1] = a;
  }
  uint4* dst = reinterpret_cast<uint4*>(flist + (size_t)it * 32);
#pragma unroll
  for (int k = 0; k < 4; ++k) dst[k] = make_uint4(E[4 * k], E[4 * k + 1], E[4 * k + 2], E[4 * k + 3]);
}

// Item record: (n << 24) | (slot << 1) | half, half 0 = side-to-move half of x.
// One lane per position; the workgroup's 256 positions get local ranks from
// LDS atomics, then reserve one range per bin with a single global atomic.
__global__ __launch_bounds__(kScatterPositions) void plan_scatter_kernel(const fnnue_pos* __restrict__ pos, uint32_t n,
                                                           uint32_t* __restrict__ ctr, uint32_t* __restrict__ items,
                                                           uint16_t* __restrict__ flist, uint32_t* __restrict__ perm,
                                                           uint8_t* __restrict__ bucket_out,
                                                           int32_t* __restrict__ psqt_out) {
  __shared__ uint32_t lcnt[kBins];
  __shared__ uint32_t lbase[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) lcnt[i] = 0;
  __syncthreads();
  const uint32_t p = blockIdx.x * kScatterPositions + threadIdx.x;
  const bool live = p < n;
  LaneBoard b;
  int kw = 0, kb = 0, kp = kItemBins + 8;
  uint32_t rw = 0, rb = 0, rp = 0;
  if (live) {
    b = lane_decode(pos + p);
    if (b.ok) {
      kw = king_block(0, b.wk) * 33 + b.cnt;
      kb = king_block(1, b.bk) * 33 + b.cnt;
      kp = kItemBins + ((b.cnt - 1) >> 2);
      rw = atomicAdd(&lcnt[kw], 1u);
      rb = atomicAdd(&lcnt[kb], 1u);
    }
    rp = atomicAdd(&lcnt[kp], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += blockDim.x)
#ifdef FT_EXP_NO_ATOMIC
    lbase[i] = lcnt[i] ? ctr[kOff + i] + (blockIdx.x * 7u) % 64u : 0;
#else
    lbase[i] = lcnt[i] ? atomicAdd(&ctr[kCur + i], lcnt[i]) : 0;
#endif
  __syncthreads();
  if (!live) return;
  const uint32_t slot = lbase[kp] + rp;
  perm[slot] = p;
  if (!b.ok) {
    bucket_out[slot] = 0xFF;
    psqt_out[p] = 0;
    return;
  }
  const int bucket = (b.cnt - 1) >> 2;
  const uint32_t iw = lbase[kw] + rw, ib = lbase[kb] + rb;
#ifndef FT_EXP_NO_ROWS_WRITE
  write_rows(b, 0, b.wk, iw, ctr, flist);
  write_rows(b, 1, b.bk, ib, ctr, flist);
#endif
  items[iw] = ((uint32_t)b.cnt << 24) | (slot << 1) | (uint32_t)(b.stm != 0);
  items[ib] = ((uint32_t)b.cnt << 24) | (slot << 1) | (uint32_t)(b.stm != 1);
  bucket_out[slot] = (uint8_t)bucket;
  // the PSQT term is summed from LDS by the slice-0 workgroups of ft_slices
}

// Number of 16-byte entries of the tile image: 32 king blocks x hd/64 slices
// x 705 rows x 8 entries per row.  Single source of truth for the allocation
// (sliced_tiles_bytes) and the relayout kernel's extent.
__host__ __device__ constexpr size_t tile_uint4_count(uint32_t hd) { return (size_t)32 * (hd / 64) * kTileU4; }

// ---------------------------------------------------------------------------
// Tile image: tile(kb, s)[q][r] (16 B) = {ft_w[kb*704+r][32s+4q .. +3],
// ft_w[kb*704+r][HD/2+32s+4q .. +3]}; r = 704 is the zero row, r = 705 padding.
template <int HD>
__global__ __launch_bounds__(256) void relayout_kernel(const int16_t* __restrict__ ftw, uint4* __restrict__ tiles) {
  constexpr int S = HD / 64;
  constexpr size_t total = tile_uint4_count(HD);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i % kPlaneU4);
    const size_t t = i / kPlaneU4;
    const int q = (int)(t & 7);
    const size_t ks = t >> 3;
    const int s = (int)(ks % S), kb = (int)(ks / S);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < kRowsPerBlock) {
      const int16_t* row = ftw + (size_t)(kb * kRowsPerBlock + r) * HD;
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
#ifdef FT_EXP_NO_LIST
  f.lst = make_uint2(f.rec & 0x70, f.rec & 0x30);
#else
  const u32x2 l = __builtin_amdgcn_raw_buffer_load_b64(flist, li * 64u + 8u * (uint32_t)(lane & 7), 0, 0);
  f.lst = make_uint2(l.x, l.y);
#endif
  return f;
}

// Reads the LDS tile rows of feature-list entries 4G .. 4G+3 (each lane its
// 16-byte chunk q of the row).

// LDS byte address of this lane's chunk of the row named by the low / high u16
// entry of `word`: base (= plane q) + entry; hipcc emits one v_add_u32_sdwa.
__device__ __forceinline__ const u32x4* row_addr(const char* base, uint32_t word, int t) {
  const uint32_t entry = (t & 1) ? (word >> 16) : (word & 0xFFFFu);
  return static_cast<const u32x4*>(__builtin_assume_aligned(base + entry, 16));
}

template <int G>
__device__ __forceinline__ void issue_rows(const uint32_t (&e)[16], const char* base, u32x4 (&v)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    v[t] = *row_addr(base, e[2 * G + (t >> 1)], t);
#ifdef FT_EXP_DUPREAD
    const u32x4 extra = *(row_addr(base, e[2 * G + (t >> 1)], t) + 1);
    uint32_t sink;
    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(sink) : "v"(extra.x), "v"(extra.y));
#endif
  }
}

__device__ __forceinline__ void accum_rows(const u32x4 (&v)[4], u16x4& lo, u16x4& hi) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    // Swizzles go through named temporaries: __builtin_bit_cast of a swizzle
    // lvalue (v.zw) reads from the vector's base address in this clang.
    const u32x2 a = __builtin_shufflevector(v[t], v[t], 0, 1);
    const u32x2 b = __builtin_shufflevector(v[t], v[t], 2, 3);
    lo += __builtin_bit_cast(u16x4, a);
#ifdef FT_EXP_EXTRAVALU
    {
      uint32_t sink;
      asm volatile("v_xor_b32 %0, %1, %2" : "=v"(sink) : "v"(a.x), "v"(b.y));
    }
#endif
#ifdef FT_EXP_DUPADD
    {
      uint32_t s0, s1, s2, s3;
      asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(s0) : "v"(a.x), "v"(a.y));
      asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(s1) : "v"(a.y), "v"(b.x));
      asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(s2) : "v"(b.x), "v"(b.y));
      asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(s3) : "v"(b.y), "v"(a.x));
    }
#endif
#ifndef FT_EXP_LO_ONLY
    hi += __builtin_bit_cast(u16x4, b);
#endif
  }
}

#ifndef FT_DEPTH
#define FT_DEPTH 3
#endif
constexpr int kDepth = FT_DEPTH;  // row groups (of 4) in flight per wave

// NG groups of 4 rows, kDepth groups in flight, no branches: the LDS queue
// stays fed and hipcc can count lgkmcnt instead of draining it.
template <int NG, int G = 0>
__device__ __forceinline__ void rows_step(const uint32_t (&e)[16], const char* base, u32x4 (&v)[kDepth][4],
                                          u16x4& lo, u16x4& hi) {
  if constexpr (G < NG) {
    accum_rows(v[G % kDepth], lo, hi);
    if constexpr (G + kDepth < NG) issue_rows<G + kDepth>(e, base, v[G % kDepth]);
    rows_step<NG, G + 1>(e, base, v, lo, hi);
  }
}

template <int NG, int G = 0>
__device__ __forceinline__ void rows_issue_head(const uint32_t (&e)[16], const char* base, u32x4 (&v)[kDepth][4]) {
  if constexpr (G < NG && G < kDepth) {
    issue_rows<G>(e, base, v[G]);
    rows_issue_head<NG, G + 1>(e, base, v);
  }
}

template <int NG>
__device__ __forceinline__ void rows_pipelined(const uint32_t (&e)[16], const char* base, u16x4& lo, u16x4& hi) {
#ifndef FT_EXP_NO_ROWS
  u32x4 v[kDepth][4];
  rows_issue_head<NG>(e, base, v);
  rows_step<NG>(e, base, v, lo, hi);
#endif
}

// One pass (8 items per wave) over the LDS tile: the lists go to the wave's
// LDS buffer, bias + rows, transform, store; in slice 0 also the PSQT part.
// maxn = the pass's longest list.  Both stores are unconditional: a lane past
// the end of the unit holds the clamped last item and rewrites its identical
// values, and slices != 0 issue their PSQT store out of the buffer's bounds
// (dropped by the hardware).  A store skipped on some path would make hipcc's
// vmcnt bookkeeping wait for every store before the next pass's rows.
template <int HD>
__device__ __forceinline__ void slice_pass(const PassFetch& f, uint2* __restrict__ lb, int lane, int it_in_wave, int s,
                                           int q, const char* base, u16x4 b_lo, u16x4 b_hi, int krow,
                                           const int32_t* ptile, __amdgpu_buffer_rsrc_t psqt_rsrc,
                                           __amdgpu_buffer_rsrc_t x_rsrc) {
  constexpr int kLastItemLane = 48;  // lane_item: lane 48 holds pass item 7, the longest list
  const uint32_t rec = f.rec;
  const int maxn = (int)(__builtin_amdgcn_readlane(rec, kLastItemLane) >> 24);
  // LDS ops of one wave complete in order: this write lands after the previous
  // pass's reads of lb and before this pass's reads.
  lb[lane] = f.lst;
  uint32_t e[16];
  const uint4* my = reinterpret_cast<const uint4*>(lb) + 4 * it_in_wave;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint4 v = my[m];
    e[4 * m] = v.x;
    e[4 * m + 1] = v.y;
    e[4 * m + 2] = v.z;
    e[4 * m + 3] = v.w;
  }
  u16x4 lo = b_lo, hi = b_hi;
  switch ((maxn + 2) >> 2) {  // maxn - 1 rows (own king in the bias); wave-uniform, straight-line cases
    case 1: rows_pipelined<1>(e, base, lo, hi); break;
    case 2: rows_pipelined<2>(e, base, lo, hi); break;
    case 3: rows_pipelined<3>(e, base, lo, hi); break;
    case 4: rows_pipelined<4>(e, base, lo, hi); break;
    case 5: rows_pipelined<5>(e, base, lo, hi); break;
    case 6: rows_pipelined<6>(e, base, lo, hi); break;
    case 7: rows_pipelined<7>(e, base, lo, hi); break;
    case 8: rows_pipelined<8>(e, base, lo, hi); break;
    default: break;
  }
  // (rec & 0xFFFFFF) = 2 * slot + half: times HD/2 it is the offset of the
  // item's half of row `slot` of x.
  const uint32_t xoff = (rec & 0xFFFFFFu) * (HD / 2) + 32 * s + 4 * q;
#ifdef FT_EXP_NO_STORE
  if (transform4(lo, hi) == 0x12345678u)
#endif
  __builtin_amdgcn_raw_buffer_store_b32(transform4(lo, hi), x_rsrc, xoff, 0, 0);
  uint32_t acc = 0;
#ifdef FT_EXP_NO_PSQT
  if (false) {
#else
  if (s == 0) {
#endif
    // PSQT part of this perspective: sum of psqtWeights[row][bucket] (int32
    // wrap).  The item's 8 lanes take entries q, q+8, q+16, q+24 (padding
    // entries name the zero row) and reduce over lane masks 1, 2, 12.
    const int bucket = (max((int)(rec >> 24), 1) - 1) >> 2;
    const uint16_t* ent = reinterpret_cast<const uint16_t*>(my);
    acc = q == 0 ? (uint32_t)ptile[krow * kPsqtBuckets + bucket] : 0u;  // own king
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += (uint32_t)ptile[(ent[q + 8 * j] >> 4) * kPsqtBuckets + bucket];
    acc += (uint32_t)__shfl_xor((int)acc, 1);
    acc += (uint32_t)__shfl_xor((int)acc, 2);
    acc += (uint32_t)__shfl_xor((int)acc, 12);
  }
  // Slices != 0 address past the buffer's range: the hardware drops the store
  // (raw buffer bounds check), so every pass issues the same store with no
  // branch and no memory traffic.
  const uint32_t poff = s == 0 ? (rec & 0xFFFFFFu) * 4u : kDroppedOffset;
  __builtin_amdgcn_raw_buffer_store_b32((int32_t)acc, psqt_rsrc, poff, 0, 0);
}

// One workgroup = one (unit, slice).  16 waves x 8 items per pass; records and
// lists are fetched two passes ahead while the current pass reads the LDS tile.
// Items of a unit are sorted by piece count, so a pass's longest list is that
// of its item 7 (clamped into the unit).
template <int HD>
__global__ __launch_bounds__(1024) void ft_slices_kernel(const uint4* __restrict__ tiles,
                                                         const int16_t* __restrict__ ftb,
                                                         const uint32_t* __restrict__ ctr,
                                                         const int4* __restrict__ units,
                                                         const uint32_t* __restrict__ items,
                                                         const uint16_t* __restrict__ flist,
                                                         const int32_t* __restrict__ psqw,
                                                         int32_t* __restrict__ psqt_part,
                                                         uint8_t* __restrict__ x) {
  constexpr int S = HD / 64;
  __shared__ uint4 img[kTileU4];
  __shared__ int32_t ptile[kTileRows * kPsqtBuckets];  // slice 0 only: PSQT rows of the king block
  __shared__ uint2 lbuf[16][64];                       // per wave: one pass's 8 feature lists
  const uint32_t w = blockIdx.x;
  const uint32_t j = w >> 3;
  const uint32_t unit = (j / S) * 8 + (w & 7);
  const int s = (int)(j % S);
  if (unit >= ctr[kNUnits]) return;
  const int4 u = units[unit];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int it_in_wave, q;
  lane_item(lane, it_in_wave, q);
  // Tile (and PSQT tile) fetch: every load in flight before the first LDS
  // store, and the first passes' lists behind them, so the fetch costs one
  // round trip instead of one per 16 KiB.
  constexpr int kTileLoads = (kTileU4 + 1023) / 1024;
  constexpr int kPtileU4 = kTileRows * kPsqtBuckets / 4, kPtileRealU4 = kRowsPerBlock * kPsqtBuckets / 4;
  const uint4* src = tiles + ((size_t)u.x * S + s) * kTileU4;
  uint4 t[kTileLoads];
#pragma unroll
  for (int k = 0; k < kTileLoads; ++k)
#ifdef FT_EXP_NO_TILE
    t[k] = make_uint4(k, 0, 0, 0);
#else
    t[k] = src[min((int)threadIdx.x + 1024 * k, kTileU4 - 1)];
#endif
  uint4 pt[2];
  const uint4* psrc = reinterpret_cast<const uint4*>(psqw + (size_t)u.x * kRowsPerBlock * kPsqtBuckets);
  if (s == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) pt[k] = psrc[min((int)threadIdx.x + 1024 * k, kPtileRealU4 - 1)];
  }
  u16x4 b_lo = *reinterpret_cast<const u16x4*>(ftb + 32 * s + 4 * q);
  u16x4 b_hi = *reinterpret_cast<const u16x4*>(ftb + HD / 2 + 32 * s + 4 * q);
  const int krow = king_row(u.x);
  const char* lbase = reinterpret_cast<const char*>(img) + kPlaneBytes * q;
  uint2* lb = lbuf[wv];
  const __amdgpu_buffer_rsrc_t psqt_rsrc = __builtin_amdgcn_make_buffer_rsrc(psqt_part, 0, kBufferRange, kBufferFlags);
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(x, 0, kBufferAll, kBufferFlags);
  const __amdgpu_buffer_rsrc_t items_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(items), 0, kBufferAll, kBufferFlags);
  const __amdgpu_buffer_rsrc_t flist_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(flist), 0, kBufferAll, kBufferFlags);
  const int last = u.z - 1;
  int base = u.y + wv * 8;
  PassFetch fa = fetch_pass(items_rsrc, flist_rsrc, base, last, lane, it_in_wave);
  PassFetch fb = fetch_pass(items_rsrc, flist_rsrc, base + 128, last, lane, it_in_wave);
#pragma unroll
  for (int k = 0; k < kTileLoads; ++k)
    if ((int)threadIdx.x + 1024 * k < kTileU4) img[threadIdx.x + 1024 * k] = t[k];
  if (s == 0) {
    uint4* pdst = reinterpret_cast<uint4*>(ptile);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = (int)threadIdx.x + 1024 * k;
      if (i < kPtileU4) pdst[i] = i < kPtileRealU4 ? pt[k] : make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();
  {  // the own-king row (every item of the unit has it) joins the bias
    const u32x4 kv = *reinterpret_cast<const u32x4*>(lbase + 16 * krow);
    const u32x2 klo = __builtin_shufflevector(kv, kv, 0, 1), khi = __builtin_shufflevector(kv, kv, 2, 3);
    b_lo += __builtin_bit_cast(u16x4, klo);
    b_hi += __builtin_bit_cast(u16x4, khi);
  }
  while (base < u.z) {
    const PassFetch cur = fa;
#ifndef FT_EXP_REUSE_LIST
    fa = fetch_pass(items_rsrc, flist_rsrc, base + 256, last, lane, it_in_wave);
#endif
    slice_pass<HD>(cur, lb, lane, it_in_wave, s, q, lbase, b_lo, b_hi, krow, ptile, psqt_rsrc, x_rsrc);
    base += 128;
    if (base >= u.z) break;
    const PassFetch cur2 = fb;
#ifndef FT_EXP_REUSE_LIST
    fb = fetch_pass(items_rsrc, flist_rsrc, base + 256, last, lane, it_in_wave);
#endif
    slice_pass<HD>(cur2, lb, lane, it_in_wave, s, q, lbase, b_lo, b_hi, krow, ptile, psqt_rsrc, x_rsrc);
    base += 128;
  }
}

template <int HD>
hipError_t relayout_t(const NetPtrs& net, void* tiles, hipStream_t stream) {
  hipLaunchKernelGGL((relayout_kernel<HD>), dim3(2048), dim3(256), 0, stream, net.ft_w, (uint4*)tiles);
  return hipGetLastError();
}

template <int HD>
hipError_t ft_slices_t(const SlicedPlan& P, const NetPtrs& net, uint8_t* x, uint32_t max_units, hipStream_t stream) {
  constexpr int S = HD / 64;
  const uint32_t groups = (max_units + 7) / 8;
  hipLaunchKernelGGL((ft_slices_kernel<HD>), dim3(groups * 8 * S), dim3(1024), 0, stream,
                     (const uint4*)P.tiles, net.ft_bias, P.ctr, (const int4*)P.units, P.items, P.flist, net.psqt_w,
                     P.psqt_part, x);
  return hipGetLastError();
}

}  // namespace

size_t sliced_tiles_bytes(uint32_t hd) { return tile_uint4_count(hd) * sizeof(uint4); }
size_t sliced_ctr_words() { return 3 * kBins + 16; }
uint32_t sliced_max_units(uint32_t chunk) { return 32 + (2 * chunk + kUnitItems - 1) / kUnitItems; }

#define FNNUE_HD_DISPATCH(hd, CALL) \
  switch (hd) {                     \
    case 128: return CALL(128);     \
    case 256: return CALL(256);     \
    case 512: return CALL(512);     \
    case 1024: return CALL(1024);   \
    case 2048: return CALL(2048);   \
    default: return hipErrorInvalidValue; \
  }

hipError_t launch_relayout_sliced(uint32_t hd, const NetPtrs& net, void* tiles, hipStream_t stream) {
#define CALL(H) relayout_t<H>(net, tiles, stream)
  FNNUE_HD_DISPATCH(hd, CALL)
#undef CALL
}

hipError_t launch_sliced_plan(const fnnue_pos* pos, uint32_t n, const SlicedPlan& P, int32_t* psqt, uint8_t* bucket,
                              uint32_t* err, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(P.ctr, 0, sliced_ctr_words() * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  // 1024-thread workgroups, at most one per CU: the per-bin global atomics that
  // merge the LDS histograms scale with the number of workgroups.
  uint32_t blocks = (n + 1023) / 1024;
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(plan_count_kernel, dim3(blocks), dim3(1024), 0, stream, pos, n, P.ctr, err);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(1024), 0, stream, P.ctr, (int4*)P.units, (uint32_t)kUnitItems);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(plan_scatter_kernel, dim3((n + kScatterPositions - 1) / kScatterPositions), dim3(kScatterPositions), 0, stream,
                     pos, n, P.ctr, P.items, P.flist, P.perm, bucket, psqt);
  return hipGetLastError();
}

hipError_t launch_sliced_ft(uint32_t hd, uint32_t n, const NetPtrs& net, const SlicedPlan& P, uint8_t* x,
                            hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t mu = sliced_max_units(n);
#define CALL(H) ft_slices_t<H>(P, net, x, mu, stream)
  FNNUE_HD_DISPATCH(hd, CALL)
#undef CALL
}

hipError_t launch_ft_sliced(uint32_t hd, const fnnue_pos* pos, uint32_t n, const NetPtrs& net, const SlicedPlan& P,
                            uint8_t* x, int32_t* psqt, uint8_t* bucket, uint32_t* err, hipStream_t stream) {
  const hipError_t e = launch_sliced_plan(pos, n, P, psqt, bucket, err, stream);
  return e != hipSuccess ? e : launch_sliced_ft(hd, n, net, P, x, stream);
}

}  // namespace fnnue
