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

#include <type_traits>

#include "sliced_common.h"

namespace fnnue {

namespace {

__global__ __launch_bounds__(1024) void plan_count_kernel(const fnnue_pos* __restrict__ pos, uint32_t n,
                                                         uint32_t* __restrict__ ctr, uint32_t* __restrict__ err) {
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    const LaneBoard b = lane_decode<false>(pos + p);  // counts only: no occupancy mask
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

// Item record: (n << 24) | (bucket << 21) | (slot << 1) | half, half 0 =
// side-to-move half of x; n = list length + 1 (pieces, + pieces in hand for
// variants), bucket = the PSQT / layer-stack bucket (pieces on board - 1) / 4
// (slot < 2^20: chunk_for_hd).
// One lane per position; the workgroup's 256 positions get local ranks from
// LDS atomics, then reserve one range per bin with a single global atomic.
__global__ __launch_bounds__(kScatterPositions) void plan_scatter_kernel(const fnnue_pos* __restrict__ pos, uint32_t n,
                                                           uint32_t* __restrict__ ctr, uint32_t* __restrict__ items,
                                                           uint16_t* __restrict__ flist, uint32_t* __restrict__ perm,
                                                           uint8_t* __restrict__ bucket_out,
                                                           int32_t* __restrict__ psqt_out) {
  __shared__ uint32_t lcnt[kBins];
  __shared__ uint32_t lbase[kBins];
  __shared__ uint32_t lists[kScatterPositions * kListStrideWords];  // write_rows staging, one row per lane
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
    lbase[i] = lcnt[i] ? atomicAdd(&ctr[kCur + i], lcnt[i]) : 0;
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
  uint32_t* mine = lists + threadIdx.x * kListStrideWords;
  write_rows(b, 0, b.wk, iw, (iw - ctr[kOff + king_block(0, b.wk) * 33]) & 1u, mine, flist);
  write_rows(b, 1, b.bk, ib, (ib - ctr[kOff + king_block(1, b.bk) * 33]) & 1u, mine, flist);
  items[iw] = ((uint32_t)b.cnt << 24) | ((uint32_t)bucket << 21) | (slot << 1) | (uint32_t)(b.stm != 0);
  items[ib] = ((uint32_t)b.cnt << 24) | ((uint32_t)bucket << 21) | (slot << 1) | (uint32_t)(b.stm != 1);
  bucket_out[slot] = (uint8_t)bucket;
  // the PSQT term is summed from LDS by the slice-0 workgroups of ft_slices
}

// One pass (8 items per wave) over the LDS tile: the lists go to the wave's
// LDS buffer, bias + rows, transform, store; in slice 0 also the PSQT part.
// maxn = the pass's longest list.  The stores are unconditional: a lane past
// the end of the unit holds the clamped last item and rewrites its identical
// values (a store skipped on some path would make hipcc's vmcnt bookkeeping
// wait for every store before the next pass's rows).
template <int HD, bool kSwar, bool kPsqt>
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
  rows_sum<kSwar>(maxn - 1, e, base, lo, hi);  // maxn - 1 rows (own king in the bias); wave-uniform, straight-line
  // (rec & kItemRowMask) = 2 * slot + half: times HD/2 it is the offset of the
  // item's half of row `slot` of x.
  const uint32_t xoff = (rec & kItemRowMask) * (HD / 2) + 32 * s + 4 * q;
  const uint32_t xv = kSwar ? transform4_swar(lo, hi) : transform4(lo, hi);
  __builtin_amdgcn_raw_buffer_store_b32(xv, x_rsrc, xoff, 0, 0);
  if constexpr (kPsqt) {
    // PSQT part of this perspective: sum of psqtWeights[row][bucket] (int32
    // wrap), own king included, in the fetch layout: lane l holds entries
    // 4(l&7) .. +3 of pass item l>>3 (f.lst, padding entries name the zero
    // row), the 8 lanes of an item are consecutive (DPP reductions), and the
    // item's record comes from its q = 0 lane in the lane_item layout (items
    // 0..7 -> lanes 0, 20, 4, 16, 32, 52, 36, 48) by one ds_bpermute.
    const uint32_t li = (uint32_t)lane >> 3;
    const int src = (int)(((li & 4u) << 3) + ((0x10041400u >> (8u * (li & 3u))) & 0xFFu));
    const uint32_t reci = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)rec);
    const int bk = (int)((reci >> 21) & 7u);
    auto pw = [&](uint32_t en) { return (uint32_t)ptile[(en >> 4) * kPsqtBuckets + bk]; };
    uint32_t a2 = (lane & 7) == 0 ? (uint32_t)ptile[krow * kPsqtBuckets + bk] : 0u;  // own king
    a2 += pw(f.lst.x & 0xFFFFu) + pw(f.lst.x >> 16) + pw(f.lst.y & 0xFFFFu) + pw(f.lst.y >> 16);
    a2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)a2, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    a2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)a2, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    a2 += (uint32_t)__builtin_amdgcn_mov_dpp((int)a2, 0x141, 0xF, 0xF, false);  // row_half_mirror: quads 0 <-> 1
    __builtin_amdgcn_raw_buffer_store_b32((int32_t)a2, psqt_rsrc,
                                          (lane & 7) == 0 ? (reci & kItemRowMask) * 4u : kDroppedOffset, 0, 0);
  }
}

// One workgroup = one (unit, slice).  16 waves x 8 items per pass; records and
// lists are fetched two passes ahead while the current pass reads the LDS tile.
// Items of a unit are sorted by piece count, so a pass's longest list is that
// of its item 7 (clamped into the unit).  kSwar: the tile is converted to SWAR
// words on its way into LDS and rows are summed as 32-bit words (swar_tile_words).
template <int HD, bool kSwar, class G = ChessGeom>
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
  constexpr int kTileU4 = G::kTileU4;
  __shared__ uint4 img[kTileU4];
  __shared__ int32_t ptile[G::kTileRows * kPsqtBuckets];  // slice 0 only: PSQT rows of the king block
  __shared__ uint2 lbuf[16][64];                       // per wave: one pass's 8 feature lists
  const uint32_t w = blockIdx.x;
  const uint32_t j = w >> 3;
  const uint32_t unit = (j / S) * 8 + (w & 7);
  const int s = (int)(j % S);
  if (unit >= ctr[G::kNUnitsWord]) return;
  const int4 u = units[unit];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int it_in_wave, q;
  lane_item(lane, it_in_wave, q);
  // Tile (and PSQT tile) fetch: every load in flight before the first LDS
  // store, and the first passes' lists behind them, so the fetch costs one
  // round trip instead of one per 16 KiB.
  constexpr int kTileLoads = (kTileU4 + 1023) / 1024;
  constexpr int kPtileU4 = G::kTileRows * kPsqtBuckets / 4, kPtileRealU4 = G::kRows * kPsqtBuckets / 4;
  static_assert(kPtileU4 <= 2048, "PSQT tile loads: two per thread");
  const uint4* src = tiles + ((size_t)u.x * S + s) * kTileU4;
  uint4 t[kTileLoads];
#pragma unroll
  for (int k = 0; k < kTileLoads; ++k)
    t[k] = src[min((int)threadIdx.x + 1024 * k, kTileU4 - 1)];
  uint4 pt[2];
  const uint4* psrc = reinterpret_cast<const uint4*>(psqw + (size_t)u.x * G::kRows * kPsqtBuckets);
  if (s == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) pt[k] = psrc[min((int)threadIdx.x + 1024 * k, kPtileRealU4 - 1)];
  }
  u16x4 b_lo = *reinterpret_cast<const u16x4*>(ftb + 32 * s + 4 * q);
  u16x4 b_hi = *reinterpret_cast<const u16x4*>(ftb + HD / 2 + 32 * s + 4 * q);
  const int krow = G::king_row(u.x);
  const char* lbase = reinterpret_cast<const char*>(img) + G::kPlaneBytes * q;
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
    if ((int)threadIdx.x + 1024 * k < kTileU4) {
      uint4 v = t[k];
      if constexpr (kSwar) v = swar_tile_words(v);
      img[threadIdx.x + 1024 * k] = v;
    }
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
  // Slice 0 also sums the PSQT part; the other slices run a copy of the loop
  // without that code (a runtime branch in the shared loop cost them 8 %).
  auto run = [&](auto psqt) {
    constexpr bool kPsqt = decltype(psqt)::value;
    while (base < u.z) {
      const PassFetch cur = fa;
      fa = fetch_pass(items_rsrc, flist_rsrc, base + 256, last, lane, it_in_wave);
      slice_pass<HD, kSwar, kPsqt>(cur, lb, lane, it_in_wave, s, q, lbase, b_lo, b_hi, krow, ptile, psqt_rsrc, x_rsrc);
      base += 128;
      if (base >= u.z) break;
      const PassFetch cur2 = fb;
      fb = fetch_pass(items_rsrc, flist_rsrc, base + 256, last, lane, it_in_wave);
      slice_pass<HD, kSwar, kPsqt>(cur2, lb, lane, it_in_wave, s, q, lbase, b_lo, b_hi, krow, ptile, psqt_rsrc,
                                   x_rsrc);
      base += 128;
    }
  };
  if (s == 0)
    run(std::true_type{});
  else
    run(std::false_type{});
}

template <int HD>
hipError_t relayout_t(const NetPtrs& net, void* tiles, hipStream_t stream) {
  hipLaunchKernelGGL((relayout_kernel<HD>), dim3(2048), dim3(256), 0, stream, net.ft_w, (uint4*)tiles);
  return hipGetLastError();
}

template <int HD, class G = ChessGeom>
hipError_t ft_slices_t(const SlicedPlan& P, const NetPtrs& net, uint8_t* x, uint32_t max_units, hipStream_t stream) {
  constexpr int S = HD / 64;
  const uint32_t groups = (max_units + 7) / 8;
  if (P.swar)
    hipLaunchKernelGGL((ft_slices_kernel<HD, true, G>), dim3(groups * 8 * S), dim3(1024), 0, stream,
                       (const uint4*)P.tiles, net.ft_bias, P.ctr, (const int4*)P.units, P.items, P.flist, net.psqt_w,
                       P.psqt_part, x);
  else
    hipLaunchKernelGGL((ft_slices_kernel<HD, false, G>), dim3(groups * 8 * S), dim3(1024), 0, stream,
                       (const uint4*)P.tiles, net.ft_bias, P.ctr, (const int4*)P.units, P.items, P.flist, net.psqt_w,
                       P.psqt_part, x);
  return hipGetLastError();
}

template <int HD, class G>
hipError_t relayout_g(const NetPtrs& net, void* tiles, hipStream_t stream) {
  hipLaunchKernelGGL((relayout_kernel<HD, G>), dim3(2048), dim3(256), 0, stream, net.ft_w, (uint4*)tiles);
  return hipGetLastError();
}

}  // namespace

size_t sliced_tiles_bytes(uint32_t hd) { return tile_uint4_count(hd) * sizeof(uint4); }
// a multiple of 4 words: hipMemsetAsync of a size that is not a multiple of
// 16 bytes runs two fill kernels
size_t sliced_ctr_words() { return (3 * kBins + 16 + 3) & ~(size_t)3; }
uint32_t sliced_max_units(uint32_t chunk) { return 32 + (2 * chunk + kUnitItems - 1) / kUnitItems; }

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
  hipLaunchKernelGGL(plan_scan_kernel_t<32>, dim3(1), dim3(1024), 0, stream, P.ctr, (int4*)P.units, (uint32_t)kUnitItems);
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

// ---- Fairy-Stockfish variant feature sets on the same kernel (variant.hip plans) ----
size_t variant_tiles_bytes(uint32_t hd, int variant) {
  const int planes = variant == kVariantCrazyhouse ? VariantGeom<kVBoardRows + kVHandRows>::kTileU4
                                                   : VariantGeom<kVBoardRows>::kTileU4;
  return (size_t)64 * (hd / 64) * planes * sizeof(uint4);
}

// Variant nets come in widths 256 / 512 / 1024 (kernels_support_variant).
#define FNNUE_VHD_DISPATCH(hd, CALL)      \
  switch (hd) {                           \
    case 256: return CALL(256);           \
    case 512: return CALL(512);           \
    case 1024: return CALL(1024);         \
    default: return hipErrorInvalidValue; \
  }
#define FNNUE_VARIANT_DISPATCH(variant, CALLG)                                   \
  if (variant == kVariantCrazyhouse) {                                          \
    using G = VariantGeom<kVBoardRows + kVHandRows>;                            \
    FNNUE_VHD_DISPATCH(hd, CALLG)                                               \
  } else if (variant == kVariantAtomic) {                                       \
    using G = VariantGeom<kVBoardRows>;                                         \
    FNNUE_VHD_DISPATCH(hd, CALLG)                                               \
  }                                                                             \
  return hipErrorInvalidValue;

hipError_t launch_relayout_variant(uint32_t hd, int variant, const NetPtrs& net, void* tiles, hipStream_t stream) {
#define CALLG(H) relayout_g<H, G>(net, tiles, stream)
  FNNUE_VARIANT_DISPATCH(variant, CALLG)
#undef CALLG
}

hipError_t launch_variant_ft(uint32_t hd, int variant, uint32_t n, const NetPtrs& net, const SlicedPlan& P, uint8_t* x,
                             hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t mu = variant_max_units(n);
#define CALLG(H) ft_slices_t<H, G>(P, net, x, mu, stream)
  FNNUE_VARIANT_DISPATCH(variant, CALLG)
#undef CALLG
}

hipError_t launch_ft_sliced(uint32_t hd, const fnnue_pos* pos, uint32_t n, const NetPtrs& net, const SlicedPlan& P,
                            uint8_t* x, int32_t* psqt, uint8_t* bucket, uint32_t* err, hipStream_t stream,
                            hipEvent_t mid) {
  hipError_t e = launch_sliced_plan(pos, n, P, psqt, bucket, err, stream);
  if (e == hipSuccess && mid) e = hipEventRecord(mid, stream);
  return e != hipSuccess ? e : launch_sliced_ft(hd, n, net, P, x, stream);
}

}  // namespace fnnue
