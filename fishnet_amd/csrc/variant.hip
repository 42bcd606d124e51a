// variant.hip — batched NNUE evaluation of Fairy-Stockfish variant positions
// (BASELINE config 5: crazyhouse / atomic) on the LDS-stationary feature
// transformer.
//
// Feature set "HalfKAv2 variants" (net.h; restated in oracle/variant_oracle.c,
// parity unpinned): per own-king square kb (64, oriented: rank flip for black,
// no mirroring) R rows = 704 board rows (orient(s) + 64 * plane, kings share
// plane 10) + for pocket variants 160 hand rows (704 + 16 * (2 * (pt - 1) +
// (owner != perspective)) + k for the k-th piece of a type in a hand).  A
// position has at most 32 pieces on board and in hand together, so every
// perspective-item's list (all features but the own king, whose row 640 + kb
// is folded into the bias) fits the 32-entry lists of the chess plan.
//
// Pipeline per chunk: vplan_count (LDS histograms of (kb, list length) and of
// layer-stack buckets) -> vplan_scan (one workgroup: bin offsets, units of
// <= kUnitItems items per kb) -> vplan_scatter (items, parity-ordered lists,
// bucket-sorted slots) -> ft_slices_kernel<HD, SWAR, VariantGeom<R>>
// (ft_sliced.hip) -> stack_kernel, exactly as for chess positions.
#include <hip/hip_runtime.h>

#include "variant_common.h"

namespace fnnue {

namespace {

__global__ __launch_bounds__(1024) void vplan_count_kernel(const fnnue_vpos* __restrict__ pos, uint32_t n, int pockets,
                                                          uint32_t* __restrict__ ctr, uint32_t* __restrict__ err) {
  __shared__ uint32_t h[kVBins];
  for (int i = threadIdx.x; i < kVBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
    const VariantBoard v = vdecode<false>(pos + p, pockets != 0);  // counts only: no occupancy mask
    if (!v.ok) {
      bad |= v.over ? 0u : 1u;  // an exploded king is a result (0, 0), not an error
      atomicAdd(&h[kVItemBins + 8], 1u);
    } else {
      atomicAdd(&h[vblock(0, v.b.wk) * 33 + v.nfeat], 1u);
      atomicAdd(&h[vblock(1, v.b.bk) * 33 + v.nfeat], 1u);
      atomicAdd(&h[kVItemBins + ((v.b.cnt - 1) >> 2)], 1u);
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(err, 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < kVBins; i += blockDim.x)
    if (h[i]) atomicAdd(&ctr[kVCnt + i], h[i]);
}

// One workgroup: exclusive scans of the item bins and of the position bins;
// the unit table (kb, first item, end) in chunks of <= kUnitItems per kb.
__global__ __launch_bounds__(1024) void vplan_scan_kernel(uint32_t* __restrict__ ctr, int4* __restrict__ units) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t kbstart[65];
  constexpr int per = (kVItemBins + 1023) / 1024;
  const int t = threadIdx.x;
  uint32_t local[per], sum = 0;
#pragma unroll
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    local[k] = i < kVItemBins ? ctr[kVCnt + i] : 0u;
    sum += local[k];
  }
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t v = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
#pragma unroll
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i < kVItemBins) {
      ctr[kVOff + i] = run;
      ctr[kVCur + i] = run;
      if (i % 33 == 0) kbstart[i / 33] = run;
    }
    run += local[k];
  }
  if (t == 1023) kbstart[64] = part[1023];
  if (t == 0) {
    uint32_t r = 0;
    for (int b = 0; b < kPosBins; ++b) {
      ctr[kVOff + kVItemBins + b] = r;
      ctr[kVCur + kVItemBins + b] = r;
      r += ctr[kVCnt + kVItemBins + b];
    }
  }
  __syncthreads();
  if (t < 64) {  // one wave: lane kb places its king block's units after a prefix sum
    const uint32_t b = kbstart[t], e = kbstart[t + 1];
    const uint32_t mine = (e - b + kUnitItems - 1) / kUnitItems;
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (t >= o) incl += v;
    }
    uint32_t u = incl - mine;
    for (uint32_t c = b; c < e; c += kUnitItems) units[u++] = make_int4(t, (int)c, (int)min(e, c + kUnitItems), 0);
    if (t == 63) ctr[kVNUnits] = incl;
  }
}

template <int R>
__global__ __launch_bounds__(kScatterPositions) void vplan_scatter_kernel(
    const fnnue_vpos* __restrict__ pos, uint32_t n, uint32_t* __restrict__ ctr, uint32_t* __restrict__ items,
    uint16_t* __restrict__ flist, uint32_t* __restrict__ perm, uint8_t* __restrict__ bucket_out,
    int32_t* __restrict__ psqt_out) {
  __shared__ uint32_t lcnt[kVBins];
  __shared__ uint32_t lbase[kVBins];
  __shared__ uint32_t lists[kScatterPositions * kVListStrideWords];
  for (int i = threadIdx.x; i < kVBins; i += blockDim.x) lcnt[i] = 0;
  __syncthreads();
  const uint32_t p = blockIdx.x * kScatterPositions + threadIdx.x;
  const bool live = p < n;
  VariantBoard v;
  int kw = 0, kb = 0, kp = kVItemBins + 8;
  uint32_t rw = 0, rb = 0, rp = 0;
  if (live) {
    v = vdecode(pos + p, R > kVBoardRows);
    if (v.ok) {
      kw = vblock(0, v.b.wk) * 33 + v.nfeat;
      kb = vblock(1, v.b.bk) * 33 + v.nfeat;
      kp = kVItemBins + ((v.b.cnt - 1) >> 2);
      rw = atomicAdd(&lcnt[kw], 1u);
      rb = atomicAdd(&lcnt[kb], 1u);
    }
    rp = atomicAdd(&lcnt[kp], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kVBins; i += blockDim.x) lbase[i] = lcnt[i] ? atomicAdd(&ctr[kVCur + i], lcnt[i]) : 0u;
  __syncthreads();
  if (!live) return;
  const uint32_t slot = lbase[kp] + rp;
  perm[slot] = p;
  if (!v.ok) {
    bucket_out[slot] = 0xFF;
    psqt_out[p] = 0;
    return;
  }
  const uint32_t iw = lbase[kw] + rw, ib = lbase[kb] + rb;
  // parity role of an item: its offset from the king block's first item (unit
  // starts are multiples of kUnitItems from there, so pass items 2k / 2k + 1)
  const uint32_t ppw = (iw - ctr[kVOff + vblock(0, v.b.wk) * 33]) & 1u;
  const uint32_t ppb = (ib - ctr[kVOff + vblock(1, v.b.bk) * 33]) & 1u;
  uint32_t* mine = lists + threadIdx.x * kVListStrideWords;
  vwrite_rows<R>(v, 0, iw, ppw, mine, flist);
  vwrite_rows<R>(v, 1, ib, ppb, mine, flist);
  const uint32_t bucket = (uint32_t)(v.b.cnt - 1) >> 2;  // pieces on board only
  items[iw] = ((uint32_t)v.nfeat << 24) | (bucket << 21) | (slot << 1) | (uint32_t)(v.b.stm != 0);
  items[ib] = ((uint32_t)v.nfeat << 24) | (bucket << 21) | (slot << 1) | (uint32_t)(v.b.stm != 1);
  bucket_out[slot] = (uint8_t)bucket;
}

}  // namespace

size_t variant_ctr_words() { return (3 * kVBins + 16 + 3) & ~(size_t)3; }  // a multiple of 4 words (one fill kernel)
uint32_t variant_max_units(uint32_t chunk) { return 64 + (2 * chunk + kUnitItems - 1) / kUnitItems; }

hipError_t launch_variant_plan(const fnnue_vpos* pos, uint32_t n, int variant, const SlicedPlan& P, int32_t* psqt,
                               uint8_t* bucket, uint32_t* err, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (variant != kVariantCrazyhouse && variant != kVariantAtomic) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(P.ctr, 0, variant_ctr_words() * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  const bool pockets = variant == kVariantCrazyhouse;
  uint32_t blocks = (n + 1023) / 1024;
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(vplan_count_kernel, dim3(blocks), dim3(1024), 0, stream, pos, n, pockets ? 1 : 0, P.ctr, err);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(vplan_scan_kernel, dim3(1), dim3(1024), 0, stream, P.ctr, (int4*)P.units);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const dim3 grid((n + kScatterPositions - 1) / kScatterPositions);
  if (pockets)
    hipLaunchKernelGGL((vplan_scatter_kernel<kVBoardRows + kVHandRows>), grid, dim3(kScatterPositions), 0, stream, pos,
                       n, P.ctr, P.items, P.flist, P.perm, bucket, psqt);
  else
    hipLaunchKernelGGL((vplan_scatter_kernel<kVBoardRows>), grid, dim3(kScatterPositions), 0, stream, pos, n, P.ctr,
                       P.items, P.flist, P.perm, bucket, psqt);
  return hipGetLastError();
}

}  // namespace fnnue
