// kernels.hip — CDNA4 (gfx950) kernels for batched Stockfish NNUE evaluation.
//
// Hot path (SURVEY.md §8a rows a2–a8):
//   ft_scratch  HalfKAv2_hm feature indices + FeatureTransformer refresh +
//               transform (clamp, pairwise product) + PSQT term.  One 64-lane
//               wave per position; the wave owns both int16 accumulators in
//               VGPRs: lane l holds elements [l*EPL, l*EPL+EPL) of each half
//               (HD/128 not a power of two: pieces, see Lanes), so every
//               weight-row read is a 1 KiB-contiguous wave load
//               (HD=1024: global_load_dwordx4 per lane) and the pairwise
//               product (j, j+HD/2) never crosses lanes.
//   ft_groups   Same, but walking a group of positions (a game's plies, or a
//               parent and its children) with incremental add/sub of the
//               changed feature rows; refresh when the perspective's king moves.
//   stack       fc_0 (HD -> 16) and fc_1 (30 -> 32) as int8 MFMA
//               (v_mfma_i32_16x16x64_i8) over 16-position tiles, SqrCReLU /
//               CReLU / fc_2 / fwd term in VALU.
// Upstream formulas restated in oracle/nnue_oracle.c (test-only); constants in
// net.h.  All arithmetic is integer and order-independent, so results are
// bit-exact regardless of scheduling.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "kernels.h"
#include "net.h"

namespace fnnue {

namespace {

// FeatureTransformer::transform for one perspective half (upstream
// nnue_feature_transformer.h): out[j] = clamp(a[j],0,127) * clamp(a[j+HD/2],0,127) / 128.
template <int EPL>
__device__ __forceinline__ void transform_store(typename Vec<EPL>::u16 lo, typename Vec<EPL>::u16 hi, uint8_t* dst) {
  typedef typename Vec<EPL>::s16 s16;
  typedef typename Vec<EPL>::u16 u16;
  const s16 zero = (s16)0, top = (s16)127;
  s16 a = __builtin_elementwise_min(__builtin_elementwise_max((s16)lo, zero), top);
  s16 b = __builtin_elementwise_min(__builtin_elementwise_max((s16)hi, zero), top);
  u16 prod = ((u16)a * (u16)b) >> (u16)7;
  *reinterpret_cast<typename Vec<EPL>::u8*>(dst) = __builtin_convertvector(prod, typename Vec<EPL>::u8);
}

// One wave's share of an accumulator half (HD/2 int16): lane l holds K
// pieces of P = lowest power of two dividing HD/128 columns, piece k at
// columns 64Pk + Pl .. +P-1.  Vector types only come in power-of-two sizes
// (an ext_vector of 12 elements occupies 16), so HD = 1536/2560/3072 use K =
// 3/5/3 pieces; every piece is one fully coalesced wave access.
template <int HD>
struct Lanes {
  static constexpr int kEpl = HD / 128, kP = kEpl & -kEpl, kK = kEpl / kP;
  typedef typename Vec<kP>::u16 u16;
  u16 v[kK];
  __device__ __forceinline__ static Lanes load(const int16_t* half, int lane) {
    Lanes r;
    const u16* p = reinterpret_cast<const u16*>(half);
#pragma unroll
    for (int k = 0; k < kK; ++k) r.v[k] = p[64 * k + lane];
    return r;
  }
  __device__ __forceinline__ Lanes& operator+=(const Lanes& o) {
#pragma unroll
    for (int k = 0; k < kK; ++k) v[k] += o.v[k];
    return *this;
  }
  __device__ __forceinline__ Lanes& operator-=(const Lanes& o) {
#pragma unroll
    for (int k = 0; k < kK; ++k) v[k] -= o.v[k];
    return *this;
  }
  // transformed output of one perspective: dst = that perspective's HD/2 bytes
  __device__ __forceinline__ static void transform(const Lanes& lo, const Lanes& hi, uint8_t* dst, int lane) {
#pragma unroll
    for (int k = 0; k < kK; ++k) transform_store<kP>(lo.v[k], hi.v[k], dst + kP * (64 * k + lane));
  }
  __device__ __forceinline__ static void zero(uint8_t* dst, int lane) {
#pragma unroll
    for (int k = 0; k < kK; ++k)
      *reinterpret_cast<typename Vec<kP>::u8*>(dst + kP * (64 * k + lane)) = (typename Vec<kP>::u8)0;
  }
};

// Adds (SIGN=+1) or subtracts the weight rows f(s) for every square s in `mask`
// to the lane's accumulator slice.  f is a per-lane value read with readlane,
// so each row address is wave-uniform (scalar base + lane offset) and each row
// is two 1 KiB-contiguous wave loads (HD=1024).  U rows are in flight per step.
template <int HD, int U>
__device__ __forceinline__ void add_rows(const int16_t* __restrict__ ftw, uint64_t mask, int f_add, int f_sub,
                                         bool do_sub, Lanes<HD>& lo, Lanes<HD>& hi, int lane) {
  typedef Lanes<HD> L;
  while (mask) {
    int fa[U], fs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (mask) {
        const int s = __builtin_ctzll(mask);
        mask &= mask - 1;
        fa[u] = __builtin_amdgcn_readlane(f_add, s);
        fs[u] = do_sub ? __builtin_amdgcn_readlane(f_sub, s) : kZeroRow;
      } else {
        fa[u] = kZeroRow;
        fs[u] = kZeroRow;
      }
    }
    L va[U][2], vs[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int16_t* ra = ftw + (size_t)fa[u] * HD;
      va[u][0] = L::load(ra, lane);
      va[u][1] = L::load(ra + HD / 2, lane);
      if (do_sub) {
        const int16_t* rs = ftw + (size_t)fs[u] * HD;
        vs[u][0] = L::load(rs, lane);
        vs[u][1] = L::load(rs + HD / 2, lane);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lo += va[u][0];
      hi += va[u][1];
      if (do_sub) {
        lo -= vs[u][0];
        hi -= vs[u][1];
      }
    }
  }
}

// PSQT term: (psqtAcc[stm][b] - psqtAcc[~stm][b]) / 2 with C truncation.
__device__ __forceinline__ int psqt_term(const int32_t* __restrict__ psqw, const Decoded& d, int lane, int bucket) {
  int fw = kZeroRow, fb = kZeroRow;
  if (d.pc) {
    fw = make_index(0, lane, d.pc, d.wk);
    fb = make_index(1, lane, d.pc, d.bk);
  }
  const int v = psqw[fw * kPsqtBuckets + bucket] - psqw[fb * kPsqtBuckets + bucket];
  int tot = wave_sum(v);
  if (d.stm) tot = -tot;
  return tot / 2;
}

template <int HD>
__device__ __forceinline__ void store_invalid(uint8_t* x, int lane) {
  Lanes<HD>::zero(x, lane);
  Lanes<HD>::zero(x + HD / 2, lane);
}

// ---------------------------------------------------------------------------
// ft_scratch: accumulators from scratch (upstream update_accumulator refresh).
template <int HD, int U>
__global__ __launch_bounds__(256) void ft_scratch_kernel(const fnnue_pos* __restrict__ pos, uint32_t n, NetPtrs net,
                                                         uint8_t* __restrict__ x, int32_t* __restrict__ psqt,
                                                         uint8_t* __restrict__ bucket_out, uint32_t* __restrict__ err) {
  typedef Lanes<HD> u16;
  const int lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const u16 b_lo = u16::load(net.ft_bias, lane), b_hi = u16::load(net.ft_bias + HD / 2, lane);
  for (uint32_t p = wid; p < n; p += nw) {
    const Decoded d = decode(pos + p, lane);
    uint8_t* xo = x + (size_t)p * HD;
    if (!d.ok) {
      store_invalid<HD>(xo, lane);
      if (lane == 0) {
        atomicOr(err, 1u);
        psqt[p] = 0;
        bucket_out[p] = 0xFF;
      }
      continue;
    }
    const int bucket = (d.cnt - 1) >> 2;
    int fw = kZeroRow, fb = kZeroRow;
    if (d.pc) {
      fw = make_index(0, lane, d.pc, d.wk);
      fb = make_index(1, lane, d.pc, d.bk);
    }
    const int v = net.psqt_w[fw * kPsqtBuckets + bucket] - net.psqt_w[fb * kPsqtBuckets + bucket];
    int tot = wave_sum(v);
    if (d.stm) tot = -tot;
    u16 w_lo = b_lo, w_hi = b_hi, k_lo = b_lo, k_hi = b_hi;
    // Both perspectives share the occupancy mask: interleave them so 4U row
    // halves are in flight per lane.
    uint64_t mask = d.occ;
    while (mask) {
      int f0[U], f1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (mask) {
          const int s = __builtin_ctzll(mask);
          mask &= mask - 1;
          f0[u] = __builtin_amdgcn_readlane(fw, s);
          f1[u] = __builtin_amdgcn_readlane(fb, s);
        } else {
          f0[u] = kZeroRow;
          f1[u] = kZeroRow;
        }
      }
      u16 r0[U][2], r1[U][2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int16_t* a = net.ft_w + (size_t)f0[u] * HD;
        const int16_t* b = net.ft_w + (size_t)f1[u] * HD;
        r0[u][0] = u16::load(a, lane);
        r0[u][1] = u16::load(a + HD / 2, lane);
        r1[u][0] = u16::load(b, lane);
        r1[u][1] = u16::load(b + HD / 2, lane);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        w_lo += r0[u][0];
        w_hi += r0[u][1];
        k_lo += r1[u][0];
        k_hi += r1[u][1];
      }
    }
    if (d.stm) {
      u16::transform(k_lo, k_hi, xo, lane);
      u16::transform(w_lo, w_hi, xo + HD / 2, lane);
    } else {
      u16::transform(w_lo, w_hi, xo, lane);
      u16::transform(k_lo, k_hi, xo + HD / 2, lane);
    }
    if (lane == 0) {
      psqt[p] = tot / 2;
      bucket_out[p] = (uint8_t)bucket;
    }
  }
}

// ---------------------------------------------------------------------------
// ft_groups: one wave walks a group.  CHAIN: base = previous position of the
// group; STAR: base = the group's first position (the parent).  Perspective c
// refreshes when there is no valid base, when its own king moved (upstream
// HalfKAv2_hm::requires_refresh), or when the delta is larger than a refresh.
template <int HD, int U>
__global__ __launch_bounds__(256) void ft_groups_kernel(const fnnue_pos* __restrict__ pos,
                                                        const uint32_t* __restrict__ off, uint32_t ngroups,
                                                        uint32_t lo, uint32_t hi, int star, NetPtrs net,
                                                        uint8_t* __restrict__ x, int32_t* __restrict__ psqt,
                                                        uint8_t* __restrict__ bucket_out,
                                                        uint32_t* __restrict__ err) {
  typedef Lanes<HD> u16;
  const int lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const u16 b_lo = u16::load(net.ft_bias, lane), b_hi = u16::load(net.ft_bias + HD / 2, lane);
  // The groups overlapping [lo, hi): from the first one ending after lo to
  // the last one starting before hi (offsets are non-decreasing; group_span's
  // check fails a call whose offsets are not), so a launch walks its chunk's
  // groups only, not all of them.
  uint32_t g0 = 0;
  for (uint32_t top = ngroups; g0 < top;) {
    const uint32_t m = (g0 + top) / 2;
    if (off[m + 1] <= lo) g0 = m + 1;
    else top = m;
  }
  for (uint32_t g = g0 + wid; g < ngroups && off[g] < hi; g += nw) {
    // the group clamped to this launch's positions [lo, hi) (a group cut at lo
    // restarts there with a refresh; malformed offsets give empty ranges)
    const uint32_t begin = max(off[g], lo), end = min(off[g + 1], hi);
    // Base state (previous ply for CHAIN, parent for STAR).
    bool have = false;
    int base_pc = 0, base_wk = 0, base_bk = 0;
    u16 bw_lo = b_lo, bw_hi = b_hi, bb_lo = b_lo, bb_hi = b_hi;
    for (uint32_t i = begin; i < end; ++i) {
      const Decoded d = decode(pos + i, lane);
      const uint32_t o = i - lo;
      uint8_t* xo = x + (size_t)o * HD;
      if (!d.ok) {
        store_invalid<HD>(xo, lane);
        if (lane == 0) {
          atomicOr(err, 1u);
          psqt[o] = 0;
          bucket_out[o] = 0xFF;
        }
        if (!star || i == begin) have = false;
        continue;
      }
      const int bucket = (d.cnt - 1) >> 2;
      const int tot = psqt_term(net.psqt_w, d, lane, bucket);
      const uint64_t changed = __ballot(d.pc != base_pc);
      const int nchg = __popcll(changed);
      u16 w_lo, w_hi, k_lo, k_hi;
      // White perspective.
      {
        const int f_new = d.pc ? make_index(0, lane, d.pc, d.wk) : kZeroRow;
        if (!have || d.wk != base_wk || 2 * nchg >= d.cnt) {
          w_lo = b_lo;
          w_hi = b_hi;
          add_rows<HD, U>(net.ft_w, d.occ, f_new, kZeroRow, false, w_lo, w_hi, lane);
        } else {
          const int f_old = base_pc ? make_index(0, lane, base_pc, d.wk) : kZeroRow;
          w_lo = bw_lo;
          w_hi = bw_hi;
          add_rows<HD, U>(net.ft_w, changed, d.pc != base_pc ? f_new : kZeroRow, f_old, true, w_lo, w_hi, lane);
        }
      }
      // Black perspective.
      {
        const int f_new = d.pc ? make_index(1, lane, d.pc, d.bk) : kZeroRow;
        if (!have || d.bk != base_bk || 2 * nchg >= d.cnt) {
          k_lo = b_lo;
          k_hi = b_hi;
          add_rows<HD, U>(net.ft_w, d.occ, f_new, kZeroRow, false, k_lo, k_hi, lane);
        } else {
          const int f_old = base_pc ? make_index(1, lane, base_pc, d.bk) : kZeroRow;
          k_lo = bb_lo;
          k_hi = bb_hi;
          add_rows<HD, U>(net.ft_w, changed, d.pc != base_pc ? f_new : kZeroRow, f_old, true, k_lo, k_hi, lane);
        }
      }
      if (d.stm) {
        u16::transform(k_lo, k_hi, xo, lane);
        u16::transform(w_lo, w_hi, xo + HD / 2, lane);
      } else {
        u16::transform(w_lo, w_hi, xo, lane);
        u16::transform(k_lo, k_hi, xo + HD / 2, lane);
      }
      if (lane == 0) {
        psqt[o] = tot;
        bucket_out[o] = (uint8_t)bucket;
      }
      if (!star || i == begin) {
        have = true;
        base_pc = d.pc;
        base_wk = d.wk;
        base_bk = d.bk;
        bw_lo = w_lo;
        bw_hi = w_hi;
        bb_lo = k_lo;
        bb_hi = k_hi;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Layer stacks (upstream nnue_architecture.h Network::propagate).  One wave per
// tile of 16 positions.  MFMA i32_16x16x64_i8 operand layout (checked on the
// device by mfma_selftest): lane l holds A[row l&15][k 16(l>>4) .. +15] and
// B[k 16(l>>4) .. +15][col l&15]; C/D: lane l holds C[row 4(l>>4)+r][col l&15].
// Transformed features are <= 126 and fc_1 inputs <= 127, so treating the u8
// activations as signed int8 is exact.
__device__ __forceinline__ int crelu(int v) { return min(127, max(0, v >> 6)); }
__device__ __forceinline__ int sqr_crelu(int v) {
  // min(127, (v*v >> 12) / 128) == min(127, v*v >> 19); clamp |v| first so
  // the square fits in 32 bits (|v| >= 8160 already saturates).
  const int a = min(abs(v), 16384);
  return min(127, (int)(((unsigned)(a * a)) >> 19));
}

// Per-bucket weights as one wave holds them: fc_1/fc_2 pieces and, unless the
// kernel keeps all fc_0 matrices in LDS (kW0InLds), the fc_0 matrix of the
// current layer stack as MFMA B fragments (HD/64 x 16 B per lane).
template <int HD, bool kW0InLds>
struct StackRegs {
  v4i w0[kW0InLds ? 1 : HD / 64];
  v4i w1a, w1b;
  int b0, b1a, b1b, w2a, w2b, b2;
  __device__ __forceinline__ void load(const NetPtrs& net, int b, int r16, int g) {
    if constexpr (!kW0InLds) {
      const v4i* wr = reinterpret_cast<const v4i*>(net.w0 + ((size_t)b * kL2 + r16) * HD);
#pragma unroll
      for (int s = 0; s < HD / 64; ++s) w0[s] = wr[4 * s + g];
    }
    const int8_t* w1 = net.w1 + (size_t)b * kL3 * kFc1In;
    w1a = g < 2 ? *reinterpret_cast<const v4i*>(w1 + r16 * kFc1In + 16 * g) : (v4i)0;
    w1b = g < 2 ? *reinterpret_cast<const v4i*>(w1 + (16 + r16) * kFc1In + 16 * g) : (v4i)0;
    b0 = net.b0[b * kL2 + r16];
    b1a = net.b1[b * kL3 + r16];
    b1b = net.b1[b * kL3 + 16 + r16];
    w2a = net.w2[b * kL3 + r16];
    w2b = net.w2[b * kL3 + 16 + r16];
    b2 = net.b2[b];
  }
};

// fc_0 weights of all 8 layer stacks in LDS (HD <= 1024: 128 KiB), one
// 1024-thread workgroup per CU, so 4 waves per SIMD stream x instead of the 2
// that fit when every wave holds a 16 KiB fc_0 matrix in VGPRs.  16-B chunk c
// of row (b, o) lives at chunk c ^ (o & (chunks - 1)): the 16 rows one
// ds_read_b128 lane group reads at a fixed K offset then cover all 64 banks.
template <int HD>
struct W0Lds {
  static constexpr bool kOn = HD <= 1024;
  static constexpr int kChunks = HD / 16;
  static constexpr int kWords = kOn ? kStacks * kL2 * kChunks : 1;
  // waves per workgroup: the x tile takes HD/16 VGPRs per lane, so HD = 1024
  // runs 3 waves per SIMD (<= 168 VGPRs) rather than 4 with spills
  static constexpr int kWaves = !kOn ? 4 : HD <= 512 ? 16 : 12;
  __device__ static __forceinline__ int slot(int b, int o, int c) {
    return (b * kL2 + o) * kChunks + (c ^ (o & (kChunks - 1)));
  }
};

// Persistent waves; wave w owns a contiguous range of 16-row tiles.  Rows come
// bucket-sorted from the sliced FT (perm != null), so a wave's weights stay in
// registers (LDS) across tiles and are reloaded only when the bucket changes.
template <int HD>
__global__ __launch_bounds__(64 * W0Lds<HD>::kWaves) void stack_kernel(
    const uint8_t* __restrict__ x, const uint8_t* __restrict__ bucket, uint32_t n, NetPtrs net,
    int32_t* __restrict__ positional, const uint32_t* __restrict__ perm, const int32_t* __restrict__ psqt_part,
    int32_t* __restrict__ psqt) {
  constexpr int KS = HD / 64;
  constexpr bool kLds = W0Lds<HD>::kOn;
  constexpr int kWaves = W0Lds<HD>::kWaves;
  __shared__ v4i w0s[W0Lds<HD>::kWords];
  // fc_1 inputs: 30 bytes per position, padded to 32 (lanes g >= 2 feed zeros)
  __shared__ __attribute__((aligned(16))) uint8_t x1s[kWaves][16][32];
  __shared__ int32_t fwds[kWaves][16];
  // x tile transpose (kLds): 16 rows x 128 B per wave, chunks XOR-swizzled
  __shared__ v4i xst[kLds ? kWaves : 1][kLds ? 128 : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (kLds) {
    const v4i* src = reinterpret_cast<const v4i*>(net.w0);
    for (int i = threadIdx.x; i < W0Lds<HD>::kWords; i += blockDim.x) {
      const int c = i % W0Lds<HD>::kChunks, row = i / W0Lds<HD>::kChunks;
      w0s[W0Lds<HD>::slot(row / kL2, row % kL2, c)] = src[i];
    }
  }
  // Zero the fc_1 input tile once (k >= 30 stays zero).
  if (g < 2) *reinterpret_cast<v4i*>(&x1s[wv][r16][16 * g]) = (v4i)0;
  if constexpr (kLds) __syncthreads();
  else wave_lds_sync();
  const uint32_t ntiles = (n + 15) / 16;
  const uint32_t nw = gridDim.x * kWaves, wid = blockIdx.x * kWaves + wv;
  const uint32_t per = (ntiles + nw - 1) / nw;
  const uint32_t t_begin = wid * per, t_end = min(ntiles, t_begin + per);
  StackRegs<HD, kLds> W;
  int cur = -1;
  for (uint32_t tile = t_begin; tile < t_end; ++tile) {
    const uint32_t p0 = tile * 16;
    const uint32_t prow = p0 + r16;
    const bool row_ok = prow < n;
    const int bk = row_ok ? bucket[prow] : 0xFF;
    if (row_ok && bk == 0xFF && g == 0) positional[perm ? perm[prow] : prow] = 0;  // invalid position
    if (psqt_part && row_ok && g == 1) {
      // upstream transform(): (psqtAcc[stm][b] - psqtAcc[~stm][b]) / 2, int32 wrap then C division
      const int v = bk == 0xFF ? 0 : (int)((uint32_t)psqt_part[2 * prow] - (uint32_t)psqt_part[2 * prow + 1]) / 2;
      psqt[perm ? perm[prow] : prow] = v;
    }
    // output rows of this lane's fc_2 results (lane r16 == 0 of group g: rows 4g .. 4g+3),
    // loaded with the tile so the stores at the end wait on nothing
    uint32_t dst[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t q = min(p0 + 4 * g + r, n - 1);
      dst[r] = perm ? perm[q] : q;
    }
    uint32_t bmask = 0;
#pragma unroll
    for (int b = 0; b < kStacks; ++b)
      if (__ballot(bk == b)) bmask |= 1u << b;
    v4i a[KS];
    if constexpr (kLds) {
      // x read as whole 128-B lines: load instruction 2j + h covers rows 8h ..
      // 8h + 7 of the tile, bytes 128j .. 128j + 127 (lane l: row l / 8, 16-B
      // chunk l % 8), then each 128-B piece goes through the wave's LDS buffer
      // into the MFMA A layout (lane l: row l % 16, chunk 4k + l / 16 of K-step
      // 2j + k).  The MFMA shape itself reads 16 rows x 64 B per instruction,
      // half lines.  Chunk c of row r sits at c ^ (r & 7): conflict-free writes
      // (8 lanes = one row) and reads (a ds_read_b128 lane group: 16 distinct
      // 4-bank sets).
      constexpr int KP = HD / 128;
      const int wr = lane >> 3, wc = lane & 7;
      const uint32_t r0 = p0 + wr, r1 = r0 + 8;
      const v4i* x0 = reinterpret_cast<const v4i*>(x + (size_t)(r0 < n ? r0 : p0) * HD) + wc;
      const v4i* x1 = reinterpret_cast<const v4i*>(x + (size_t)(r1 < n ? r1 : p0) * HD) + wc;
#pragma unroll
      // x is read exactly once: non-temporal loads (-1 %; non-temporal STORES of x
      // in the FT cost +3 % there and +6 % here, x then misses the Infinity Cache)
      for (int j = 0; j < KP; ++j) {
        a[2 * j] = r0 < n ? __builtin_nontemporal_load(x0 + 8 * j) : (v4i)0;
        a[2 * j + 1] = r1 < n ? __builtin_nontemporal_load(x1 + 8 * j) : (v4i)0;
      }
      v4i* st = xst[wv];
#pragma unroll
      for (int j = 0; j < KP; ++j) {  // in place: LDS ops of one wave complete in order
        st[wr * 8 + (wc ^ (wr & 7))] = a[2 * j];
        st[(wr + 8) * 8 + (wc ^ (wr & 7))] = a[2 * j + 1];
        // other lanes' stores are read back: keep the compiler from reordering
        // across the exchange (no instruction: the hardware keeps the order)
        wave_lds_sync();
        a[2 * j] = st[r16 * 8 + (g ^ (r16 & 7))];
        a[2 * j + 1] = st[r16 * 8 + ((4 + g) ^ (r16 & 7))];
        wave_lds_sync();  // this step's reads before the next step's stores
      }
    } else {
      const v4i* xr = reinterpret_cast<const v4i*>(x + (size_t)(row_ok ? prow : p0) * HD);
#pragma unroll
      for (int s = 0; s < KS; ++s) a[s] = row_ok ? __builtin_nontemporal_load(xr + 4 * s + g) : (v4i)0;
    }
    while (bmask) {
      const int b = __builtin_ctz(bmask);
      bmask &= bmask - 1;
      if (b != cur) {
        W.load(net, b, r16, g);
        cur = b;
      }
      // fc_0: y[pos][out] = b0 + sum_k x[pos][k] * w0[out][k]
      v4i acc = (v4i)0;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        v4i wf;
        if constexpr (kLds) wf = w0s[W0Lds<HD>::slot(b, r16, 4 * s + g)];
        else wf = W.w0[s];
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[s], wf, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = acc[r] + W.b0;
        const int p = 4 * g + r;
        if (r16 < kL2 - 1) {
          x1s[wv][p][r16] = (uint8_t)sqr_crelu(y);
          x1s[wv][p][15 + r16] = (uint8_t)crelu(y);
        } else {
          // fwdOut = y15 * (600 * OutputScale) / (127 * (1 << WeightScaleBits))
          fwds[wv][p] = (int)(((long long)y * 9600) / 8128);
        }
      }
      wave_lds_sync();
      // fc_1 (30 -> 32, k padded to 64 with zeros), two MFMAs for outputs 0..15, 16..31.
      const v4i a1 = g < 2 ? *reinterpret_cast<const v4i*>(&x1s[wv][r16][16 * g]) : (v4i)0;
      const v4i z0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, W.w1a, (v4i)0, 0, 0, 0);
      const v4i z1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, W.w1b, (v4i)0, 0, 0, 0);
      int part[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) part[r] = W.w2a * crelu(z0[r] + W.b1a) + W.w2b * crelu(z1[r] + W.b1b);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[r] += __shfl_xor(part[r], o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 4 * g + r;
        const int pb = __shfl(bk, p);
        if (r16 == 0 && pb == b) positional[dst[r]] = W.b2 + part[r] + fwds[wv][p];
      }
      wave_lds_sync();
    }
  }
}

// ---------------------------------------------------------------------------
// MFMA layout self test: C = A * B with A[i][k] = (i*7 + k*3) % 19 - 9 and
// B[k][j] = (k*5 + j*11) % 23 - 11 loaded with the kernels' lane map.
__global__ void mfma_selftest_kernel(int* out) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, g = lane >> 4;
  v4i a, b;
  int8_t* ap = reinterpret_cast<int8_t*>(&a);
  int8_t* bp = reinterpret_cast<int8_t*>(&b);
  for (int j = 0; j < 16; ++j) {
    const int k = 16 * g + j;
    ap[j] = (int8_t)((r16 * 7 + k * 3) % 19 - 9);
    bp[j] = (int8_t)((k * 5 + r16 * 11) % 23 - 11);
  }
  const v4i c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, (v4i)0, 0, 0, 0);
  int bad = 0;
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * g + r, jj = r16;
    int ref = 0;
    for (int k = 0; k < 64; ++k) ref += ((i * 7 + k * 3) % 19 - 9) * ((k * 5 + jj * 11) % 23 - 11);
    bad += ref != c[r];
  }
  atomicAdd(out, bad);
}

template <int HD>
hipError_t launch_scratch_t(const fnnue_pos* pos, uint32_t n, const NetPtrs& net, uint8_t* x, int32_t* psqt,
                            uint8_t* bucket, uint32_t* err, hipStream_t stream) {
  const uint32_t waves = n;
  uint32_t blocks = (waves + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((ft_scratch_kernel<HD, 4>), dim3(blocks), dim3(256), 0, stream, pos, n, net, x, psqt, bucket, err);
  return hipGetLastError();
}

template <int HD>
hipError_t launch_groups_t(const fnnue_pos* pos, const uint32_t* off, uint32_t ngroups, uint32_t lo, uint32_t hi,
                           int mode,
                           const NetPtrs& net, uint8_t* x, int32_t* psqt, uint8_t* bucket, uint32_t* err,
                           hipStream_t stream) {
  // one wave per group of the chunk (about hi - lo positions' worth at most,
  // empty groups aside: the waves grid-stride)
  uint32_t blocks = std::min((ngroups + 3) / 4, (hi - lo + 3) / 4 + 1);
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((ft_groups_kernel<HD, 4>), dim3(blocks), dim3(256), 0, stream, pos, off, ngroups, lo, hi,
                     mode == FNNUE_GROUP_STAR, net, x, psqt, bucket, err);
  return hipGetLastError();
}

template <int HD>
hipError_t launch_stack_t(const uint8_t* x, const uint8_t* bucket, uint32_t n, const NetPtrs& net, int32_t* positional,
                          const uint32_t* perm, const int32_t* psqt_part, int32_t* psqt, hipStream_t stream) {
  // Persistent, contiguous tile ranges: HD <= 1024 one workgroup per CU (fc_0
  // in LDS), else two 4-wave workgroups per CU (fc_0 in VGPRs).
  constexpr uint32_t kWaves = W0Lds<HD>::kWaves, kMaxBlocks = W0Lds<HD>::kOn ? 256 : 512;
  const uint32_t tiles = (n + 15) / 16;
  uint32_t blocks = (tiles + kWaves - 1) / kWaves;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((stack_kernel<HD>), dim3(blocks), dim3(64 * kWaves), 0, stream, x, bucket, n, net, positional,
                     perm, psqt_part, psqt);
  return hipGetLastError();
}

}  // namespace

bool kernels_support_hd(uint32_t hd) {
  return hd == 128 || hd == 256 || hd == 512 || hd == 1024 || hd == 1536 || hd == 2048 || hd == 2560 ||
         hd == 3072;
}

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

hipError_t launch_ft_scratch(uint32_t hd, const fnnue_pos* pos, uint32_t n, const NetPtrs& net, uint8_t* x,
                             int32_t* psqt, uint8_t* bucket, uint32_t* err, hipStream_t stream) {
#define CALL(H) launch_scratch_t<H>(pos, n, net, x, psqt, bucket, err, stream)
  FNNUE_HD_DISPATCH(hd, CALL)
#undef CALL
}

hipError_t launch_ft_groups(uint32_t hd, const fnnue_pos* pos, const uint32_t* off, uint32_t ngroups, uint32_t lo,
                            uint32_t hi, int mode, const NetPtrs& net, uint8_t* x, int32_t* psqt, uint8_t* bucket,
                            uint32_t* err, hipStream_t stream) {
#define CALL(H) launch_groups_t<H>(pos, off, ngroups, lo, hi, mode, net, x, psqt, bucket, err, stream)
  FNNUE_HD_DISPATCH(hd, CALL)
#undef CALL
}

hipError_t launch_stack(uint32_t hd, const uint8_t* x, const uint8_t* bucket, uint32_t n, const NetPtrs& net,
                        int32_t* positional, const uint32_t* perm, const int32_t* psqt_part, int32_t* psqt,
                        hipStream_t stream) {
#define CALL(H) launch_stack_t<H>(x, bucket, n, net, positional, perm, psqt_part, psqt, stream)
  FNNUE_HD_DISPATCH(hd, CALL)
#undef CALL
}

hipError_t run_mfma_selftest(int* bad) {
  int* d = nullptr;
  hipError_t e = hipMalloc(&d, sizeof(int));
  if (e != hipSuccess) return e;
  e = hipMemset(d, 0, sizeof(int));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mfma_selftest_kernel, dim3(1), dim3(64), 0, 0, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(bad, d, sizeof(int), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return e;
}

}  // namespace fnnue
