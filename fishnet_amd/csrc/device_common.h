// device_common.h — device helpers shared by the NNUE kernels: packed-position
// decode (one 64-lane wave per position, lane = square), HalfKAv2_hm feature
// indices, wave reductions.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/fnnue.h"
#include "net.h"

namespace fnnue {
namespace {

constexpr int kZeroRow = kFeatures;  // all-zero padding row in ft_w / psqt_w

typedef int v4i __attribute__((ext_vector_type(4)));

template <int N> struct Vec {
  typedef unsigned short u16 __attribute__((ext_vector_type(N)));
  typedef short s16 __attribute__((ext_vector_type(N)));
  typedef unsigned char u8 __attribute__((ext_vector_type(N)));
};

// HalfKAv2_hm::make_index (upstream features/half_ka_v2_hm.cpp):
//   orient(p, s, ksq) = s ^ (p * SQ_A8) ^ ((file_of(ksq) < FILE_E) * SQ_H1)
//   index = orient(s) + PieceSquareIndex[p][pc] + PS_NB * KingBuckets[orient(ksq)]
// KingBuckets[o] = 4*(7-rank(o)) + (7-file(o)) for the e..h files o lands on.
__device__ __forceinline__ int make_index(int persp, int s, int pc, int ksq) {
  const int flip = (persp ? 56 : 0) ^ (((ksq & 7) < 4) ? 7 : 0);
  const int os = s ^ flip, ok = ksq ^ flip;
  const int type = pc & 7;
  const int plane = type == 6 ? 10 : 2 * (type - 1) + ((pc >> 3) != persp);
  return os + 64 * plane + 704 * (4 * (7 - (ok >> 3)) + (7 - (ok & 7)));
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Decoded position as seen by one wave: lane l = square l.
struct Decoded {
  int pc;        // piece on this lane's square
  uint64_t occ;  // occupied squares
  int stm, wk, bk, cnt;
  bool ok;
};

__device__ __forceinline__ Decoded decode(const fnnue_pos* p, int lane) {
  Decoded d;
  const uint8_t* pp = reinterpret_cast<const uint8_t*>(p);
  const int byte = pp[lane >> 1];
  d.pc = (byte >> ((lane & 1) * 4)) & 15;
  d.stm = pp[32];
  d.occ = __ballot(d.pc != 0);
  const uint64_t wkm = __ballot(d.pc == 6), bkm = __ballot(d.pc == 14);
  const uint64_t bad = __ballot(d.pc == 7 || d.pc == 8 || d.pc == 15);
  d.cnt = __popcll(d.occ);
  d.ok = !bad && __popcll(wkm) == 1 && __popcll(bkm) == 1 && d.cnt <= 32 && d.stm <= 1;
  d.wk = wkm ? __builtin_ctzll(wkm) : 0;
  d.bk = bkm ? __builtin_ctzll(bkm) : 0;
  return d;
}

// KingBuckets[orient(p, ksq, ksq)] — the 704-row block of the FT table that
// perspective p's features live in (upstream features/half_ka_v2_hm.h).
__device__ __forceinline__ int king_block(int persp, int ksq) {
  const int flip = (persp ? 56 : 0) ^ (((ksq & 7) < 4) ? 7 : 0);
  const int ok = ksq ^ flip;
  return 4 * (7 - (ok >> 3)) + (7 - (ok & 7));
}

}  // namespace
}  // namespace fnnue
