// vbuilder.hip — device batch builder for Fairy-Stockfish variants
// (crazyhouse, atomic): the variant half of IncomingBatch::from_acquired
// ([ref] src/queue.rs:524-552 with body.variant != Standard, routed to the
// MultiVariant engine at :530-539; variants from src/assets.rs:384-391).
//
// As builder.hip for chess: one thread per game parses the FEN (holdings,
// promoted marks) and replays the UCI moves (drops "P@e4", pockets,
// explosions) with the rules of vboard.h — the same source the host replay
// (fnnue_game_vpositions) runs, which the tests hold it to record for record —
// writing one fnnue_vpos per ply; CHILDREN adds one thread per ply for its
// legal children (drops included).
#include <hip/hip_runtime.h>

#include <vector>

#include "builder.h"
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

__device__ __forceinline__ void vlatch(uint32_t* err, uint32_t code, uint32_t game, uint32_t ply) {
  if (atomicCAS(&err[0], 0u, code) == 0u) {
    err[1] = game;
    err[2] = ply;
  }
}

__global__ void vreplay_kernel(int variant, const char* __restrict__ text, const uint32_t* __restrict__ fen_off,
                               const uint32_t* __restrict__ mv_off, uint32_t ngames,
                               const uint32_t* __restrict__ ply_off, fnnue_vpos* __restrict__ out,
                               vb::VBoard* __restrict__ states, uint32_t* __restrict__ err,
                               uint8_t* __restrict__ final) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngames) return;
  vb::VBoard b;
  if (!vb::parse_fen(text, fen_off[g], mv_off[g], variant, b)) {
    vlatch(err, kBuildErrFen, g, 0);
    return;
  }
  uint32_t o = ply_off[g];
  if (out) out[o] = vb::pack(b);
  if (states) states[o] = b;
  uint32_t p = mv_off[g], st, ply = 0;
  const uint32_t end = fen_off[g + 1];
  int len;
  while ((len = vb::next_token(text, p, end, st)) > 0) {
    ++ply;
    vb::VMove m;
    if (!vb::match_uci(b, text + st, len, m)) {
      vlatch(err, kBuildErrMove, g, ply);
      return;
    }
    vb::do_move(b, m);
    ++o;
    if (out) out[o] = vb::pack(b);
    if (states) states[o] = b;
  }
  if (final) final[g] = vb::final_state(b);
}

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

BuildResult build_vbatch_device(int variant, const char* d_text, const uint32_t* d_fen_off, const uint32_t* d_mv_off,
                                uint32_t ngames, bool children, fnnue_vpos* d_out, size_t cap, uint32_t* d_group_off,
                                size_t off_cap, hipStream_t s, uint8_t* d_final) {
  BuildResult R;
  auto fail = [&](hipError_t e) {
    R.hip = e;
    return R;
  };
  hipError_t e;
  uint32_t *plies = nullptr, *ply_off = nullptr, *err = nullptr, *cnt = nullptr, *coff = nullptr;
  vb::VBoard* states = nullptr;
  struct Free {
    std::vector<void*> p;
    ~Free() {
      for (void* x : p) (void)hipFree(x);
    }
  } F;
  auto alloc = [&](void** p, size_t bytes) {
    hipError_t a = hipMalloc(p, bytes ? bytes : 4);
    if (a == hipSuccess) F.p.push_back(*p);
    return a;
  };
  if ((e = alloc((void**)&plies, (size_t)(ngames + 1) * 4)) != hipSuccess) return fail(e);
  if ((e = alloc((void**)&ply_off, (size_t)(ngames + 1) * 4)) != hipSuccess) return fail(e);
  if ((e = alloc((void**)&err, 16)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(err, 0, 16, s)) != hipSuccess) return fail(e);
  if ((e = hipMemsetAsync(plies + ngames, 0, 4, s)) != hipSuccess) return fail(e);
  const uint32_t bs = 64;
  hipLaunchKernelGGL(vcount_plies_kernel, dim3((ngames + bs - 1) / bs), dim3(bs), 0, s, d_text, d_fen_off, d_mv_off,
                     ngames, plies);
  if ((e = hipGetLastError()) != hipSuccess) return fail(e);
  if ((e = builder_exclusive_scan(plies, ply_off, ngames, s)) != hipSuccess) return fail(e);
  uint32_t total_plies = 0;
  if ((e = hipMemcpy(&total_plies, ply_off + ngames, 4, hipMemcpyDeviceToHost)) != hipSuccess) return fail(e);
  if (!children) {
    R.n_out = total_plies;
    R.n_groups = ngames;
    if (cap < total_plies || off_cap < (size_t)ngames + 1 || !d_out || !d_group_off) {
      R.capacity = true;
      return R;
    }
    hipLaunchKernelGGL(vreplay_kernel, dim3((ngames + bs - 1) / bs), dim3(bs), 0, s, variant, d_text, d_fen_off,
                       d_mv_off, ngames, ply_off, d_out, (vb::VBoard*)nullptr, err, d_final);
    if ((e = hipGetLastError()) != hipSuccess) return fail(e);
    if ((e = hipMemcpyAsync(d_group_off, ply_off, (size_t)(ngames + 1) * 4, hipMemcpyDeviceToDevice, s)) !=
        hipSuccess)
      return fail(e);
  } else {
    if ((e = alloc((void**)&states, (size_t)total_plies * sizeof(vb::VBoard))) != hipSuccess) return fail(e);
    if ((e = alloc((void**)&cnt, (size_t)(total_plies + 1) * 4)) != hipSuccess) return fail(e);
    if ((e = alloc((void**)&coff, (size_t)(total_plies + 1) * 4)) != hipSuccess) return fail(e);
    hipLaunchKernelGGL(vreplay_kernel, dim3((ngames + bs - 1) / bs), dim3(bs), 0, s, variant, d_text, d_fen_off,
                       d_mv_off, ngames, ply_off, (fnnue_vpos*)nullptr, states, err, d_final);
    if ((e = hipGetLastError()) != hipSuccess) return fail(e);
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
    if ((e = builder_exclusive_scan(cnt, coff, total_plies, s)) != hipSuccess) return fail(e);
    uint32_t total = 0;
    if ((e = hipMemcpy(&total, coff + total_plies, 4, hipMemcpyDeviceToHost)) != hipSuccess) return fail(e);
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
