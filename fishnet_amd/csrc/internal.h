// internal.h — host-side internals shared by the C ABI translation units
// (capi.cpp: single-device contexts; multi.cpp: one process driving several
// devices over RCCL).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <string>
#include <vector>

#include "../../include/fnnue.h"
#include "builder.h"
#include "kernels.h"
#include "net.h"

struct fnnue_net {
  fnnue::Net net;
  uint8_t sha256[32] = {};  // SHA-256 of the file bytes (net identity, fnnue_net_sha256)
};

struct fnnue_ctx {
  int device = 0;
  uint32_t hd = 0;
  int variant = 0;             // fnnue::kVariant* of the net (chess or a Fairy-Stockfish feature set)
  uint32_t nfeat = 0;          // feature rows of the net
  uint8_t* image = nullptr;
  size_t image_bytes = 0;
  fnnue::NetPtrs ptrs{};
  uint32_t chunk = 0;          // positions per launch pair (chunk_for_hd)
  uint8_t* x = nullptr;        // [chunk][hd] transformed features
  uint8_t* bucket = nullptr;   // [chunk]
  uint32_t* err = nullptr;     // latched position errors
  hipStream_t stream = nullptr;
  // host-API staging
  fnnue_pos* d_pos = nullptr;
  uint32_t* d_off = nullptr;
  int32_t* d_psqt = nullptr;
  int32_t* d_positional = nullptr;
  size_t stage_cap = 0, off_cap = 0;
  char* d_btext = nullptr;     // fnnue_build_batch input staging (text, then FEN / move offsets), grow-only
  size_t btext_cap = 0;
  fnnue::BuilderScratch bscratch;  // the device batch builder's temporaries, grow-only
  int ft_impl = FNNUE_FT_AUTO;
  int32_t acc_bound = 0;       // accumulator_bound of the net (SWAR rows allowed below 2^15)
  fnnue::SlicedPlan plan{};
  fnnue::SegPlan seg{};                // incremental sliced path for groups (allocated on first use)
  int timing = 0;  // FNNUE_TIMING_*: 0 off, 1 every phase, 2 the FT main kernel only
  // per timed launch: before the FT plan, before the FT main kernel, before the
  // layer stacks, after them
  std::vector<std::array<hipEvent_t, 4>> evpool;
  size_t evused = 0;
  // Workspace ordering across streams: every *_device call writes the same
  // workspace (x, bucket, plan, err); it waits for ws_event (recorded by the
  // previous call on its stream) and records ws_event on its own stream.
  hipEvent_t ws_event = nullptr;
  bool ws_recorded = false;
  // The last call ran on `stream` (the context's own, which lives as long as
  // the context) and recorded no event: a call on the same stream needs no
  // ordering, one on another stream records ws_event on `stream` first.
  bool ws_own_pending = false;
  // fnnue_eval_groups_dual_device: this context (the big net) plans, the
  // small net's main kernel and stacks run on the small context's stream
  // between dual_fork (after this net's main kernel) and dual_join.
  hipEvent_t dual_fork = nullptr, dual_join = nullptr;
};


namespace fnnue::detail {

extern thread_local std::string g_err;
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define HIP_TRY(expr, what)                              \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return ::fnnue::detail::hip_fail(_e, what); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

void ctx_destroy(fnnue_ctx* c);
// Allocates a context on `device` for width hd: everything except the image contents.
int ctx_alloc(int device, uint32_t hd, fnnue_ctx** out, int variant);
// Derives the LDS-tile layout of the FT weights from the (just written) image.
int finish_upload(fnnue_ctx* c);
// Grow-only host-API staging: positions (sized for fnnue_vpos) + outputs, offsets.
int ensure_stage(fnnue_ctx* c, size_t npos, size_t noff);
// Grow-only staging of a batch builder's input text and offsets.
int ensure_builder_input(fnnue_ctx* c, size_t bytes);
// Reads and clears the latched device error word.
int latched(fnnue_ctx* c);
// The device's position rule on the host (one king per side, <= 32 pieces, valid codes, stm 0/1).
bool valid_host_pos(const fnnue_pos& p);
// After FNNUE_E_POSITION latched: names the first invalid position.
int name_invalid(int rc, const fnnue_pos* pos, size_t n);
// A variant position as the device sees it: 0 invalid, 1 evaluated, 2 atomic
// game over (one king exploded: result (0, 0), not an error).
int host_vpos_state(const fnnue_vpos& p, int variant);
int name_invalid_v(int rc, const fnnue_vpos* pos, size_t n, int variant, size_t base);
// fnnue_game_end for standard chess (board.cpp rules).
int game_end_chess(const char* fen, const char* moves, int* flags);

}  // namespace fnnue::detail
