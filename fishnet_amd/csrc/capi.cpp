// capi.cpp — the C ABI (include/fnnue.h).  Host runtime: net ownership, device
// contexts (one per GPU, weights resident in HBM), chunked launches, error
// mapping to fishnet's PositionFailed semantics, batch building.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fnnue.h"
#include "board.h"
#include "builder.h"
#include "internal.h"
#include "kernels.h"
#include "net.h"
#include "sha256.h"

using namespace fnnue;
using namespace fnnue::detail;

namespace fnnue::detail {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(FNNUE_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace fnnue::detail

namespace {

// Positions per launch pair: 2^20, fewer for hd > 2047 so the transformed-
// feature workspace (chunk * hd bytes, 1 GiB at hd = 1024) stays inside one
// raw buffer resource (num_records <= 2^31 - 1).
constexpr uint32_t kChunk = 1u << 20;
uint32_t chunk_for_hd(uint32_t hd) {
  return std::min<uint32_t>(kChunk, (0x7FFFFFFFu / hd) & ~1023u);
}

}  // namespace

namespace fnnue::detail {

void ctx_destroy(fnnue_ctx* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  for (auto& quad : c->evpool)
    for (auto e : quad)
      if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {c->ws_event, c->dual_fork, c->dual_join})
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  c->bscratch.release();
  for (void* p : {(void*)c->image, (void*)c->x, (void*)c->bucket, (void*)c->err, (void*)c->d_pos, (void*)c->d_off, (void*)c->d_btext,
                  (void*)c->d_psqt, (void*)c->d_positional, c->plan.tiles, (void*)c->plan.ctr, c->plan.units,
                  (void*)c->plan.items, (void*)c->plan.flist, (void*)c->plan.perm,
                  (void*)c->plan.psqt_part, (void*)c->seg.ref, (void*)c->seg.cref, c->seg.dtmp, c->seg.drec,
                  (void*)c->seg.ipos, (void*)c->seg.len, c->seg.items, c->seg.span, c->seg.scan_temp})
    if (p) (void)hipFree(p);
  delete c;
}

NetPtrs make_ptrs(uint8_t* img, uint32_t hd, uint32_t nfeat) {
  const ImageLayout L = image_layout(hd, nfeat);
  NetPtrs p;
  p.ft_w = reinterpret_cast<const int16_t*>(img + L.ft_w);
  p.ft_bias = reinterpret_cast<const int16_t*>(img + L.ft_bias);
  p.psqt_w = reinterpret_cast<const int32_t*>(img + L.psqt_w);
  p.w0 = reinterpret_cast<const int8_t*>(img + L.w0);
  p.b0 = reinterpret_cast<const int32_t*>(img + L.b0);
  p.w1 = reinterpret_cast<const int8_t*>(img + L.w1);
  p.b1 = reinterpret_cast<const int32_t*>(img + L.b1);
  p.w2 = reinterpret_cast<const int8_t*>(img + L.w2);
  p.b2 = reinterpret_cast<const int32_t*>(img + L.b2);
  return p;
}

// Allocates everything except the image contents.
int ctx_alloc(int device, uint32_t hd, fnnue_ctx** out, int variant) {
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(FNNUE_E_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(FNNUE_E_DEVICE, "device ordinal out of range");
  if (!kernels_support_hd(hd)) return fail(FNNUE_E_ARCH, "no kernel instantiation for hd " + std::to_string(hd));
  if (variant != kVariantChess && hd != 256 && hd != 512 && hd != 1024)
    return fail(FNNUE_E_ARCH, "variant nets: hd 256, 512 or 1024, not " + std::to_string(hd));
  std::unique_ptr<fnnue_ctx, void (*)(fnnue_ctx*)> c(new (std::nothrow) fnnue_ctx, ctx_destroy);
  if (!c) return fail(FNNUE_E_OOM, "host allocation failed");
  c->device = device;
  c->hd = hd;
  c->variant = variant;
  c->nfeat = features_of(variant);
  c->chunk = chunk_for_hd(hd);
  const uint32_t chunk = c->chunk;
  DeviceGuard g(device);
  c->image_bytes = image_layout(hd, c->nfeat).total;
  if (hipMalloc(&c->image, c->image_bytes) != hipSuccess) return fail(FNNUE_E_OOM, "device allocation (net image)");
  if (hipMalloc(&c->x, (size_t)chunk * hd) != hipSuccess) return fail(FNNUE_E_OOM, "device allocation (workspace)");
  if (hipMalloc(&c->bucket, chunk) != hipSuccess) return fail(FNNUE_E_OOM, "device allocation (workspace)");
  if (hipMalloc(&c->err, sizeof(uint32_t)) != hipSuccess) return fail(FNNUE_E_OOM, "device allocation (error word)");
  HIP_TRY(hipMemset(c->err, 0, sizeof(uint32_t)), "hipMemset");
  SlicedPlan& P = c->plan;
  const size_t tiles = variant == kVariantChess ? sliced_tiles_bytes(hd) : variant_tiles_bytes(hd, variant);
  const size_t units = std::max({sliced_max_units(chunk), seg_max_units(chunk), variant_max_units(chunk)});
  if (hipMalloc(&P.tiles, tiles) != hipSuccess ||
      hipMalloc(&P.ctr, std::max({sliced_ctr_words(), variant_ctr_words(), seg_ctr_words()}) * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&P.units, units * 16) != hipSuccess ||
      hipMalloc(&P.items, (size_t)2 * chunk * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&P.flist, (size_t)2 * chunk * 32 * sizeof(uint16_t)) != hipSuccess ||
      hipMalloc(&P.perm, (size_t)chunk * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&P.psqt_part, (size_t)2 * chunk * sizeof(int32_t)) != hipSuccess)
    return fail(FNNUE_E_OOM, "device allocation (sliced plan)");
  if (const char* impl = std::getenv("FNNUE_FT_IMPL"))
    c->ft_impl = std::strcmp(impl, "gather") == 0   ? FNNUE_FT_GATHER
                 : std::strcmp(impl, "sliced") == 0 ? FNNUE_FT_SLICED
                                                    : FNNUE_FT_AUTO;
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
  HIP_TRY(hipEventCreateWithFlags(&c->ws_event, hipEventDisableTiming), "hipEventCreate");
  c->ptrs = make_ptrs(c->image, hd, c->nfeat);
  *out = c.release();
  return FNNUE_OK;
}

int ensure_stage(fnnue_ctx* c, size_t npos, size_t noff) {
  if (npos > c->stage_cap) {
    for (void* p : {(void*)c->d_pos, (void*)c->d_psqt, (void*)c->d_positional})
      if (p) (void)hipFree(p);
    c->d_pos = nullptr;
    c->d_psqt = c->d_positional = nullptr;
    c->stage_cap = 0;
    // sized for the larger record (fnnue_vpos) so both entry points share it
    if (hipMalloc(&c->d_pos, npos * sizeof(fnnue_vpos)) != hipSuccess ||
        hipMalloc(&c->d_psqt, npos * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&c->d_positional, npos * sizeof(int32_t)) != hipSuccess)
      return fail(FNNUE_E_OOM, "device allocation (staging)");
    c->stage_cap = npos;
  }
  if (noff > c->off_cap) {
    if (c->d_off) (void)hipFree(c->d_off);
    c->d_off = nullptr;
    c->off_cap = 0;
    if (hipMalloc(&c->d_off, noff * sizeof(uint32_t)) != hipSuccess)
      return fail(FNNUE_E_OOM, "device allocation (offsets)");
    c->off_cap = noff;
  }
  return FNNUE_OK;
}

// Grow-only staging of fnnue_build_batch's input (text + two offset arrays).
int ensure_builder_input(fnnue_ctx* c, size_t bytes) {
  if (bytes <= c->btext_cap) return FNNUE_OK;
  if (c->d_btext) (void)hipFree(c->d_btext);
  c->d_btext = nullptr;
  c->btext_cap = 0;
  if (hipMalloc(&c->d_btext, bytes) != hipSuccess) return fail(FNNUE_E_OOM, "device allocation (builder input)");
  c->btext_cap = bytes;
  return FNNUE_OK;
}

int latched(fnnue_ctx* c) {
  uint32_t h = 0;
  HIP_TRY(hipMemcpy(&h, c->err, sizeof(h), hipMemcpyDeviceToHost), "hipMemcpy(error word)");
  if (h) {
    HIP_TRY(hipMemset(c->err, 0, sizeof(uint32_t)), "hipMemset");
    if (h & 2u) return fail(FNNUE_E_ARG, "group offsets must be non-decreasing and span [0, npos)");
    return fail(FNNUE_E_POSITION, "batch contains an invalid position (needs one king per side, <= 32 pieces, "
                                  "valid piece codes, stm 0/1)");
  }
  return FNNUE_OK;
}

bool valid_host_pos(const fnnue_pos& p) {
  int n = 0, wk = 0, bk = 0;
  for (int s = 0; s < 64; ++s) {
    const int pc = (p.sq[s >> 1] >> (4 * (s & 1))) & 15;
    if (!pc) continue;
    if (pc == 7 || pc == 8 || pc == 15) return false;
    ++n;
    wk += pc == 6;
    bk += pc == 14;
  }
  return wk == 1 && bk == 1 && n <= 32 && p.stm <= 1;
}

int host_vpos_state(const fnnue_vpos& p, int variant) {
  int n = 0, wk = 0, bk = 0;
  for (int s = 0; s < 64; ++s) {
    const int pc = (p.sq[s >> 1] >> (4 * (s & 1))) & 15;
    if (!pc) continue;
    if (pc == 7 || pc == 8 || pc == 15) return 0;
    ++n;
    wk += pc == 6;
    bk += pc == 14;
  }
  for (int i = 0; i < 10; ++i) {
    if (p.hand[i] > kVHandSlots || (variant != kVariantCrazyhouse && p.hand[i])) return 0;
    n += p.hand[i];
  }
  if (n > 32 || p.stm > 1) return 0;
  if (variant == kVariantAtomic && wk + bk == 1) return 2;
  return wk == 1 && bk == 1 ? 1 : 0;
}

int name_invalid_v(int rc, const fnnue_vpos* pos, size_t n, int variant, size_t base) {
  if (rc != FNNUE_E_POSITION) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!host_vpos_state(pos[i], variant))
      return fail(FNNUE_E_POSITION, "invalid variant position at index " + std::to_string(base + i) +
                                        " (one king per side, or atomic with one king exploded; <= 32 pieces on "
                                        "board and in hand, <= 16 of a type in hand, valid piece codes, stm 0/1)");
  return rc;
}

// After the device latched FNNUE_E_POSITION: the message names the first
// invalid position (the host rule is the device's, valid_host_pos).
int name_invalid(int rc, const fnnue_pos* pos, size_t n) {
  if (rc != FNNUE_E_POSITION) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!valid_host_pos(pos[i])) return fail(FNNUE_E_POSITION, "invalid position at index " + std::to_string(i));
  return rc;
}

// Derives the LDS-tile layout of the FT weights from the (just uploaded) image.
int finish_upload(fnnue_ctx* c) {
  // May ft_slices sum rows as SWAR words?  Decided from the weights on the
  // device (they may come from an RCCL broadcast): a one-off host copy.
  {
    const ImageLayout L = image_layout(c->hd, c->nfeat);
    std::vector<int16_t> w, b;
    try {
      w.resize((size_t)c->nfeat * c->hd);
      b.resize(c->hd);
    } catch (const std::bad_alloc&) {
      return fail(FNNUE_E_OOM, "host allocation failed");
    }
    HIP_TRY(hipMemcpy(w.data(), c->image + L.ft_w, w.size() * 2, hipMemcpyDeviceToHost), "hipMemcpy(ft weights)");
    HIP_TRY(hipMemcpy(b.data(), c->image + L.ft_bias, b.size() * 2, hipMemcpyDeviceToHost), "hipMemcpy(ft bias)");
    c->acc_bound = accumulator_bound(w.data(), b.data(), c->hd, c->variant);
    const char* env = std::getenv("FNNUE_SWAR");
    c->plan.swar = c->acc_bound < 32768 && !(env && env[0] == '0');
  }
  if (c->variant == kVariantChess)
    HIP_TRY(launch_relayout_sliced(c->hd, c->ptrs, c->plan.tiles, c->stream), "relayout launch");
  else
    HIP_TRY(launch_relayout_variant(c->hd, c->variant, c->ptrs, c->plan.tiles, c->stream), "relayout launch");
  HIP_TRY(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  return FNNUE_OK;
}

}  // namespace fnnue::detail

namespace {

// Timing events for the next launch (grown on demand, reused after a read).
int next_events(fnnue_ctx* c, std::array<hipEvent_t, 4>** out) {
  *out = nullptr;
  if (!c->timing) return FNNUE_OK;
  if (c->evused == c->evpool.size()) {
    std::array<hipEvent_t, 4> quad{nullptr, nullptr, nullptr, nullptr};
    // timing only: no system-scope fence (an L2 write-back per record, which
    // the stream waits for between two kernels)
    for (auto& e : quad) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence), "hipEventCreate");
    c->evpool.push_back(quad);
  }
  *out = &c->evpool[c->evused++];
  return FNNUE_OK;
}

int ensure_seg(fnnue_ctx* c) {
  SegPlan& G = c->seg;
  G.unit_plies = seg_unit_plies(c->hd);
  if (G.ref) return FNNUE_OK;
  const size_t n2 = 2 * (size_t)c->chunk;
  G.scan_temp_bytes = seg_scan_temp_bytes(c->chunk);
  if (hipMalloc(&G.ref, (n2 + 1) * 4) != hipSuccess || hipMalloc(&G.cref, (n2 + 1) * 4) != hipSuccess ||
      hipMalloc(&G.dtmp, n2 * 16) != hipSuccess || hipMalloc(&G.drec, n2 * 16 + 16) != hipSuccess ||
      hipMalloc(&G.ipos, n2 * 4) != hipSuccess || hipMalloc(&G.len, n2 * 4) != hipSuccess ||
      hipMalloc(&G.items, n2 * 16) != hipSuccess || hipMalloc(&G.scan_temp, G.scan_temp_bytes + 16) != hipSuccess)
    return fail(FNNUE_E_OOM, "device allocation (segment plan)");
  return FNNUE_OK;
}

// The per-position group span table of a grouped call (8 B per position of
// the call, grow-only: a call above the workspace keeps its whole span table
// in HBM instead of reading its offsets on the host).  Growing frees the old
// table, which hipFree orders after the device's pending work.
int ensure_span(fnnue_ctx* c, size_t npos) {
  SegPlan& G = c->seg;
  const size_t want = std::max<size_t>(npos, c->chunk);
  if (G.span && G.span_cap >= want) return FNNUE_OK;
  if (G.span) (void)hipFree(G.span);
  G.span = nullptr;
  G.span_cap = 0;
  if (hipMalloc(&G.span, want * 8) != hipSuccess) return fail(FNNUE_E_OOM, "device allocation (group spans)");
  G.span_cap = want;
  return FNNUE_OK;
}

// Records timing event k of a chunk (0: before the plan, 1: before the FT
// main kernel, 2: before the stacks, 3: after them); FNNUE_TIMING_FT records
// only events 1 and 2.
int record_event(const fnnue_ctx* c, std::array<hipEvent_t, 4>* ev, int k, hipStream_t s) {
  if (!ev || (c->timing == FNNUE_TIMING_FT && (k == 0 || k == 3))) return FNNUE_OK;
  HIP_TRY(hipEventRecord((*ev)[k], s), "hipEventRecord");
  return FNNUE_OK;
}

// Runs the stack kernel for [0, n) of the workspace and records timing.
int run_chunk_tail(fnnue_ctx* c, uint32_t n, int32_t* d_positional, hipStream_t s, std::array<hipEvent_t, 4>* ev,
                   const uint32_t* perm = nullptr, const int32_t* psqt_part = nullptr, int32_t* d_psqt = nullptr) {
  if (int rc = record_event(c, ev, 2, s)) return rc;
  HIP_TRY(launch_stack(c->hd, c->x, c->bucket, n, c->ptrs, d_positional, perm, psqt_part, d_psqt, s),
          "stack kernel launch");
  return record_event(c, ev, 3, s);
}

// Workspace ordering across streams (the workspace is shared by every call on
// a ctx): a call on a caller's stream records ws_event on it when its work is
// enqueued (also after an error: part of it may be), and each call first
// waits for that event.  No caller stream handle of an earlier call is ever
// used again, so a caller may destroy a stream right after a call on it.  A
// call on the context's own stream records nothing (an event record between
// two kernels idles the stream for microseconds): the next call on the same
// stream is ordered by the stream, and a call on another stream records
// ws_event on the own stream, which lives as long as the context, first.
struct WorkspaceUse {
  fnnue_ctx* c;
  hipStream_t s;
  ~WorkspaceUse() {
    if (s == c->stream) {
      c->ws_own_pending = true;
    } else if (hipEventRecord(c->ws_event, s) == hipSuccess) {
      c->ws_recorded = true;
      c->ws_own_pending = false;
    } else {
      // No event for this call's work: the stale one (an earlier call's) would
      // let the next call on another stream overwrite the workspace while this
      // one still reads it.  Wait for the work instead (a destructor cannot
      // return the error; the ordering is what must hold).
      (void)hipStreamSynchronize(s);
      c->ws_recorded = false;
      c->ws_own_pending = false;
    }
  }
};

int order_workspace(fnnue_ctx* c, hipStream_t s) {
  if (c->ws_own_pending) {
    if (s == c->stream) return FNNUE_OK;
    HIP_TRY(hipEventRecord(c->ws_event, c->stream), "hipEventRecord");
    c->ws_recorded = true;
    c->ws_own_pending = false;
  }
  if (c->ws_recorded) HIP_TRY(hipStreamWaitEvent(s, c->ws_event, 0), "hipStreamWaitEvent");
  return FNNUE_OK;
}

hipEvent_t mid_event(std::array<hipEvent_t, 4>* ev) { return ev ? (*ev)[1] : nullptr; }

}  // namespace

extern "C" {

const char* fnnue_last_error(void) { return g_err.c_str(); }
uint32_t fnnue_abi_version(void) { return (3u << 16) | 1u; }  // 3.1: fnnue_backend_go_timeout, FNNUE_E_TIMEOUT

int fnnue_net_load_mem(const void* buf, size_t len, fnnue_net** out) {
  if (!buf || !out) return fail(FNNUE_E_ARG, "null argument");
  *out = nullptr;
  std::unique_ptr<fnnue_net> n(new (std::nothrow) fnnue_net);
  if (!n) return fail(FNNUE_E_OOM, "host allocation failed");
  std::string err;
  try {
    const int rc = parse_net(static_cast<const uint8_t*>(buf), len, n->net, err);
    if (rc) return fail(rc, err);
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  sha256(static_cast<const uint8_t*>(buf), len, n->sha256);
  *out = n.release();
  return FNNUE_OK;
}

int fnnue_net_load_variant_mem(const void* buf, size_t len, int variant, fnnue_net** out) {
  if (!buf || !out) return fail(FNNUE_E_ARG, "null argument");
  *out = nullptr;
  if (variant != FNNUE_VARIANT_CRAZYHOUSE && variant != FNNUE_VARIANT_ATOMIC)
    return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  std::unique_ptr<fnnue_net> n(new (std::nothrow) fnnue_net);
  if (!n) return fail(FNNUE_E_OOM, "host allocation failed");
  std::string err;
  try {
    const int rc = parse_net(static_cast<const uint8_t*>(buf), len, n->net, err, variant);
    if (rc) return fail(rc, err);
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  sha256(static_cast<const uint8_t*>(buf), len, n->sha256);
  *out = n.release();
  return FNNUE_OK;
}

namespace {

int read_file(const char* path, std::vector<uint8_t>& buf) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) return fail(FNNUE_E_IO, std::string("cannot open ") + path);
  const std::streamsize len = f.tellg();
  f.seekg(0);
  try {
    buf.resize((size_t)len);
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  if (!f.read(reinterpret_cast<char*>(buf.data()), len)) return fail(FNNUE_E_IO, std::string("cannot read ") + path);
  return FNNUE_OK;
}

// Net identity: a file named nn-<12 hex>.nnue claims that its SHA-256 starts
// with those digits (upstream's net naming; [ref] build.rs:7 pins
// nn-ad9b42354671.nnue and build.rs:100-112 deletes a corrupt download).
// A mismatch is a corrupt or renamed file: FNNUE_E_FORMAT, the net freed.
int check_identity(const char* path, fnnue_net** out) {
  const std::string claim = net_name_digest_prefix(path);
  if (claim.empty()) return FNNUE_OK;
  const std::string got = hex_lower((*out)->sha256, 32);
  if (got.compare(0, 12, claim) == 0) return FNNUE_OK;
  fnnue_net_free(*out);
  *out = nullptr;
  return fail(FNNUE_E_FORMAT, std::string(path) + ": SHA-256 " + got.substr(0, 12) + "... does not match the name's " +
                                  claim + " (corrupt or renamed net file)");
}

}  // namespace

int fnnue_net_load_variant(const char* path, int variant, fnnue_net** out) {
  if (!path || !out) return fail(FNNUE_E_ARG, "null argument");
  *out = nullptr;
  std::vector<uint8_t> buf;
  if (int rc = read_file(path, buf)) return rc;
  if (int rc = fnnue_net_load_variant_mem(buf.data(), buf.size(), variant, out)) return rc;
  return check_identity(path, out);
}

int fnnue_net_variant(const fnnue_net* net, int* variant) {
  if (!net || !variant) return fail(FNNUE_E_ARG, "null argument");
  *variant = net->net.variant;
  return FNNUE_OK;
}

int fnnue_net_load(const char* path, fnnue_net** out) {
  if (!path || !out) return fail(FNNUE_E_ARG, "null argument");
  *out = nullptr;
  std::vector<uint8_t> buf;
  if (int rc = read_file(path, buf)) return rc;
  if (int rc = fnnue_net_load_mem(buf.data(), buf.size(), out)) return rc;
  return check_identity(path, out);
}

int fnnue_net_sha256(const fnnue_net* net, uint8_t* digest) {
  if (!net || !digest) return fail(FNNUE_E_ARG, "null argument");
  std::memcpy(digest, net->sha256, 32);
  return FNNUE_OK;
}

int fnnue_net_info(const fnnue_net* net, uint32_t* hd, uint32_t* file_hash, const char** desc) {
  if (!net) return fail(FNNUE_E_ARG, "null net");
  if (hd) *hd = net->net.hd;
  if (file_hash) *file_hash = net->net.file_hash;
  if (desc) *desc = net->net.desc.c_str();
  return FNNUE_OK;
}

void fnnue_net_free(fnnue_net* net) { delete net; }

int fnnue_net_synthesize(uint64_t seed, uint32_t hd, uint32_t flags, void** buf, size_t* len) {
  if (!buf || !len) return fail(FNNUE_E_ARG, "null argument");
  if (!hd_supported(hd)) return fail(FNNUE_E_ARCH, "unsupported hd");
  try {
    Net n;
    synthesize_net(seed, hd, flags, n);
    std::vector<uint8_t> bytes;
    write_net(n, flags & FNNUE_SYNTH_LEB128, bytes);
    void* p = std::malloc(bytes.size());
    if (!p) return fail(FNNUE_E_OOM, "host allocation failed");
    std::memcpy(p, bytes.data(), bytes.size());
    *buf = p;
    *len = bytes.size();
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  return FNNUE_OK;
}

int fnnue_net_synthesize_variant(uint64_t seed, uint32_t hd, int variant, uint32_t flags, void** buf, size_t* len) {
  if (!buf || !len) return fail(FNNUE_E_ARG, "null argument");
  if (variant != FNNUE_VARIANT_CRAZYHOUSE && variant != FNNUE_VARIANT_ATOMIC)
    return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  if (!hd_supported(hd)) return fail(FNNUE_E_ARCH, "unsupported hd");
  try {
    Net n;
    synthesize_net(seed, hd, flags, n, variant);
    std::vector<uint8_t> bytes;
    write_net(n, flags & FNNUE_SYNTH_LEB128, bytes);
    void* p = std::malloc(bytes.size());
    if (!p) return fail(FNNUE_E_OOM, "host allocation failed");
    std::memcpy(p, bytes.data(), bytes.size());
    *buf = p;
    *len = bytes.size();
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  return FNNUE_OK;
}

void fnnue_buffer_free(void* buf) { std::free(buf); }

int fnnue_device_count(int* count) {
  if (!count) return fail(FNNUE_E_ARG, "null argument");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return FNNUE_OK;
}

int fnnue_net_image_size(const fnnue_net* net, size_t* bytes) {
  if (!net || !bytes) return fail(FNNUE_E_ARG, "null argument");
  *bytes = image_layout(net->net.hd, net->net.nfeat).total;
  return FNNUE_OK;
}

int fnnue_net_image_pack(const fnnue_net* net, void* host_buf, size_t bytes) {
  if (!net || !host_buf) return fail(FNNUE_E_ARG, "null argument");
  if (bytes < image_layout(net->net.hd, net->net.nfeat).total) return fail(FNNUE_E_CAPACITY, "image buffer too small");
  pack_image(net->net, static_cast<uint8_t*>(host_buf));
  return FNNUE_OK;
}

int fnnue_ctx_create(const fnnue_net* net, int device, fnnue_ctx** out) {
  if (!net || !out) return fail(FNNUE_E_ARG, "null argument");
  fnnue_ctx* c = nullptr;
  int rc = ctx_alloc(device, net->net.hd, &c, net->net.variant);
  if (rc) return rc;
  std::vector<uint8_t> img;
  try {
    img.resize(c->image_bytes);
  } catch (const std::bad_alloc&) {
    ctx_destroy(c);
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  pack_image(net->net, img.data());
  DeviceGuard g(device);
  hipError_t e = hipMemcpy(c->image, img.data(), img.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    ctx_destroy(c);
    return hip_fail(e, "hipMemcpy(net image)");
  }
  if ((rc = finish_upload(c)) != FNNUE_OK) {
    ctx_destroy(c);
    return rc;
  }
  *out = c;
  return FNNUE_OK;
}

int fnnue_ctx_create_from_image(int device, uint32_t hd, const void* device_image, size_t bytes, fnnue_ctx** out) {
  if (!device_image || !out) return fail(FNNUE_E_ARG, "null argument");
  if (!hd_supported(hd)) return fail(FNNUE_E_ARCH, "unsupported hd");
  if (bytes != image_layout(hd).total) return fail(FNNUE_E_ARG, "image size does not match hd");
  fnnue_ctx* c = nullptr;
  int rc = ctx_alloc(device, hd, &c, kVariantChess);
  if (rc) return rc;
  DeviceGuard g(device);
  hipError_t e = hipMemcpy(c->image, device_image, bytes, hipMemcpyDeviceToDevice);
  if (e != hipSuccess) {
    ctx_destroy(c);
    return hip_fail(e, "hipMemcpy(device image)");
  }
  if ((rc = finish_upload(c)) != FNNUE_OK) {
    ctx_destroy(c);
    return rc;
  }
  *out = c;
  return FNNUE_OK;
}

int fnnue_ctx_image(fnnue_ctx* ctx, const void** device_image, size_t* bytes) {
  if (!ctx || !device_image || !bytes) return fail(FNNUE_E_ARG, "null argument");
  *device_image = ctx->image;
  *bytes = ctx->image_bytes;
  return FNNUE_OK;
}

void fnnue_ctx_free(fnnue_ctx* ctx) { ctx_destroy(ctx); }

int fnnue_ctx_set_ft_impl(fnnue_ctx* ctx, int impl) {
  if (!ctx || (impl != FNNUE_FT_SLICED && impl != FNNUE_FT_GATHER && impl != FNNUE_FT_AUTO))
    return fail(FNNUE_E_ARG, "bad ft impl");
  ctx->ft_impl = impl;
  return FNNUE_OK;
}

int fnnue_ctx_swar(const fnnue_ctx* ctx, int* enabled, int32_t* bound) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (enabled) *enabled = ctx->plan.swar ? 1 : 0;
  if (bound) *bound = ctx->acc_bound;
  return FNNUE_OK;
}

int fnnue_ctx_set_swar(fnnue_ctx* ctx, int enable) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (enable && ctx->acc_bound >= 32768)
    return fail(FNNUE_E_ARCH, "accumulator bound " + std::to_string(ctx->acc_bound) + " >= 2^15: SWAR rows not exact");
  ctx->plan.swar = enable != 0;
  return FNNUE_OK;
}

int fnnue_net_accumulator_bound(const fnnue_net* net, int32_t* bound) {
  if (!net || !bound) return fail(FNNUE_E_ARG, "null argument");
  *bound = accumulator_bound(net->net.ft_w.data(), net->net.ft_bias.data(), net->net.hd, net->net.variant);
  return FNNUE_OK;
}

int fnnue_ctx_set_timing(fnnue_ctx* ctx, int enable) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  ctx->timing = enable == FNNUE_TIMING_FT ? FNNUE_TIMING_FT : enable ? FNNUE_TIMING_ALL : FNNUE_TIMING_OFF;
  ctx->evused = 0;
  return FNNUE_OK;
}

int fnnue_ctx_timing_phases(fnnue_ctx* ctx, uint32_t* launches, double* plan_ms, double* ft_ms, double* stack_ms) {
  if (!ctx || !launches || !plan_ms || !ft_ms || !stack_ms) return fail(FNNUE_E_ARG, "null argument");
  *launches = 0;
  *plan_ms = *ft_ms = *stack_ms = 0;
  DeviceGuard g(ctx->device);
  for (size_t i = 0; i < ctx->evused; ++i) {
    auto& e = ctx->evpool[i];
    float a = 0, b = 0, c = 0;
    const bool all = ctx->timing != FNNUE_TIMING_FT;
    HIP_TRY(hipEventSynchronize(all ? e[3] : e[2]), "hipEventSynchronize");
    if (all) HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]), "hipEventElapsedTime");
    HIP_TRY(hipEventElapsedTime(&b, e[1], e[2]), "hipEventElapsedTime");
    if (all) HIP_TRY(hipEventElapsedTime(&c, e[2], e[3]), "hipEventElapsedTime");
    *plan_ms += a;
    *ft_ms += b;
    *stack_ms += c;
  }
  *launches = (uint32_t)ctx->evused;
  ctx->evused = 0;
  return FNNUE_OK;
}

int fnnue_ctx_timing_read(fnnue_ctx* ctx, uint32_t* launches, double* ft_ms, double* stack_ms) {
  if (!ctx || !launches || !ft_ms || !stack_ms) return fail(FNNUE_E_ARG, "null argument");
  double plan = 0, ft = 0;
  const int rc = fnnue_ctx_timing_phases(ctx, launches, &plan, &ft, stack_ms);
  *ft_ms = plan + ft;
  return rc;
}

int fnnue_eval_positions_device(fnnue_ctx* ctx, const fnnue_pos* d_pos, size_t n, int32_t* d_psqt,
                                int32_t* d_positional, void* stream) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (ctx->variant != kVariantChess) return fail(FNNUE_E_ARCH, "variant net: use fnnue_eval_vpositions*");
  if (n == 0) return FNNUE_OK;
  if (!d_pos || !d_psqt || !d_positional) return fail(FNNUE_E_ARG, "null buffer");
  DeviceGuard g(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  int rc = order_workspace(ctx, s);
  if (rc) return rc;
  WorkspaceUse use{ctx, s};
  // FNNUE_FT_AUTO: a call of at most FNNUE_FT_GATHER_MAX positions gathers
  // (the sliced path's plan and tile loads are a fixed cost it cannot amortise)
  const bool gather = ctx->ft_impl == FNNUE_FT_GATHER || (ctx->ft_impl == FNNUE_FT_AUTO && n <= FNNUE_FT_GATHER_MAX);
  for (size_t b = 0; b < n; b += ctx->chunk) {
    const uint32_t m = (uint32_t)std::min<size_t>(ctx->chunk, n - b);
    std::array<hipEvent_t, 4>* ev = nullptr;
    rc = next_events(ctx, &ev);
    if (rc) return rc;
    if ((rc = record_event(ctx, ev, 0, s))) return rc;
    const uint32_t* perm = nullptr;
    const int32_t* psqt_part = nullptr;
    if (gather) {
      if ((rc = record_event(ctx, ev, 1, s))) return rc;
      HIP_TRY(launch_ft_scratch(ctx->hd, d_pos + b, m, ctx->ptrs, ctx->x, d_psqt + b, ctx->bucket, ctx->err, s),
              "ft_scratch launch");
    } else {
      HIP_TRY(launch_ft_sliced(ctx->hd, d_pos + b, m, ctx->ptrs, ctx->plan, ctx->x, d_psqt + b, ctx->bucket,
                               ctx->err, s, mid_event(ev)),
              "ft_sliced launch");
      perm = ctx->plan.perm;
      psqt_part = ctx->plan.psqt_part;
    }
    rc = run_chunk_tail(ctx, m, d_positional + b, s, ev, perm, psqt_part, d_psqt + b);
    if (rc) return rc;
  }
  return FNNUE_OK;
}

}  // extern "C"

namespace {

// Grouped evaluation on the device (chess or a variant feature set): the
// offsets stay on the device (no D2H, no stream drain, at any size): they are
// checked there (group_span_kernel, latched as FNNUE_E_ARG), and a call above
// one workspace is cut into chunks at fixed positions; a group cut by a chunk
// boundary restarts there with a refresh (results are identical).
int eval_groups_device(fnnue_ctx* ctx, const void* d_pos, size_t pos_bytes, const uint32_t* d_off, size_t ngroups,
                       size_t npos, int mode, int32_t* d_psqt, int32_t* d_positional, void* stream) {
  if (mode != FNNUE_GROUP_CHAIN && mode != FNNUE_GROUP_STAR) return fail(FNNUE_E_ARG, "bad group mode");
  if (ngroups == 0) return npos == 0 ? FNNUE_OK : fail(FNNUE_E_ARG, "positions without groups");
  if (ngroups > 0xFFFFFFFFu || npos > 0xFFFFFFFFu) return fail(FNNUE_E_ARG, "batch too large");
  if (!d_pos || !d_off || !d_psqt || !d_positional) return fail(FNNUE_E_ARG, "null buffer");
  DeviceGuard g(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  int rc = order_workspace(ctx, s);
  if (rc) return rc;
  WorkspaceUse use{ctx, s};
  const bool sliced = ctx->ft_impl != FNNUE_FT_GATHER || ctx->variant != kVariantChess;
  if (sliced && ((rc = ensure_seg(ctx)) || (rc = ensure_span(ctx, npos)))) return rc;
  if (sliced && npos <= seg_small_plan_max()) {
    // a small call (a game or a few): spans, the offset check and the whole
    // plan in one workgroup, then the main kernel and the stacks
    std::array<hipEvent_t, 4>* ev = nullptr;
    if ((rc = next_events(ctx, &ev)) || (rc = record_event(ctx, ev, 0, s))) return rc;
    HIP_TRY(launch_seg_plan_small(ctx->variant, d_pos, (uint32_t)npos, d_off, (uint32_t)ngroups, ctx->seg.span, mode,
                                  ctx->plan, ctx->seg, ctx->bucket, ctx->err, s),
            "segment plan launch");
    if ((rc = record_event(ctx, ev, 1, s))) return rc;
    HIP_TRY(launch_seg_ft(ctx->hd, ctx->variant, (uint32_t)npos, mode, ctx->ptrs, ctx->plan, ctx->seg, ctx->x, s),
            "ft_segments launch");
    return run_chunk_tail(ctx, (uint32_t)npos, d_positional, s, ev, nullptr, ctx->plan.psqt_part, d_psqt);
  }
  HIP_TRY(launch_group_span(d_off, (uint32_t)ngroups, (uint32_t)npos, sliced ? ctx->seg.span : nullptr, true,
                            ctx->err, s),
          "group_span launch");
  const uint2* span = static_cast<const uint2*>(ctx->seg.span);
  const char* pos = static_cast<const char*>(d_pos);
  for (size_t b = 0; b < npos; b += ctx->chunk) {
    const uint32_t m = (uint32_t)std::min<size_t>(ctx->chunk, npos - b);
    std::array<hipEvent_t, 4>* ev = nullptr;
    if ((rc = next_events(ctx, &ev))) return rc;
    if ((rc = record_event(ctx, ev, 0, s))) return rc;
    if (sliced) {
      HIP_TRY(launch_ft_segments(ctx->hd, ctx->variant, pos + b * pos_bytes, m, span + b, (uint32_t)b, mode,
                                 ctx->ptrs, ctx->plan, ctx->seg, ctx->x, ctx->bucket, ctx->err, s, mid_event(ev)),
              "ft_segments launch");
      rc = run_chunk_tail(ctx, m, d_positional + b, s, ev, nullptr, ctx->plan.psqt_part, d_psqt + b);
    } else {
      if ((rc = record_event(ctx, ev, 1, s))) return rc;
      HIP_TRY(launch_ft_groups(ctx->hd, static_cast<const fnnue_pos*>(d_pos), d_off, (uint32_t)ngroups, (uint32_t)b,
                               (uint32_t)(b + m), mode, ctx->ptrs, ctx->x, d_psqt + b, ctx->bucket, ctx->err, s),
              "ft_groups launch");
      rc = run_chunk_tail(ctx, m, d_positional + b, s, ev);
    }
    if (rc) return rc;
  }
  return FNNUE_OK;
}

// Big + small net over the same CHAIN / STAR batch ("dual NNUE": both nets
// read the same HalfKAv2_hm features and update their accumulators from the
// same deltas, upstream evaluate_nnue.cpp with two networks).  The plan
// (group spans, deltas, segments, lists, units) is built once in the big
// context's workspace on the call's stream s; then s forks: the small net's
// main kernel and stacks run on the small context's stream over that plan
// while s runs the big net's main kernel and stacks (the small net's few
// hundred (unit, slice) workgroups interleave with the big net's thousands on
// the CUs), and s joins before the next chunk's plan overwrites what the small
// FT reads.  (Forking after the big net's main kernel instead, so that the
// small FT ran beside the big net's stacks only, measured 878M against 928M
// plies/s for two independent calls: the small FT then sat on the critical
// path.)
int eval_groups_dual_device(fnnue_ctx* a, fnnue_ctx* b, const fnnue_pos* d_pos, const uint32_t* d_off, size_t ngroups,
                            size_t npos, int mode, int32_t* d_psqt, int32_t* d_positional, int32_t* d_psqt2,
                            int32_t* d_positional2, void* stream) {
  if (!a || !b) return fail(FNNUE_E_ARG, "null ctx");
  if (a == b) return fail(FNNUE_E_ARG, "the two nets need two contexts");
  if (a->variant != kVariantChess || b->variant != kVariantChess)
    return fail(FNNUE_E_ARCH, "dual evaluation: two chess (HalfKAv2_hm) nets");
  if (a->device != b->device) return fail(FNNUE_E_ARG, "the two contexts must be on one device");
  if (a->ft_impl == FNNUE_FT_GATHER || b->ft_impl == FNNUE_FT_GATHER)
    return fail(FNNUE_E_ARG, "dual evaluation runs on the sliced feature transformer");
  if (mode != FNNUE_GROUP_CHAIN && mode != FNNUE_GROUP_STAR) return fail(FNNUE_E_ARG, "bad group mode");
  if (ngroups == 0) return npos == 0 ? FNNUE_OK : fail(FNNUE_E_ARG, "positions without groups");
  if (ngroups > 0xFFFFFFFFu || npos > 0xFFFFFFFFu) return fail(FNNUE_E_ARG, "batch too large");
  if (!d_pos || !d_off || !d_psqt || !d_positional || !d_psqt2 || !d_positional2)
    return fail(FNNUE_E_ARG, "null buffer");
  DeviceGuard g(a->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : a->stream;
  hipStream_t s2 = b->stream;
  int rc = order_workspace(a, s);
  if (rc || (rc = order_workspace(b, s2))) return rc;
  WorkspaceUse use_a{a, s};
  WorkspaceUse use_b{b, s2};
  if ((rc = ensure_seg(a)) || (rc = ensure_span(a, npos))) return rc;
  for (fnnue_ctx* c : {a})
    for (hipEvent_t* e : {&c->dual_fork, &c->dual_join})
      if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
  HIP_TRY(launch_group_span(d_off, (uint32_t)ngroups, (uint32_t)npos, a->seg.span, true, a->err, s),
          "group_span launch");
  const uint2* span = static_cast<const uint2*>(a->seg.span);
  const uint32_t chunk = std::min(a->chunk, b->chunk);
  // the small net over the big context's plan: its own tiles, SWAR flag and PSQT parts
  SlicedPlan pb = a->plan;
  pb.tiles = b->plan.tiles;
  pb.swar = b->plan.swar;
  pb.psqt_part = b->plan.psqt_part;
  // A small net (HD <= 256) works best on units of half the plies (§4.4): it
  // gets a unit table of its own, cut from the same sorted items into its own
  // context's unit buffer and counter.
  const uint32_t small_plies = seg_unit_plies(b->hd);
  const bool own_units = small_plies != a->seg.unit_plies;
  if (own_units) {
    pb.units = b->plan.units;
    pb.ctr = b->plan.ctr;
  }
  for (size_t i0 = 0; i0 < npos; i0 += chunk) {
    const uint32_t m = (uint32_t)std::min<size_t>(chunk, npos - i0);
    std::array<hipEvent_t, 4>*ev = nullptr, *ev2 = nullptr;
    if ((rc = next_events(a, &ev)) || (rc = next_events(b, &ev2))) return rc;
    if ((rc = record_event(a, ev, 0, s))) return rc;
    HIP_TRY(launch_seg_plan(kVariantChess, d_pos + i0, m, span + i0, (uint32_t)i0, mode, a->plan, a->seg, a->bucket,
                            a->err, s),
            "segment plan launch");
    HIP_TRY(hipEventRecord(a->dual_fork, s), "hipEventRecord");
    HIP_TRY(hipStreamWaitEvent(s2, a->dual_fork, 0), "hipStreamWaitEvent");
    // From the fork on, s must wait for s2 before returning, error or not
    // (ADVICE r04): the next call on `a` overwrites the plan the small net's
    // kernels on s2 read.
    auto forked = [&]() -> int {
      // (on the small context's stream: its unit buffer and counter are
      // written in that context's workspace order)
      if (own_units)
        HIP_TRY(launch_seg_units(kVariantChess, a->plan, pb.units, pb.ctr, small_plies, s2), "segment units launch");
      int r = record_event(a, ev, 1, s);
      if (r) return r;
      HIP_TRY(launch_seg_ft(a->hd, kVariantChess, m, mode, a->ptrs, a->plan, a->seg, a->x, s), "ft_segments launch");
      // the small net has no plan of its own: its plan phase is empty
      if ((r = record_event(b, ev2, 0, s2)) || (r = record_event(b, ev2, 1, s2))) return r;
      HIP_TRY(launch_seg_ft(b->hd, kVariantChess, m, mode, b->ptrs, pb, a->seg, b->x, s2), "ft_segments launch");
      if ((r = record_event(b, ev2, 2, s2))) return r;
      HIP_TRY(launch_stack(b->hd, b->x, a->bucket, m, b->ptrs, d_positional2 + i0, nullptr, b->plan.psqt_part,
                           d_psqt2 + i0, s2),
              "stack kernel launch");
      if ((r = record_event(b, ev2, 3, s2))) return r;
      return run_chunk_tail(a, m, d_positional + i0, s, ev, nullptr, a->plan.psqt_part, d_psqt + i0);
    };
    rc = forked();
    if (hipEventRecord(a->dual_join, s2) != hipSuccess || hipStreamWaitEvent(s, a->dual_join, 0) != hipSuccess) {
      (void)hipStreamSynchronize(s2);  // no event to order by: the small net's work is done before s goes on
      if (!rc) rc = fail(FNNUE_E_DEVICE, "dual join event failed");
    }
    if (rc) return rc;
  }
  return FNNUE_OK;
}

}  // namespace

extern "C" {

int fnnue_eval_groups_dual_device(fnnue_ctx* big, fnnue_ctx* small, const fnnue_pos* d_pos, const uint32_t* d_off,
                                  size_t ngroups, size_t npos, int mode, int32_t* d_psqt, int32_t* d_positional,
                                  int32_t* d_psqt_small, int32_t* d_positional_small, void* stream) {
  return eval_groups_dual_device(big, small, d_pos, d_off, ngroups, npos, mode, d_psqt, d_positional, d_psqt_small,
                                 d_positional_small, stream);
}

int fnnue_eval_groups_device(fnnue_ctx* ctx, const fnnue_pos* d_pos, const uint32_t* d_off, size_t ngroups,
                             size_t npos, int mode, int32_t* d_psqt, int32_t* d_positional, void* stream) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (ctx->variant != kVariantChess) return fail(FNNUE_E_ARCH, "variant net: use fnnue_eval_vgroups*");
  return eval_groups_device(ctx, d_pos, sizeof(fnnue_pos), d_off, ngroups, npos, mode, d_psqt, d_positional, stream);
}

int fnnue_eval_vgroups_device(fnnue_ctx* ctx, const fnnue_vpos* d_pos, const uint32_t* d_off, size_t ngroups,
                              size_t npos, int mode, int32_t* d_psqt, int32_t* d_positional, void* stream) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (ctx->variant == kVariantChess) return fail(FNNUE_E_ARCH, "chess net: use fnnue_eval_groups*");
  return eval_groups_device(ctx, d_pos, sizeof(fnnue_vpos), d_off, ngroups, npos, mode, d_psqt, d_positional, stream);
}

int fnnue_eval_vpositions_device(fnnue_ctx* ctx, const fnnue_vpos* d_pos, size_t n, int32_t* d_psqt,
                                 int32_t* d_positional, void* stream) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (ctx->variant == kVariantChess) return fail(FNNUE_E_ARCH, "chess net: use fnnue_eval_positions*");
  if (n == 0) return FNNUE_OK;
  if (!d_pos || !d_psqt || !d_positional) return fail(FNNUE_E_ARG, "null buffer");
  DeviceGuard g(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  int rc = order_workspace(ctx, s);
  if (rc) return rc;
  WorkspaceUse use{ctx, s};
  for (size_t b = 0; b < n; b += ctx->chunk) {
    const uint32_t m = (uint32_t)std::min<size_t>(ctx->chunk, n - b);
    std::array<hipEvent_t, 4>* ev = nullptr;
    if ((rc = next_events(ctx, &ev))) return rc;
    if ((rc = record_event(ctx, ev, 0, s))) return rc;
    HIP_TRY(launch_variant_plan(d_pos + b, m, ctx->variant, ctx->plan, d_psqt + b, ctx->bucket, ctx->err, s),
            "variant plan launch");
    if ((rc = record_event(ctx, ev, 1, s))) return rc;
    HIP_TRY(launch_variant_ft(ctx->hd, ctx->variant, m, ctx->ptrs, ctx->plan, ctx->x, s), "variant ft launch");
    if ((rc = run_chunk_tail(ctx, m, d_positional + b, s, ev, ctx->plan.perm, ctx->plan.psqt_part, d_psqt + b)))
      return rc;
  }
  return FNNUE_OK;
}

int fnnue_eval_vpositions(fnnue_ctx* ctx, const fnnue_vpos* pos, size_t n, int32_t* psqt, int32_t* positional) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (ctx->variant == kVariantChess) return fail(FNNUE_E_ARCH, "chess net: use fnnue_eval_positions*");
  if (n == 0) return FNNUE_OK;
  if (!pos || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  DeviceGuard g(ctx->device);
  const size_t step = std::min<size_t>(n, 4 * (size_t)ctx->chunk);
  int rc = ensure_stage(ctx, step, 0);
  if (rc) return rc;
  fnnue_vpos* d_vpos = reinterpret_cast<fnnue_vpos*>(ctx->d_pos);  // staging sized for fnnue_vpos
  for (size_t b = 0; b < n; b += step) {
    const size_t m = std::min(step, n - b);
    HIP_TRY(hipMemcpyAsync(d_vpos, pos + b, m * sizeof(fnnue_vpos), hipMemcpyHostToDevice, ctx->stream), "H2D");
    rc = fnnue_eval_vpositions_device(ctx, d_vpos, m, ctx->d_psqt, ctx->d_positional, ctx->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(psqt + b, ctx->d_psqt, m * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
    HIP_TRY(hipMemcpyAsync(positional + b, ctx->d_positional, m * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
    HIP_TRY(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if ((rc = latched(ctx))) return name_invalid_v(rc, pos + b, m, ctx->variant, b);
  }
  return FNNUE_OK;
}

int fnnue_ctx_check(fnnue_ctx* ctx) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  DeviceGuard g(ctx->device);
  // Only this context's work: its own stream, and the last *_device call
  // (whatever stream it ran on; calls are chained by ws_event, so the last
  // one's completion implies every earlier one's).  Other streams of the
  // device (other contexts, torch) are not drained.
  HIP_TRY(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
  if (ctx->ws_recorded) HIP_TRY(hipEventSynchronize(ctx->ws_event), "hipEventSynchronize");
  return latched(ctx);
}

int fnnue_eval_positions(fnnue_ctx* ctx, const fnnue_pos* pos, size_t n, int32_t* psqt, int32_t* positional) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (n == 0) return FNNUE_OK;
  if (!pos || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  // Positions are validated on the device (latched error word): the host
  // scans them only to name the first bad index once an error is latched.
  DeviceGuard g(ctx->device);
  const size_t step = std::min<size_t>(n, 4 * (size_t)ctx->chunk);
  int rc = ensure_stage(ctx, step, 0);
  if (rc) return rc;
  for (size_t b = 0; b < n; b += step) {
    const size_t m = std::min(step, n - b);
    HIP_TRY(hipMemcpyAsync(ctx->d_pos, pos + b, m * sizeof(fnnue_pos), hipMemcpyHostToDevice, ctx->stream), "H2D");
    rc = fnnue_eval_positions_device(ctx, ctx->d_pos, m, ctx->d_psqt, ctx->d_positional, ctx->stream);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(psqt + b, ctx->d_psqt, m * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
    HIP_TRY(hipMemcpyAsync(positional + b, ctx->d_positional, m * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
    HIP_TRY(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    rc = latched(ctx);
    if (rc) return name_invalid(rc, pos, n);
  }
  return FNNUE_OK;
}

int fnnue_eval_groups(fnnue_ctx* ctx, const fnnue_pos* pos, size_t npos, const uint32_t* off, size_t ngroups,
                      int mode, int32_t* psqt, int32_t* positional) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (mode != FNNUE_GROUP_CHAIN && mode != FNNUE_GROUP_STAR) return fail(FNNUE_E_ARG, "bad group mode");
  if (ngroups == 0) return npos == 0 ? FNNUE_OK : fail(FNNUE_E_ARG, "positions without groups");
  if (ngroups > 0xFFFFFFFFu || npos > 0xFFFFFFFFu) return fail(FNNUE_E_ARG, "batch too large");
  if (!pos || !off || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  if (off[0] != 0) return fail(FNNUE_E_ARG, "off[0] must be 0");
  for (size_t g = 0; g < ngroups; ++g)
    if (off[g + 1] < off[g]) return fail(FNNUE_E_ARG, "group offsets must be non-decreasing");
  if (off[ngroups] != npos) return fail(FNNUE_E_ARG, "off[ngroups] must equal npos");
  DeviceGuard g(ctx->device);
  int rc = ensure_stage(ctx, std::max<size_t>(npos, 1), ngroups + 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(ctx->d_pos, pos, npos * sizeof(fnnue_pos), hipMemcpyHostToDevice, ctx->stream), "H2D");
  HIP_TRY(hipMemcpyAsync(ctx->d_off, off, (ngroups + 1) * 4, hipMemcpyHostToDevice, ctx->stream), "H2D");
  rc = fnnue_eval_groups_device(ctx, ctx->d_pos, ctx->d_off, ngroups, npos, mode, ctx->d_psqt, ctx->d_positional,
                                ctx->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(psqt, ctx->d_psqt, npos * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
  HIP_TRY(hipMemcpyAsync(positional, ctx->d_positional, npos * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
  HIP_TRY(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
  return name_invalid(latched(ctx), pos, npos);
}

int fnnue_eval_vgroups(fnnue_ctx* ctx, const fnnue_vpos* pos, size_t npos, const uint32_t* off, size_t ngroups,
                       int mode, int32_t* psqt, int32_t* positional) {
  if (!ctx) return fail(FNNUE_E_ARG, "null ctx");
  if (ctx->variant == kVariantChess) return fail(FNNUE_E_ARCH, "chess net: use fnnue_eval_groups*");
  if (mode != FNNUE_GROUP_CHAIN && mode != FNNUE_GROUP_STAR) return fail(FNNUE_E_ARG, "bad group mode");
  if (ngroups == 0) return npos == 0 ? FNNUE_OK : fail(FNNUE_E_ARG, "positions without groups");
  if (ngroups > 0xFFFFFFFFu || npos > 0xFFFFFFFFu) return fail(FNNUE_E_ARG, "batch too large");
  if (!pos || !off || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  if (off[0] != 0) return fail(FNNUE_E_ARG, "off[0] must be 0");
  for (size_t g = 0; g < ngroups; ++g)
    if (off[g + 1] < off[g]) return fail(FNNUE_E_ARG, "group offsets must be non-decreasing");
  if (off[ngroups] != npos) return fail(FNNUE_E_ARG, "off[ngroups] must equal npos");
  DeviceGuard g(ctx->device);
  int rc = ensure_stage(ctx, std::max<size_t>(npos, 1), ngroups + 1);
  if (rc) return rc;
  fnnue_vpos* d_vpos = reinterpret_cast<fnnue_vpos*>(ctx->d_pos);  // staging sized for fnnue_vpos
  HIP_TRY(hipMemcpyAsync(d_vpos, pos, npos * sizeof(fnnue_vpos), hipMemcpyHostToDevice, ctx->stream), "H2D");
  HIP_TRY(hipMemcpyAsync(ctx->d_off, off, (ngroups + 1) * 4, hipMemcpyHostToDevice, ctx->stream), "H2D");
  rc = fnnue_eval_vgroups_device(ctx, d_vpos, ctx->d_off, ngroups, npos, mode, ctx->d_psqt, ctx->d_positional,
                                 ctx->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(psqt, ctx->d_psqt, npos * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
  HIP_TRY(hipMemcpyAsync(positional, ctx->d_positional, npos * 4, hipMemcpyDeviceToHost, ctx->stream), "D2H");
  HIP_TRY(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
  return name_invalid_v(latched(ctx), pos, npos, ctx->variant, 0);
}

// ---- batch building ----

int fnnue_pos_from_fen(const char* fen, fnnue_pos* out) {
  if (!fen || !out) return fail(FNNUE_E_ARG, "null argument");
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  *out = b.pack();
  return FNNUE_OK;
}

namespace {
int split_moves(const char* moves, std::vector<std::string>& out) {
  out.clear();
  if (!moves) return FNNUE_OK;
  const char* p = moves;
  while (*p) {
    while (*p == ' ' || *p == '\t' || *p == '\n') ++p;
    const char* q = p;
    while (*q && *q != ' ' && *q != '\t' && *q != '\n') ++q;
    if (q > p) out.emplace_back(p, q);
    p = q;
  }
  return FNNUE_OK;
}
}  // namespace
}  // extern "C"

namespace fnnue::detail {

int game_end_chess(const char* fen, const char* moves, int* flags) {
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  std::vector<std::string> ms;
  split_moves(moves, ms);
  for (size_t i = 0; i < ms.size(); ++i) {
    Move m;
    if (!parse_uci(b, ms[i].c_str(), m))
      return fail(FNNUE_E_MOVE, "illegal move " + ms[i] + " at ply " + std::to_string(i + 1) + " in " + b.fen());
    b.do_move(m);
  }
  std::vector<Move> legal;
  b.legal_moves(legal);
  *flags = (legal.empty() ? FNNUE_END_NO_MOVES : 0) | (b.in_check() ? FNNUE_END_CHECK : 0);
  return FNNUE_OK;
}

}  // namespace fnnue::detail

extern "C" {

int fnnue_game_positions(const char* fen, const char* moves, fnnue_pos* out, size_t cap, size_t* n_out) {
  if (!fen || !n_out) return fail(FNNUE_E_ARG, "null argument");
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  std::vector<std::string> ms;
  split_moves(moves, ms);
  *n_out = ms.size() + 1;
  if (!out || cap < ms.size() + 1) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  out[0] = b.pack();
  for (size_t i = 0; i < ms.size(); ++i) {
    Move m;
    if (!parse_uci(b, ms[i].c_str(), m))
      return fail(FNNUE_E_MOVE, "illegal move " + ms[i] + " at ply " + std::to_string(i + 1) + " in " + b.fen());
    b.do_move(m);
    out[i + 1] = b.pack();
  }
  return FNNUE_OK;
}

int fnnue_game_children(const char* fen, const char* moves, fnnue_pos* out, size_t cap, uint32_t* off,
                        size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!fen || !n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  std::vector<std::string> ms;
  split_moves(moves, ms);
  std::vector<fnnue_pos> res;
  std::vector<uint32_t> offs{0};
  std::vector<Move> legal;
  for (size_t i = 0; i <= ms.size(); ++i) {
    res.push_back(b.pack());
    b.legal_moves(legal);
    for (const Move& m : legal) {
      Board c = b;
      c.do_move(m);
      res.push_back(c.pack());
    }
    offs.push_back((uint32_t)res.size());
    if (i == ms.size()) break;
    Move m;
    if (!parse_uci(b, ms[i].c_str(), m))
      return fail(FNNUE_E_MOVE, "illegal move " + ms[i] + " at ply " + std::to_string(i + 1));
    b.do_move(m);
  }
  *n_out = res.size();
  *n_groups = offs.size() - 1;
  if (!out || !off || cap < res.size() || off_cap < offs.size()) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  std::memcpy(out, res.data(), res.size() * sizeof(fnnue_pos));
  std::memcpy(off, offs.data(), offs.size() * sizeof(uint32_t));
  return FNNUE_OK;
}

int fnnue_random_playouts(uint64_t seed, size_t count, uint32_t min_plies, uint32_t max_plies, int mode, int threads,
                          fnnue_pos* out, size_t cap, uint32_t* off, size_t off_cap, size_t* n_out,
                          size_t* n_groups) {
  if (!n_out || !n_groups || !out) return fail(FNNUE_E_ARG, "null argument");
  if (mode < FNNUE_PLAYOUT_FINAL || mode > FNNUE_PLAYOUT_CHILDREN) return fail(FNNUE_E_ARG, "bad playout mode");
  if (min_plies > max_plies) return fail(FNNUE_E_ARG, "min_plies > max_plies");
  if (mode != FNNUE_PLAYOUT_FINAL && !off) return fail(FNNUE_E_ARG, "grouped modes need off[]");
  Board start;
  board_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", start, nullptr);
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  // Each playout is generated independently from (seed, index), so results do
  // not depend on the thread count.  Per-playout outputs are gathered into
  // per-thread vectors and concatenated in index order.
  struct Part {
    std::vector<fnnue_pos> pos;
    std::vector<uint32_t> sizes;  // group sizes
  };
  std::vector<Part> parts(threads);
  auto work = [&](int t) {
    const size_t b = count * t / threads, e = count * (t + 1) / threads;
    Part& P = parts[t];
    for (size_t i = b; i < e; ++i) {
      uint64_t st = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
      const uint32_t L = min_plies + (uint32_t)(splitmix64(st) % ((uint64_t)max_plies - min_plies + 1));
      Board bd = start;
      auto emit = [&](const Board& x) {
        if (mode == FNNUE_PLAYOUT_PLIES) {
          P.pos.push_back(x.pack());
        } else if (mode == FNNUE_PLAYOUT_CHILDREN) {
          P.pos.push_back(x.pack());
          std::vector<Move> ch;
          x.legal_moves(ch);
          for (const Move& m : ch) {
            Board c = x;
            c.do_move(m);
            P.pos.push_back(c.pack());
          }
          P.sizes.push_back((uint32_t)(ch.size() + 1));
        }
      };
      const size_t before = P.pos.size();
      emit(bd);
      for (uint32_t ply = 0; ply < L; ++ply) {
        Move m;
        if (bd.halfmove >= 100 || !bd.random_legal_move(st, m)) break;
        bd.do_move(m);
        emit(bd);
      }
      if (mode == FNNUE_PLAYOUT_FINAL) P.pos.push_back(bd.pack());
      else if (mode == FNNUE_PLAYOUT_PLIES) P.sizes.push_back((uint32_t)(P.pos.size() - before));
    }
  };
  try {
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  } catch (const std::exception& ex) {
    return fail(FNNUE_E_OOM, std::string("playout generation failed: ") + ex.what());
  }
  size_t total = 0, groups = 0;
  for (auto& P : parts) {
    total += P.pos.size();
    groups += P.sizes.size();
  }
  *n_out = total;
  *n_groups = groups;
  if (cap < total) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  if (mode != FNNUE_PLAYOUT_FINAL && off_cap < groups + 1) return fail(FNNUE_E_CAPACITY, "offset buffer too small");
  size_t k = 0, gk = 0;
  if (mode != FNNUE_PLAYOUT_FINAL) off[0] = 0;
  for (auto& P : parts) {
    std::memcpy(out + k, P.pos.data(), P.pos.size() * sizeof(fnnue_pos));
    for (uint32_t sz : P.sizes) {
      off[gk + 1] = off[gk] + sz;
      ++gk;
    }
    k += P.pos.size();
  }
  return FNNUE_OK;
}

int fnnue_perft(const char* fen, int depth, uint64_t* nodes) {
  if (!fen || !nodes || depth < 0) return fail(FNNUE_E_ARG, "bad argument");
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  *nodes = perft(b, depth);
  return FNNUE_OK;
}

int fnnue_selftest_mfma(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(FNNUE_E_DEVICE, "no such device");
  DeviceGuard g(device);
  int bad = -1;
  HIP_TRY(run_mfma_selftest(&bad), "mfma selftest");
  if (bad) return fail(FNNUE_E_DEVICE, "MFMA operand layout mismatch: " + std::to_string(bad) + " outputs differ");
  return FNNUE_OK;
}


int fnnue_build_batch_device(fnnue_ctx* ctx, const char* d_text, const uint32_t* d_fen_off,
                             const uint32_t* d_moves_off, size_t ngames, int mode, fnnue_pos* d_out, size_t cap,
                             uint32_t* d_off, size_t off_cap, size_t* n_out, size_t* n_groups, void* stream) {
  if (!ctx || !n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  if (mode != FNNUE_PLAYOUT_PLIES && mode != FNNUE_PLAYOUT_CHILDREN) return fail(FNNUE_E_ARG, "bad build mode");
  *n_out = *n_groups = 0;
  if (ngames == 0) return FNNUE_OK;
  if (!d_text || !d_fen_off || !d_moves_off) return fail(FNNUE_E_ARG, "null buffer");
  if (ngames > (1u << 26)) return fail(FNNUE_E_ARG, "too many games");
  DeviceGuard g(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const BuildResult R = build_batch_device(d_text, d_fen_off, d_moves_off, (uint32_t)ngames,
                                           mode == FNNUE_PLAYOUT_CHILDREN, d_out, cap, d_off, off_cap, s,
                                           ctx->bscratch);
  if (R.hip != hipSuccess) return hip_fail(R.hip, "device batch builder");
  *n_out = R.n_out;
  *n_groups = R.n_groups;
  if (R.err_code == kBuildErrFen)
    return fail(FNNUE_E_FEN, "unparsable FEN in game " + std::to_string(R.err_game));
  if (R.err_code == kBuildErrMove)
    return fail(FNNUE_E_MOVE, "illegal move at ply " + std::to_string(R.err_ply) + " of game " +
                                  std::to_string(R.err_game));
  if (R.capacity) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  return FNNUE_OK;
}

int fnnue_build_batch(fnnue_ctx* ctx, const char* text, size_t text_len, const uint32_t* fen_off,
                      const uint32_t* moves_off, size_t ngames, int mode, fnnue_pos* out, size_t cap, uint32_t* off,
                      size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!ctx || !n_out || !n_groups || (ngames && (!text || !fen_off || !moves_off)))
    return fail(FNNUE_E_ARG, "null argument");
  *n_out = *n_groups = 0;
  if (ngames == 0) return FNNUE_OK;
  if (fen_off[ngames] > text_len) return fail(FNNUE_E_ARG, "offsets exceed the text");
  for (size_t i = 0; i < ngames; ++i)
    if (fen_off[i] > moves_off[i] || moves_off[i] > fen_off[i + 1]) return fail(FNNUE_E_ARG, "offsets out of order");
  DeviceGuard g(ctx->device);
  // Input and output staging are per-context and grow-only (host-API calls are
  // synchronous), so a steady stream of batches allocates nothing.
  const size_t text_bytes = (text_len + 255) / 256 * 256;
  const size_t fo_bytes = (ngames + 1) * 4, mo_bytes = ngames * 4;
  int rc = ensure_builder_input(ctx, text_bytes + fo_bytes + mo_bytes);
  if (rc) return rc;
  char* d_text = ctx->d_btext;
  uint32_t* d_fo = reinterpret_cast<uint32_t*>(d_text + text_bytes);
  uint32_t* d_mo = d_fo + (ngames + 1);
  hipStream_t s = ctx->stream;
  HIP_TRY(hipMemcpyAsync(d_text, text, text_len, hipMemcpyHostToDevice, s), "H2D");
  HIP_TRY(hipMemcpyAsync(d_fo, fen_off, fo_bytes, hipMemcpyHostToDevice, s), "H2D");
  HIP_TRY(hipMemcpyAsync(d_mo, moves_off, mo_bytes, hipMemcpyHostToDevice, s), "H2D");
  rc = fnnue_build_batch_device(ctx, d_text, d_fo, d_mo, ngames, mode, nullptr, 0, nullptr, 0, n_out, n_groups, s);
  if (rc != FNNUE_E_CAPACITY) return rc;  // sizing pass: always "too small" with no outputs
  if (!out || !off || cap < *n_out || off_cap < *n_groups + 1) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  if ((rc = ensure_stage(ctx, *n_out, *n_groups + 1))) return rc;
  fnnue_pos* d_out = ctx->d_pos;
  uint32_t* d_off = ctx->d_off;
  rc = fnnue_build_batch_device(ctx, d_text, d_fo, d_mo, ngames, mode, d_out, *n_out, d_off, *n_groups + 1, n_out,
                                n_groups, s);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, d_out, *n_out * sizeof(fnnue_pos), hipMemcpyDeviceToHost, s), "D2H");
  HIP_TRY(hipMemcpyAsync(off, d_off, (*n_groups + 1) * 4, hipMemcpyDeviceToHost, s), "D2H");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return FNNUE_OK;
}

int fnnue_perft_device(fnnue_ctx* ctx, const char* fen, int depth, uint64_t* nodes) {
  if (!ctx || !fen || !nodes || depth < 1 || depth > 8) return fail(FNNUE_E_ARG, "bad argument");
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  // host expands the first depth - 3 levels, the device counts the rest
  std::vector<Board> level{b}, next;
  std::vector<Move> ms;
  for (int d = depth; d > 3; --d) {
    next.clear();
    for (const Board& x : level) {
      x.legal_moves(ms);
      for (const Move& m : ms) {
        Board c = x;
        c.do_move(m);
        next.push_back(c);
      }
    }
    level.swap(next);
  }
  std::vector<DBoard> frontier;
  frontier.reserve(level.size());
  for (const Board& x : level) frontier.push_back(to_dboard(x));
  DeviceGuard g(ctx->device);
  HIP_TRY(perft_device(frontier, std::min(depth, 3), nodes), "device perft");
  return FNNUE_OK;
}

int fnnue_random_game(uint64_t seed, const char* fen, uint32_t plies, char* moves, size_t cap, size_t* len) {
  if (!fen || !len) return fail(FNNUE_E_ARG, "null argument");
  Board b;
  std::string err;
  if (!board_from_fen(fen, b, &err)) return fail(FNNUE_E_FEN, err);
  uint64_t st = seed;
  std::string out;
  for (uint32_t i = 0; i < plies; ++i) {
    Move m;
    if (!b.random_legal_move(st, m)) break;
    if (!out.empty()) out += ' ';
    out += b.uci(m, b.chess960);
    b.do_move(m);
  }
  *len = out.size();
  if (!moves || cap < out.size() + 1) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  std::memcpy(moves, out.c_str(), out.size() + 1);
  return FNNUE_OK;
}
}  // extern "C"
