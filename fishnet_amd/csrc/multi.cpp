// multi.cpp — several GPUs from one process (include/fnnue.h "multi-GPU").
//
// The reference scales by running one single-threaded engine per core, each
// fed whole positions by the queue ([ref] src/main.rs:156-170,
// src/configure.rs:196-206).  Here one fnnue_multi owns one context per GPU:
//  * the net is uploaded once to devices[0] and RCCL-broadcast over xGMI to the
//    others (ncclCommInitAll: one communicator per device, single process);
//  * positions are independent, so a batch is sharded with no data-path
//    collective: contiguous ranges of positions, or whole groups (a game's
//    plies, a parent and its children: never split) balanced by position
//    count (fnnue_partition_groups);
//  * host-buffer calls run one host thread per device (H2D of its shard, the
//    device path, D2H into its disjoint slice of the caller's buffers);
//    device-buffer calls enqueue on every device's stream (the caller's, or
//    the context's own) and return without any host synchronisation.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "internal.h"

using namespace fnnue;
using namespace fnnue::detail;

struct fnnue_multi {
  std::vector<int> devices;
  std::vector<fnnue_ctx*> ctx;
  std::vector<ncclComm_t> comms;
};

namespace {

void multi_destroy(fnnue_multi* m) {
  if (!m) return;
  for (ncclComm_t c : m->comms)
    if (c) (void)ncclCommDestroy(c);
  for (fnnue_ctx* c : m->ctx) ctx_destroy(c);
  delete m;
}

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(FNNUE_E_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

// Runs f(i) for every device on its own host thread; the first failing
// device's code and message (prefixed with the device) become the call's.
template <class F>
int per_device(const fnnue_multi* m, F&& f) {
  const size_t nd = m->ctx.size();
  std::vector<int> rc(nd, FNNUE_OK);
  std::vector<std::string> msg(nd);
  auto run = [&](size_t i) {
    rc[i] = f(i);
    if (rc[i]) msg[i] = fnnue_last_error();
  };
  std::vector<std::thread> th;
  try {
    for (size_t i = 1; i < nd; ++i) th.emplace_back(run, i);
  } catch (const std::exception& e) {
    for (auto& t : th) t.join();
    return fail(FNNUE_E_OOM, std::string("cannot start device threads: ") + e.what());
  }
  run(0);
  for (auto& t : th) t.join();
  for (size_t i = 0; i < nd; ++i)
    if (rc[i]) return fail(rc[i], "device " + std::to_string(m->devices[i]) + ": " + msg[i]);
  return FNNUE_OK;
}

}  // namespace

extern "C" {

int fnnue_partition_groups(const uint32_t* off, size_t ngroups, int nparts, uint32_t* cut) {
  if (!off || !cut || nparts < 1) return fail(FNNUE_E_ARG, "bad argument");
  if (ngroups > 0xFFFFFFFFu) return fail(FNNUE_E_ARG, "too many groups");
  if (off[0] != 0) return fail(FNNUE_E_ARG, "off[0] must be 0");
  for (size_t g = 0; g < ngroups; ++g)
    if (off[g + 1] < off[g]) return fail(FNNUE_E_ARG, "group offsets must be non-decreasing");
  // Part k ends at the group boundary nearest to k/nparts of the positions:
  // contiguous whole groups, each part within half the largest group of its
  // share.
  const uint64_t total = off[ngroups];
  cut[0] = 0;
  for (int k = 1; k < nparts; ++k) {
    const uint64_t target = total * (uint64_t)k / (uint64_t)nparts;
    size_t g = std::lower_bound(off + cut[k - 1], off + ngroups + 1, (uint32_t)target) - off;
    if (g > cut[k - 1] && g <= ngroups && target - off[g - 1] < (uint64_t)off[std::min(g, ngroups)] - target) --g;
    cut[k] = (uint32_t)std::min(g, ngroups);
  }
  cut[nparts] = (uint32_t)ngroups;
  return FNNUE_OK;
}

int fnnue_multi_create(const fnnue_net* net, const int* devices, int ndev, fnnue_multi** out) {
  if (!net || !devices || !out || ndev < 1) return fail(FNNUE_E_ARG, "bad argument");
  *out = nullptr;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail == 0) return fail(FNNUE_E_DEVICE, "no HIP device available");
  for (int i = 0; i < ndev; ++i) {
    if (devices[i] < 0 || devices[i] >= avail)
      return fail(FNNUE_E_DEVICE, "device ordinal " + std::to_string(devices[i]) + " out of range");
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i]) return fail(FNNUE_E_ARG, "device listed twice");
  }
  std::unique_ptr<fnnue_multi, void (*)(fnnue_multi*)> m(new (std::nothrow) fnnue_multi, multi_destroy);
  if (!m) return fail(FNNUE_E_OOM, "host allocation failed");
  m->devices.assign(devices, devices + ndev);
  m->ctx.assign(ndev, nullptr);
  const uint32_t hd = net->net.hd;
  for (int i = 0; i < ndev; ++i)
    if (int rc = ctx_alloc(devices[i], hd, &m->ctx[i], net->net.variant)) return rc;
  // net image: packed once on the host, uploaded to devices[0] ...
  std::vector<uint8_t> img;
  try {
    img.resize(m->ctx[0]->image_bytes);
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  pack_image(net->net, img.data());
  {
    DeviceGuard g(devices[0]);
    HIP_TRY(hipMemcpy(m->ctx[0]->image, img.data(), img.size(), hipMemcpyHostToDevice), "hipMemcpy(net image)");
  }
  // ... and RCCL-broadcast over xGMI to every device (in place on the root).
  m->comms.assign(ndev, nullptr);
  ncclResult_t r = ncclCommInitAll(m->comms.data(), ndev, devices);
  if (r != ncclSuccess) {
    m->comms.clear();
    return nccl_fail(r, "ncclCommInitAll");
  }
  if ((r = ncclGroupStart()) != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
  for (int i = 0; i < ndev; ++i) {
    DeviceGuard g(devices[i]);
    r = ncclBroadcast(m->ctx[0]->image, m->ctx[i]->image, m->ctx[i]->image_bytes, ncclUint8, 0, m->comms[i],
                      m->ctx[i]->stream);
    if (r != ncclSuccess) break;
  }
  const ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess) return nccl_fail(r, "ncclBroadcast(net image)");
  if (r2 != ncclSuccess) return nccl_fail(r2, "ncclGroupEnd");
  for (int i = 0; i < ndev; ++i) {
    DeviceGuard g(devices[i]);
    HIP_TRY(hipStreamSynchronize(m->ctx[i]->stream), "hipStreamSynchronize(broadcast)");
    if (int rc = finish_upload(m->ctx[i])) return rc;
  }
  *out = m.release();
  return FNNUE_OK;
}

void fnnue_multi_free(fnnue_multi* m) { multi_destroy(m); }

int fnnue_multi_size(const fnnue_multi* m, int* ndev) {
  if (!m || !ndev) return fail(FNNUE_E_ARG, "null argument");
  *ndev = (int)m->ctx.size();
  return FNNUE_OK;
}

int fnnue_multi_ctx(fnnue_multi* m, int i, fnnue_ctx** ctx) {
  if (!m || !ctx || i < 0 || i >= (int)m->ctx.size()) return fail(FNNUE_E_ARG, "bad argument");
  *ctx = m->ctx[i];
  return FNNUE_OK;
}

int fnnue_multi_eval_positions(fnnue_multi* m, const fnnue_pos* pos, size_t n, int32_t* psqt, int32_t* positional) {
  if (!m) return fail(FNNUE_E_ARG, "null multi");
  if (n == 0) return FNNUE_OK;
  if (!pos || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  const size_t nd = m->ctx.size();
  return per_device(m, [&](size_t i) {
    const size_t lo = n * i / nd, hi = n * (i + 1) / nd;
    return fnnue_eval_positions(m->ctx[i], pos + lo, hi - lo, psqt + lo, positional + lo);
  });
}

int fnnue_multi_eval_groups(fnnue_multi* m, const fnnue_pos* pos, size_t npos, const uint32_t* off, size_t ngroups,
                            int mode, int32_t* psqt, int32_t* positional) {
  if (!m) return fail(FNNUE_E_ARG, "null multi");
  if (mode != FNNUE_GROUP_CHAIN && mode != FNNUE_GROUP_STAR) return fail(FNNUE_E_ARG, "bad group mode");
  if (ngroups == 0) return npos == 0 ? FNNUE_OK : fail(FNNUE_E_ARG, "positions without groups");
  if (!pos || !off || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  const int nd = (int)m->ctx.size();
  std::vector<uint32_t> cut(nd + 1);
  if (int rc = fnnue_partition_groups(off, ngroups, nd, cut.data())) return rc;
  if (off[ngroups] != npos) return fail(FNNUE_E_ARG, "off[ngroups] must equal npos");
  return per_device(m, [&](size_t i) {
    const uint32_t g0 = cut[i], g1 = cut[i + 1], base = off[g0];
    if (g1 == g0) return (int)FNNUE_OK;
    std::vector<uint32_t> local(off + g0, off + g1 + 1);
    for (uint32_t& v : local) v -= base;
    return fnnue_eval_groups(m->ctx[i], pos + base, off[g1] - base, local.data(), g1 - g0, mode, psqt + base,
                             positional + base);
  });
}

// Device-buffer calls: every device's work is enqueued on streams[i] (or, for
// a null array / entry, its context's own stream) and the call returns; no
// host synchronisation at any batch size, so the devices run concurrently.
namespace {
void* stream_of(void* const* streams, size_t i) { return streams ? streams[i] : nullptr; }
}  // namespace

int fnnue_multi_eval_positions_device(fnnue_multi* m, const fnnue_pos* const* d_pos, const size_t* n,
                                      int32_t* const* d_psqt, int32_t* const* d_positional, void* const* streams) {
  if (!m || !d_pos || !n || !d_psqt || !d_positional) return fail(FNNUE_E_ARG, "null argument");
  for (size_t i = 0; i < m->ctx.size(); ++i)
    if (int rc = fnnue_eval_positions_device(m->ctx[i], d_pos[i], n[i], d_psqt[i], d_positional[i],
                                             stream_of(streams, i)))
      return fail(rc, "device " + std::to_string(m->devices[i]) + ": " + fnnue_last_error());
  return FNNUE_OK;
}

int fnnue_multi_eval_groups_device(fnnue_multi* m, const fnnue_pos* const* d_pos, const uint32_t* const* d_off,
                                   const size_t* ngroups, const size_t* npos, int mode, int32_t* const* d_psqt,
                                   int32_t* const* d_positional, void* const* streams) {
  if (!m || !d_pos || !d_off || !ngroups || !npos || !d_psqt || !d_positional)
    return fail(FNNUE_E_ARG, "null argument");
  for (size_t i = 0; i < m->ctx.size(); ++i)
    if (int rc = fnnue_eval_groups_device(m->ctx[i], d_pos[i], d_off[i], ngroups[i], npos[i], mode, d_psqt[i],
                                          d_positional[i], stream_of(streams, i)))
      return fail(rc, "device " + std::to_string(m->devices[i]) + ": " + fnnue_last_error());
  return FNNUE_OK;
}

int fnnue_multi_eval_vgroups_device(fnnue_multi* m, const fnnue_vpos* const* d_pos, const uint32_t* const* d_off,
                                    const size_t* ngroups, const size_t* npos, int mode, int32_t* const* d_psqt,
                                    int32_t* const* d_positional, void* const* streams) {
  if (!m || !d_pos || !d_off || !ngroups || !npos || !d_psqt || !d_positional)
    return fail(FNNUE_E_ARG, "null argument");
  for (size_t i = 0; i < m->ctx.size(); ++i)
    if (int rc = fnnue_eval_vgroups_device(m->ctx[i], d_pos[i], d_off[i], ngroups[i], npos[i], mode, d_psqt[i],
                                           d_positional[i], stream_of(streams, i)))
      return fail(rc, "device " + std::to_string(m->devices[i]) + ": " + fnnue_last_error());
  return FNNUE_OK;
}

int fnnue_multi_eval_vpositions(fnnue_multi* m, const fnnue_vpos* pos, size_t n, int32_t* psqt, int32_t* positional) {
  if (!m) return fail(FNNUE_E_ARG, "null multi");
  if (n == 0) return FNNUE_OK;
  if (!pos || !psqt || !positional) return fail(FNNUE_E_ARG, "null buffer");
  const size_t nd = m->ctx.size();
  return per_device(m, [&](size_t i) {
    const size_t lo = n * i / nd, hi = n * (i + 1) / nd;
    return fnnue_eval_vpositions(m->ctx[i], pos + lo, hi - lo, psqt + lo, positional + lo);
  });
}

int fnnue_multi_eval_vpositions_device(fnnue_multi* m, const fnnue_vpos* const* d_pos, const size_t* n,
                                       int32_t* const* d_psqt, int32_t* const* d_positional, void* const* streams) {
  if (!m || !d_pos || !n || !d_psqt || !d_positional) return fail(FNNUE_E_ARG, "null argument");
  for (size_t i = 0; i < m->ctx.size(); ++i)
    if (int rc = fnnue_eval_vpositions_device(m->ctx[i], d_pos[i], n[i], d_psqt[i], d_positional[i],
                                              stream_of(streams, i)))
      return fail(rc, "device " + std::to_string(m->devices[i]) + ": " + fnnue_last_error());
  return FNNUE_OK;
}

int fnnue_multi_sync(fnnue_multi* m) {
  if (!m) return fail(FNNUE_E_ARG, "null multi");
  int first = FNNUE_OK;
  std::string msg;
  for (size_t i = 0; i < m->ctx.size(); ++i) {  // every device drained, even after an error
    const int rc = fnnue_ctx_check(m->ctx[i]);
    if (rc && !first) {
      first = rc;
      msg = "device " + std::to_string(m->devices[i]) + ": " + fnnue_last_error();
    }
  }
  return first ? fail(first, msg) : FNNUE_OK;
}

}  // extern "C"
