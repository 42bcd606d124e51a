// kernels.h — launchers for the CDNA4 NNUE kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/fnnue.h"

namespace fnnue {

struct NetPtrs {
  const int16_t* ft_w;     // [kFeatures+1][hd] (last row zero)
  const int16_t* ft_bias;  // [hd]
  const int32_t* psqt_w;   // [kFeatures+1][8] (last row zero)
  const int8_t* w0;        // [8][16][hd]
  const int32_t* b0;       // [8][16]
  const int8_t* w1;        // [8][32][32]
  const int32_t* b1;       // [8][32]
  const int8_t* w2;        // [8][32]
  const int32_t* b2;       // [8]
};

// Feature transformer from scratch: one wave per position.  Writes the
// transformed features x[n][hd] (u8, stm half first), psqt[n] and bucket[n]
// (0xFF for an invalid position, latched in *err).
hipError_t launch_ft_scratch(uint32_t hd, const fnnue_pos* pos, uint32_t n, const NetPtrs& net, uint8_t* x,
                             int32_t* psqt, uint8_t* bucket, uint32_t* err, hipStream_t stream);

// Feature transformer along groups (CHAIN: incremental along plies; STAR:
// children derived from the group's first position).  One wave per group.
// Positions [lo, hi) of the call (a chunk): every group is clamped to it, a
// group cut at lo restarting there with a refresh; x / psqt / bucket are
// chunk-relative (row i - lo).
hipError_t launch_ft_groups(uint32_t hd, const fnnue_pos* pos, const uint32_t* off, uint32_t ngroups,
                            uint32_t lo, uint32_t hi, int mode, const NetPtrs& net, uint8_t* x, int32_t* psqt,
                            uint8_t* bucket, uint32_t* err, hipStream_t stream);

// Layer stacks: 16 positions per wave, int8 MFMA for fc_0 and fc_1.  Row i of
// x / bucket is written to positional[perm ? perm[i] : i]; when psqt_part is
// given, psqt[perm[i]] = (psqt_part[2i] - psqt_part[2i+1]) / 2 as well.
hipError_t launch_stack(uint32_t hd, const uint8_t* x, const uint8_t* bucket, uint32_t n, const NetPtrs& net,
                        int32_t* positional, const uint32_t* perm, const int32_t* psqt_part, int32_t* psqt,
                        hipStream_t stream);

// LDS-stationary feature transformer (ft_sliced.hip).
// Perspective-items per (king block) work unit: 48 passes of 128 items.
// Measured on config 2 (1M positions): 4096 595-600M, 5120 586-592M, 6144
// 603-613M, 7168 594-599M, 8192 592-597M positions/s (crazyhouse: neutral).
// Must stay a multiple of 128 (a pass step) so pass items 2k / 2k + 1 keep
// their parity roles (write_rows).
#ifndef FT_UNIT_ITEMS
#define FT_UNIT_ITEMS 6144
#endif
constexpr uint32_t kUnitItems = FT_UNIT_ITEMS;
static_assert(kUnitItems % 128 == 0, "units are whole pass steps");
struct SlicedPlan {
  void* tiles;       // [32 king blocks][hd/64 slices][705 rows][8] x 16 B (relayout of ft_w)
  uint32_t* ctr;     // sliced_ctr_words() counters / offsets
  void* units;       // int4 [sliced_max_units(chunk)]
  uint32_t* items;   // [2 * chunk] item records
  uint16_t* flist;   // [2 * chunk][32] feature rows relative to the king block
  uint32_t* perm;    // [chunk] bucket-sorted slot -> position index
  int32_t* psqt_part;// [chunk][2] per-slot PSQT sums of the stm / nstm perspective
  bool swar;          // ft_slices may sum rows as SWAR words (accumulator_bound < 2^15)
};
size_t sliced_tiles_bytes(uint32_t hd);
size_t sliced_ctr_words();
uint32_t sliced_max_units(uint32_t chunk);
hipError_t launch_relayout_sliced(uint32_t hd, const NetPtrs& net, void* tiles, hipStream_t stream);
// The two halves of launch_ft_sliced, for pipelining chunks over streams:
// the plan (psqt[pos] of invalid positions, bucket[slot], P.perm, lists) and
// the LDS-stationary slices (x[slot], P.psqt_part).
hipError_t launch_sliced_plan(const fnnue_pos* pos, uint32_t n, const SlicedPlan& P, int32_t* psqt, uint8_t* bucket,
                              uint32_t* err, hipStream_t stream);
hipError_t launch_sliced_ft(uint32_t hd, uint32_t n, const NetPtrs& net, const SlicedPlan& P, uint8_t* x,
                            hipStream_t stream);
// Writes psqt[pos], x[slot], bucket[slot] and P.perm; then run launch_stack with P.perm.
// `mid` (optional) is recorded between the plan and the main kernel (phase timing).
hipError_t launch_ft_sliced(uint32_t hd, const fnnue_pos* pos, uint32_t n, const NetPtrs& net, const SlicedPlan& P,
                            uint8_t* x, int32_t* psqt, uint8_t* bucket, uint32_t* err, hipStream_t stream,
                            hipEvent_t mid = nullptr);

// Fairy-Stockfish variant nets (net.h kVariant*): positions fnnue_vpos; the
// plan (variant.hip) fills a SlicedPlan with the variant counter layout, the
// main kernel is ft_slices over the variant tile geometry, then launch_stack
// with P.perm / P.psqt_part as for chess.
size_t variant_tiles_bytes(uint32_t hd, int variant);
uint32_t variant_max_units(uint32_t chunk);
size_t variant_ctr_words();
hipError_t launch_relayout_variant(uint32_t hd, int variant, const NetPtrs& net, void* tiles, hipStream_t stream);
hipError_t launch_variant_plan(const fnnue_vpos* pos, uint32_t n, int variant, const SlicedPlan& P, int32_t* psqt,
                               uint8_t* bucket, uint32_t* err, hipStream_t stream);
hipError_t launch_variant_ft(uint32_t hd, int variant, uint32_t n, const NetPtrs& net, const SlicedPlan& P, uint8_t* x,
                             hipStream_t stream);

// Incremental FT on LDS tiles for CHAIN / STAR groups (ft_segments.hip).
// Uses the sliced plan's tiles, counters, unit table, lists and psqt_part;
// writes x[i], bucket[i], psqt_part[2i + half] in position order, then run
// launch_stack with perm = null and psqt_part.
struct SegPlan {
  uint32_t* ref;      // [2 * chunk + 1] refresh flags per (perspective, position)
  uint32_t* cref;     // [2 * chunk + 1] exclusive scan of ref
  void* dtmp;         // uint4 [2 * chunk] delta records by position
  void* drec;         // uint4 [2 * chunk] delta records at root + rank
  uint32_t* ipos;     // [2 * chunk] item -> root position
  uint32_t* len;      // [2 * chunk] segment length at the root
  void* items;        // uint4 [2 * chunk] sorted item records
  void* span;         // uint2 [span_cap] group {first, end} per position of a call (grow-only)
  size_t span_cap;
  void* scan_temp;
  size_t scan_temp_bytes;
  uint32_t unit_plies;  // work per segment unit (seg_unit_plies_for the planning net's HD)
};
size_t seg_scan_temp_bytes(uint32_t chunk);
size_t seg_ctr_words();  // counter words of the segment plans (any feature set)
// unit-table entries ft_segments may need for units of unit_plies (0: the
// smallest units any net uses, for sizing)
uint32_t seg_max_units(uint32_t chunk, uint32_t unit_plies = 0);
uint32_t seg_unit_plies(uint32_t hd);  // the segment unit size of a net of width hd
// Once per grouped call: span[i] = {first, end} of position i's group
// (absolute, npos entries; span == nullptr: check only).  check: the offsets
// are checked on the device (non-decreasing, spanning [0, npos)), latching
// error bit 2 (FNNUE_E_ARG); every kernel stays in bounds regardless.
hipError_t launch_group_span(const uint32_t* off, uint32_t ngroups, uint32_t npos, void* span, bool check,
                             uint32_t* err, hipStream_t stream);
// One chunk: positions pos[0, n) = the call's positions [sbase, sbase + n),
// span = the call's span table + sbase.  Groups cut by the chunk's edges are
// clamped to it (their first in-chunk position refreshes).
// variant: kVariantChess (pos = fnnue_pos) or a Fairy-Stockfish feature set
// (pos = fnnue_vpos; hd 256 / 512 / 1024; P.tiles / counters of that set).
hipError_t launch_ft_segments(uint32_t hd, int variant, const void* pos, uint32_t n, const void* span, uint32_t sbase,
                              int mode, const NetPtrs& net, const SlicedPlan& P, const SegPlan& G, uint8_t* x,
                              uint8_t* bucket, uint32_t* err, hipStream_t stream, hipEvent_t mid = nullptr);
// Its two halves.  The plan depends on the positions, the groups and the
// feature set only, not on the net: a second net of the same feature set (the
// small net beside the big one) runs its main kernel over the same plan
// (P.ctr / units / flist and G), with its own tiles, swar flag, psqt_part, x.
// A grouped call of at most seg_small_plan_max() positions: spans, offset
// check and the whole plan of its one chunk in one workgroup (then
// launch_seg_ft).
uint32_t seg_small_plan_max();
hipError_t launch_seg_plan_small(int variant, const void* pos, uint32_t n, const uint32_t* off, uint32_t ngroups,
                                 void* span, int mode, const SlicedPlan& P, const SegPlan& G, uint8_t* bucket,
                                 uint32_t* err, hipStream_t stream);
hipError_t launch_seg_plan(int variant, const void* pos, uint32_t n, const void* span, uint32_t sbase, int mode,
                           const SlicedPlan& P, const SegPlan& G, uint8_t* bucket, uint32_t* err, hipStream_t stream);
// A second unit table over a chunk's plan (after launch_seg_plan): units of
// unit_plies into `units`, their count into ctr_out's unit-count slot, P's
// counters untouched — the small net of a dual call runs its main kernel over
// these (P.units = units, P.ctr = ctr_out) instead of the big net's units.
hipError_t launch_seg_units(int variant, const SlicedPlan& P, void* units, uint32_t* ctr_out, uint32_t unit_plies,
                            hipStream_t stream);
hipError_t launch_seg_ft(uint32_t hd, int variant, uint32_t n, int mode, const NetPtrs& net, const SlicedPlan& P,
                         const SegPlan& G, uint8_t* x, hipStream_t stream);

// MFMA operand-layout self test: returns number of mismatching outputs in *bad.
hipError_t run_mfma_selftest(int* bad);

bool kernels_support_hd(uint32_t hd);

}  // namespace fnnue
