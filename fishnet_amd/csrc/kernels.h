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
hipError_t launch_ft_groups(uint32_t hd, const fnnue_pos* pos, const uint32_t* off, uint32_t ngroups,
                            uint32_t base, int mode, const NetPtrs& net, uint8_t* x, int32_t* psqt, uint8_t* bucket,
                            uint32_t* err, hipStream_t stream);

// Layer stacks: 16 positions per wave, int8 MFMA for fc_0 and fc_1.
hipError_t launch_stack(uint32_t hd, const uint8_t* x, const uint8_t* bucket, uint32_t n, const NetPtrs& net,
                        int32_t* positional, hipStream_t stream);

// MFMA operand-layout self test: returns number of mismatching outputs in *bad.
hipError_t run_mfma_selftest(int* bad);

bool kernels_support_hd(uint32_t hd);

}  // namespace fnnue
