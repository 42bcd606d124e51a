// net.h — .nnue file model: parser, writer, synthetic generator and the
// contiguous device image layout shared by the host code and the kernels.
//
// File format follows upstream Stockfish 15.1 (SFNNv5): evaluate_nnue.cpp
// read_header/read_parameters, nnue_feature_transformer.h read_parameters,
// layers/affine_transform.h read_parameters, nnue_common.h (little-endian,
// COMPRESSED_LEB128).  The pinned net is nn-ad9b42354671.nnue ([ref] build.rs:7).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace fnnue {

constexpr uint32_t kVersion = 0x7AF32F20u;
constexpr uint32_t kFtHashBase = 0x7F234CB8u;   // HalfKAv2_hm::HashValue
constexpr uint32_t kNetHashBase = 0xEC42E90Du;  // Network::get_hash_value seed
constexpr int kFeatures = 22528;                // 64 king sq / 2 (mirror) * 11 planes * 64
// Fairy-Stockfish variant nets ("HalfKAv2 variants", recalled; parity
// unpinned): 8x8 boards, 64 own-king squares, no mirroring;
// per king square 704 board rows plus, with pockets, 2 colours x 5 piece
// types x 16 hand slots.
constexpr uint32_t kFtHashBaseVariants = 0x5F234CB8u;  // HalfKAv2::HashValue
constexpr int kVariantChess = 0, kVariantCrazyhouse = 1, kVariantAtomic = 2;
constexpr int kVBoardRows = 704, kVHandSlots = 16, kVHandRows = 2 * 5 * kVHandSlots;
constexpr uint32_t variant_rows(int variant) {  // feature rows per own-king square
  return variant == kVariantCrazyhouse ? kVBoardRows + kVHandRows : kVBoardRows;
}
constexpr uint32_t features_of(int variant) {
  return variant == kVariantChess ? (uint32_t)kFeatures : 64u * variant_rows(variant);
}
constexpr int kPsqtBuckets = 8;
constexpr int kStacks = 8;
constexpr int kL2 = 16;   // FC_0_OUTPUTS + 1 (the last is the "fwd" skip output)
constexpr int kL3 = 32;   // FC_1_OUTPUTS
constexpr int kFc1In = 32;// 2*FC_0_OUTPUTS = 30 padded to 32

uint32_t ft_hash(uint32_t hd, int variant);  // FeatureSet::HashValue ^ 2 * hd
uint32_t net_hash(uint32_t hd);
bool hd_supported(uint32_t hd);

struct Stack {
  int32_t b0[kL2];
  std::vector<int8_t> w0;  // [kL2][hd]
  int32_t b1[kL3];
  int8_t w1[kL3 * kFc1In];
  int32_t b2;
  int8_t w2[kL3];
};

struct Net {
  int variant = kVariantChess;
  uint32_t nfeat = kFeatures;     // features_of(variant)
  uint32_t hd = 0;
  uint32_t file_hash = 0;
  std::string desc;
  std::vector<int16_t> ft_bias;   // [hd]
  std::vector<int16_t> ft_w;      // [nfeat][hd]
  std::vector<int32_t> psqt_w;    // [nfeat][kPsqtBuckets]
  Stack st[kStacks];
};

// Returns 0 or a FNNUE_E_* code; err receives a message.
// variant: the feature set the file must carry (chess HalfKAv2_hm or a Fairy
// variant set); the header hash tells them apart and is checked.
int parse_net(const uint8_t* buf, size_t len, Net& net, std::string& err, int variant = kVariantChess);
void write_net(const Net& net, bool leb128, std::vector<uint8_t>& out);
void synthesize_net(uint64_t seed, uint32_t hd, uint32_t flags, Net& net, int variant = kVariantChess);

// Device image: one contiguous buffer, sections 256-byte aligned.  The FT
// weight table gets one extra all-zero row (index kFeatures) and the PSQT
// table one extra zero row, used as padding targets by the gather loops.
struct ImageLayout {
  size_t ft_w, ft_bias, psqt_w, w0, b0, w1, b1, w2, b2, total;
};
ImageLayout image_layout(uint32_t hd, uint32_t nfeat = kFeatures);
void pack_image(const Net& net, uint8_t* dst);  // dst has image_layout(hd).total bytes

// Largest possible |true int32 sum| of an accumulator column over every
// reachable accumulator: per king block kb and column j,
// |bias_j + w[own king row][j]| + the 31 largest |w[r][j]| of the other rows
// of kb (a position has at most 31 pieces besides the perspective's king),
// taken over the first half's even ("low") columns and, counted twice, over
// every second-half column (those are kept doubled in the SWAR tile).  Below
// 2^15 the feature transformer may sum column pairs as 32-bit words
// (ft_slices' SWAR rows) and still be bit-exact.
// rows / blocks: the feature set's rows per own-king block and block count
// (chess: 704 x 32, own king row 640 + KingBuckets order; variants: rows x 64,
// own king row 640 + oriented king square).
int32_t accumulator_bound(const int16_t* ft_w, const int16_t* ft_bias, uint32_t hd, int variant = kVariantChess);

}  // namespace fnnue
