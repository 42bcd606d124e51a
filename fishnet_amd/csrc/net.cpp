// net.cpp — .nnue parsing/writing, synthetic nets and the device image.
#include "net.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>
#include <cstring>

#include "../../include/fnnue.h"
#include "board.h"

namespace fnnue {

static const char kLebMagic[] = "COMPRESSED_LEB128";
static constexpr size_t kLebMagicLen = sizeof(kLebMagic) - 1;

// layers/affine_transform.h get_hash_value
static uint32_t affine_hash(uint32_t prev, uint32_t out) {
  return (0xCC03DAE4u + out) ^ (prev >> 1) ^ (prev << 31);
}
// layers/clipped_relu.h get_hash_value
static uint32_t crelu_hash(uint32_t prev) { return 0x538D24C7u + prev; }

uint32_t ft_hash(uint32_t hd, int variant) {
  return (variant == kVariantChess ? kFtHashBase : kFtHashBaseVariants) ^ (hd * 2);
}

uint32_t net_hash(uint32_t hd) {
  uint32_t h = kNetHashBase ^ (hd * 2);
  h = affine_hash(h, kL2);   // fc_0
  h = crelu_hash(h);         // ac_0 (ac_sqr_0 is not part of the chain)
  h = affine_hash(h, kL3);   // fc_1
  h = crelu_hash(h);         // ac_1
  h = affine_hash(h, 1);     // fc_2
  return h;
}

// Kernels need hd/2 to be a multiple of 64 lanes and hd a multiple of the
// 64-deep MFMA k-step.
bool hd_supported(uint32_t hd) { return hd >= 128 && hd <= 4096 && hd % 128 == 0; }

namespace {

struct Reader {
  const uint8_t* p;
  size_t n, off = 0;
  bool fail = false;
  uint32_t u32() {
    if (off + 4 > n) { fail = true; return 0; }
    uint32_t v;
    std::memcpy(&v, p + off, 4);
    off += 4;
    return v;
  }
  template <typename T>
  void ints(T* dst, size_t count) {
    if (off + kLebMagicLen <= n && std::memcmp(p + off, kLebMagic, kLebMagicLen) == 0) {
      off += kLebMagicLen;
      const uint32_t bytes = u32();
      if (fail || off + bytes > n) { fail = true; return; }
      const uint8_t* q = p + off;
      size_t i = 0, pos = 0;
      for (; i < count; ++i) {
        int64_t r = 0;
        unsigned shift = 0;
        uint8_t byte = 0x80;
        while (byte & 0x80) {
          if (pos >= bytes || shift > 8 * sizeof(T) + 7) { fail = true; return; }
          byte = q[pos++];
          r |= int64_t(byte & 0x7f) << shift;
          shift += 7;
        }
        if (shift < 64 && (byte & 0x40)) r |= -(int64_t(1) << shift);
        dst[i] = T(r);
      }
      if (pos != bytes) { fail = true; return; }
      off += bytes;
      return;
    }
    if (off + sizeof(T) * count > n) { fail = true; return; }
    std::memcpy(dst, p + off, sizeof(T) * count);  // host is little-endian (x86-64)
    off += sizeof(T) * count;
  }
};

struct Writer {
  std::vector<uint8_t>& o;
  void u32(uint32_t v) { const uint8_t* b = (const uint8_t*)&v; o.insert(o.end(), b, b + 4); }
  template <typename T>
  void ints(const T* src, size_t count, bool leb) {
    if (!leb) {
      const uint8_t* b = (const uint8_t*)src;
      o.insert(o.end(), b, b + sizeof(T) * count);
      return;
    }
    std::vector<uint8_t> body;
    body.reserve(count * 2);
    for (size_t i = 0; i < count; ++i) {
      int64_t v = src[i];
      while (true) {
        uint8_t byte = v & 0x7f;
        v >>= 7;  // arithmetic
        if ((v == 0 && !(byte & 0x40)) || (v == -1 && (byte & 0x40))) { body.push_back(byte); break; }
        body.push_back(byte | 0x80);
      }
    }
    o.insert(o.end(), kLebMagic, kLebMagic + kLebMagicLen);
    u32((uint32_t)body.size());
    o.insert(o.end(), body.begin(), body.end());
  }
};

}  // namespace

int parse_net(const uint8_t* buf, size_t len, Net& net, std::string& err, int variant) {
  Reader r{buf, len};
  const uint32_t version = r.u32(), file_hash = r.u32(), dlen = r.u32();
  if (r.fail) { err = "truncated header"; return FNNUE_E_FORMAT; }
  if (version != kVersion) { err = "unsupported .nnue version"; return FNNUE_E_FORMAT; }
  if (r.off + dlen > len) { err = "truncated description"; return FNNUE_E_FORMAT; }
  net.desc.assign((const char*)buf + r.off, dlen);
  r.off += dlen;
  const uint32_t fth = r.u32();
  const uint32_t hd = (fth ^ ft_hash(0, variant)) / 2;
  if (r.fail || ft_hash(hd, variant) != fth) {
    err = variant == kVariantChess ? "feature transformer hash is not HalfKAv2_hm"
                                   : "feature transformer hash is not HalfKAv2 (variants)";
    return FNNUE_E_FORMAT;
  }
  if (!hd_supported(hd)) { err = "unsupported transformed feature dimension " + std::to_string(hd); return FNNUE_E_ARCH; }
  if ((ft_hash(hd, variant) ^ net_hash(hd)) != file_hash) {
    err = "file hash does not match the SFNNv5 structure";
    return FNNUE_E_FORMAT;
  }
  net.variant = variant;
  net.nfeat = features_of(variant);
  net.hd = hd;
  net.file_hash = file_hash;
  net.ft_bias.resize(hd);
  net.ft_w.resize((size_t)hd * net.nfeat);
  net.psqt_w.resize((size_t)kPsqtBuckets * net.nfeat);
  r.ints(net.ft_bias.data(), hd);
  r.ints(net.ft_w.data(), net.ft_w.size());
  r.ints(net.psqt_w.data(), net.psqt_w.size());
  if (r.fail) { err = "truncated feature transformer"; return FNNUE_E_FORMAT; }
  const uint32_t nh = net_hash(hd);
  for (int b = 0; b < kStacks; ++b) {
    Stack& s = net.st[b];
    if (r.u32() != nh || r.fail) { err = "layer stack " + std::to_string(b) + " hash mismatch"; return FNNUE_E_FORMAT; }
    s.w0.resize((size_t)kL2 * hd);
    r.ints(s.b0, kL2);
    r.ints(s.w0.data(), s.w0.size());
    r.ints(s.b1, kL3);
    r.ints(s.w1, kL3 * kFc1In);
    r.ints(&s.b2, 1);
    r.ints(s.w2, kL3);
    if (r.fail) { err = "truncated layer stack " + std::to_string(b); return FNNUE_E_FORMAT; }
  }
  if (r.off != len) { err = "trailing bytes after the last layer stack"; return FNNUE_E_FORMAT; }
  return FNNUE_OK;
}

void write_net(const Net& net, bool leb, std::vector<uint8_t>& out) {
  out.clear();
  Writer w{out};
  w.u32(kVersion);
  w.u32(ft_hash(net.hd, net.variant) ^ net_hash(net.hd));
  w.u32((uint32_t)net.desc.size());
  out.insert(out.end(), net.desc.begin(), net.desc.end());
  w.u32(ft_hash(net.hd, net.variant));
  w.ints(net.ft_bias.data(), net.ft_bias.size(), leb);
  w.ints(net.ft_w.data(), net.ft_w.size(), leb);
  w.ints(net.psqt_w.data(), net.psqt_w.size(), leb);
  for (int b = 0; b < kStacks; ++b) {
    const Stack& s = net.st[b];
    w.u32(net_hash(net.hd));
    // Upstream writes AffineTransform biases/weights plainly (only the FT is LEB128).
    w.ints(s.b0, kL2, false);
    w.ints(s.w0.data(), s.w0.size(), false);
    w.ints(s.b1, kL3, false);
    w.ints(s.w1, kL3 * kFc1In, false);
    w.ints(&s.b2, 1, false);
    w.ints(s.w2, kL3, false);
  }
}

namespace {
struct Rng {
  uint64_t s;
  uint64_t next() { return splitmix64(s); }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  // Irwin-Hall(4) approximation of N(0,1): deterministic and libm-free.
  double gauss() { return (uni() + uni() + uni() + uni() - 2.0) * 1.7320508075688772; }
  int64_t range(int64_t lo, int64_t hi) { return lo + (int64_t)(next() % (uint64_t)(hi - lo + 1)); }
};
template <typename T>
T clampT(double v, double lo, double hi) { return (T)std::llround(v < lo ? lo : (v > hi ? hi : v)); }
}  // namespace

// Magnitudes are chosen so that every clamp regime of the evaluation is hit
// (accumulators below 0, inside [0,127] and above 127; L1 outputs that
// saturate CReLU and SqrCReLU both ways), see tests/test_oracle.py.
void synthesize_net(uint64_t seed, uint32_t hd, uint32_t flags, Net& net, int variant) {
  Rng g{seed * 0x2545F4914F6CDD1Dull + hd + 0x9E3779B97F4A7C15ull * (uint64_t)variant};
  net.variant = variant;
  net.nfeat = features_of(variant);
  net.hd = hd;
  net.file_hash = ft_hash(hd, variant) ^ net_hash(hd);
  net.desc = "fishnet-amd synthetic SFNNv5 net seed=" + std::to_string(seed) + " hd=" + std::to_string(hd) +
             " flags=" + std::to_string(flags) +
             (variant ? " variant=" + std::string(variant == kVariantCrazyhouse ? "crazyhouse" : "atomic") : "");
  net.ft_bias.resize(hd);
  net.ft_w.resize((size_t)hd * net.nfeat);
  net.psqt_w.resize((size_t)kPsqtBuckets * net.nfeat);
  const bool wrap = flags & FNNUE_SYNTH_WRAP;
  for (auto& b : net.ft_bias) b = (int16_t)g.range(-16, 112);
  const double ftsd = wrap ? 9000.0 : 11.0;
  for (auto& w : net.ft_w) w = clampT<int16_t>(g.gauss() * ftsd, -32768, 32767);
  for (auto& p : net.psqt_w) p = clampT<int32_t>(g.gauss() * 450.0, -1e6, 1e6);
  for (int b = 0; b < kStacks; ++b) {
    Stack& s = net.st[b];
    for (auto& v : s.b0) v = (int32_t)g.range(-3000, 6000);
    s.w0.resize((size_t)kL2 * hd);
    const double sd0 = 4.0 * std::sqrt(1024.0 / hd);
    for (auto& w : s.w0) {
      const uint64_t r = g.next() % 2048;
      w = r == 0 ? (int8_t)-128 : (r == 1 ? (int8_t)127 : clampT<int8_t>(g.gauss() * sd0, -128, 127));
    }
    for (auto& v : s.b1) v = (int32_t)g.range(-2000, 5000);
    for (int o = 0; o < kL3; ++o)
      for (int i = 0; i < kFc1In; ++i) {
        const bool pad = i >= 30;
        s.w1[o * kFc1In + i] = (pad && !(flags & FNNUE_SYNTH_FC1_PAD)) ? 0 : clampT<int8_t>(g.gauss() * 18.0, -128, 127);
      }
    s.b2 = (int32_t)g.range(-2000, 2000);
    for (auto& w : s.w2) w = clampT<int8_t>(g.gauss() * 40.0, -128, 127);
  }
}

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

ImageLayout image_layout(uint32_t hd, uint32_t nfeat) {
  ImageLayout L{};
  size_t o = 0;
  L.ft_w = o;    o = align256(o + (size_t)(nfeat + 1) * hd * sizeof(int16_t));
  L.ft_bias = o; o = align256(o + (size_t)hd * sizeof(int16_t));
  L.psqt_w = o;  o = align256(o + (size_t)(nfeat + 1) * kPsqtBuckets * sizeof(int32_t));
  L.w0 = o;      o = align256(o + (size_t)kStacks * kL2 * hd);
  L.b0 = o;      o = align256(o + (size_t)kStacks * kL2 * sizeof(int32_t));
  L.w1 = o;      o = align256(o + (size_t)kStacks * kL3 * kFc1In);
  L.b1 = o;      o = align256(o + (size_t)kStacks * kL3 * sizeof(int32_t));
  L.w2 = o;      o = align256(o + (size_t)kStacks * kL3);
  L.b2 = o;      o = align256(o + (size_t)kStacks * sizeof(int32_t));
  L.total = o;
  return L;
}

void pack_image(const Net& net, uint8_t* dst) {
  const uint32_t hd = net.hd;
  const ImageLayout L = image_layout(hd, net.nfeat);
  std::memset(dst, 0, L.total);
  std::memcpy(dst + L.ft_w, net.ft_w.data(), net.ft_w.size() * sizeof(int16_t));
  std::memcpy(dst + L.ft_bias, net.ft_bias.data(), hd * sizeof(int16_t));
  std::memcpy(dst + L.psqt_w, net.psqt_w.data(), net.psqt_w.size() * sizeof(int32_t));
  for (int b = 0; b < kStacks; ++b) {
    const Stack& s = net.st[b];
    std::memcpy(dst + L.w0 + (size_t)b * kL2 * hd, s.w0.data(), (size_t)kL2 * hd);
    std::memcpy(dst + L.b0 + (size_t)b * kL2 * 4, s.b0, kL2 * 4);
    std::memcpy(dst + L.w1 + (size_t)b * kL3 * kFc1In, s.w1, kL3 * kFc1In);
    std::memcpy(dst + L.b1 + (size_t)b * kL3 * 4, s.b1, kL3 * 4);
    std::memcpy(dst + L.w2 + (size_t)b * kL3, s.w2, kL3);
    std::memcpy(dst + L.b2 + (size_t)b * 4, &s.b2, 4);
  }
}

int32_t accumulator_bound(const int16_t* ft_w, const int16_t* ft_bias, uint32_t hd, int variant) {
  const int kRows = (int)(variant == kVariantChess ? kFeatures / 32 : variant_rows(variant));  // rows per king block
  const int kBlocks = variant == kVariantChess ? 32 : 64;
  // Columns a SWAR word's exactness depends on: the first half's even columns
  // (low halves, partial sums must stay in int16) and every second-half column,
  // counted twice (kept doubled in the tile, swar_word_hi in sliced_common.h).
  std::vector<uint32_t> cols;
  for (uint32_t c = 0; c < hd / 2; c += 2) cols.push_back(c);
  for (uint32_t c = hd / 2; c < hd; ++c) cols.push_back(c);
  const size_t ncol = cols.size();
  int64_t worst = 0;
  std::vector<int32_t> mag(ncol * kRows);  // [column][row], |w|
  for (int kb = 0; kb < kBlocks; ++kb) {
    // own-king row of king block kb: plane 10, oriented king square on files e-h
    // (KingBuckets is a bijection kb <-> oriented square; upstream half_ka_v2_hm.h);
    // variants: block kb = oriented king square itself
    const int krow = variant == kVariantChess ? 640 + 8 * (7 - (kb >> 2)) + (7 - (kb & 3)) : 640 + kb;
    const int16_t* blk = ft_w + (size_t)kb * kRows * hd;
    for (int r = 0; r < kRows; ++r)
      for (size_t i = 0; i < ncol; ++i)
        mag[i * kRows + r] = r == krow ? 0 : std::abs((int32_t)blk[(size_t)r * hd + cols[i]]);
    for (size_t i = 0; i < ncol; ++i) {
      int32_t* m = mag.data() + i * kRows;
      std::nth_element(m, m + 31, m + kRows, std::greater<int32_t>());
      int64_t b = std::abs((int32_t)ft_bias[cols[i]] + (int32_t)blk[(size_t)krow * hd + cols[i]]);
      for (int k = 0; k < 31; ++k) b += m[k];
      worst = std::max(worst, cols[i] < hd / 2 ? b : 2 * b);
    }
  }
  return (int32_t)std::min<int64_t>(worst, INT32_MAX);
}

}  // namespace fnnue
