// Host-side sanitizer driver (tests/test_sanitizers.py builds it with
// -fsanitize=address,undefined and runs it on the CPU): the product's host code
// (net.cpp parser / writer / generator, board.cpp FEN / UCI / movegen / perft /
// packing) and the oracle (scalar + SIMD CPU paths), fed valid and corrupt
// inputs.  Exit 0 = every check passed and the sanitizers stayed silent.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../fishnet_amd/csrc/board.h"
#include "../../fishnet_amd/csrc/net.h"

extern "C" {
#include "../../oracle/nnue_oracle.h"
int oracle_net_load_mem(const void* buf, size_t len, onet** out);
void oracle_net_free(onet* n);
int oracle_eval_packed(const onet* n, const uint8_t* packed, size_t count, int32_t* psqt, int32_t* positional,
                       int threads);
int cpu_simd_eval_packed(const onet* n, const uint8_t* packed, size_t count, int32_t* psqt, int32_t* positional,
                         int threads);
int cpu_simd_eval_groups(const onet* n, const uint8_t* packed, const uint32_t* off, size_t ngroups, int mode,
                         int32_t* psqt, int32_t* positional, int threads);
int cpu_simd_set_isa(int isa512);
int voracle_eval_packed(const onet* n, const uint8_t* packed, size_t count, int32_t* psqt, int32_t* positional,
                        int threads);
int voracle_eval_groups(const onet* n, const uint8_t* packed, const uint32_t* off, size_t ngroups, int mode,
                        int32_t* psqt, int32_t* positional);
}

using namespace fnnue;

static int failures = 0;
#define CHECK(cond, what)                                                    \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "FAIL %s (%s:%d)\n", what, __FILE__, __LINE__);   \
      ++failures;                                                            \
    }                                                                        \
  } while (0)

static const char* kFens[] = {
    "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
    "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
    "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
    "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1",
    "bqnb1rkr/pp3ppp/3ppn2/2p5/5P2/P2P4/NPP1P1PP/BQ1BNRKR w HFhf - 2 9",
};
static const uint64_t kPerft3[] = {8902, 97862, 2812, 9467, 0};
static const char* kBadFens[] = {
    "", "garbage", "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP w", "9/8/8/8/8/8/8/8 w - - 0 1",
    "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR x KQkq - 0 1",
    "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNRR w KQkq - 0 1", "8/8/8/8/8/8/8/8 w - - 0 1",
};

int main() {
  // ---- board: FEN, perft, UCI round trips, random playouts ----
  for (int i = 0; i < 5; ++i) {
    Board b;
    std::string err;
    CHECK(board_from_fen(kFens[i], b, &err), "valid FEN parses");
    if (kPerft3[i]) CHECK(perft(b, 3) == kPerft3[i], "perft depth 3");
    std::vector<Move> mv;
    b.legal_moves(mv);
    for (const Move& m : mv) {
      Move back;
      CHECK(parse_uci(b, b.uci(m, b.chess960).c_str(), back), "uci round trip");
      Board c = b;
      c.do_move(m);
      (void)c.pack();
      (void)c.fen();
    }
  }
  for (const char* f : kBadFens) {
    Board b;
    std::string err;
    CHECK(!board_from_fen(f, b, &err), "malformed FEN rejected");
  }
  {
    Board b;
    board_from_fen(kFens[0], b, nullptr);
    Move m;
    for (const char* u : {"", "e2", "e2e5", "e7e5", "a1a1", "e2e4q", "zz99", "e1g1x"})
      CHECK(!parse_uci(b, u, m), "illegal or malformed UCI rejected");
  }
  std::vector<fnnue_pos> pos;
  uint64_t rng = 12345;
  for (int g = 0; g < 60; ++g) {
    Board b;
    board_from_fen(kFens[g % 5], b, nullptr);
    const int plies = (int)(splitmix64(rng) % 120);
    for (int k = 0; k < plies; ++k) {
      Move m;
      if (!b.random_legal_move(rng, m)) break;
      b.do_move(m);
      pos.push_back(b.pack());
    }
  }
  CHECK(pos.size() > 100, "random playouts produced positions");

  // ---- nets: synthesize, write (plain / LEB128), parse; corrupt copies fail cleanly ----
  for (uint32_t flags : {0u, (uint32_t)FNNUE_SYNTH_WRAP, (uint32_t)FNNUE_SYNTH_FC1_PAD}) {
    Net net;
    synthesize_net(7 + flags, 128, flags, net);
    for (bool leb : {false, true}) {
      std::vector<uint8_t> buf;
      write_net(net, leb, buf);
      Net back;
      std::string err;
      CHECK(parse_net(buf.data(), buf.size(), back, err) == 0, "synthetic net parses");
      CHECK(back.ft_w == net.ft_w && back.psqt_w == net.psqt_w, "parse(write(net)) == net");
      std::vector<uint8_t> img(image_layout(back.hd).total);
      pack_image(back, img.data());
      for (size_t cut : {(size_t)0, (size_t)3, (size_t)12, (size_t)40, buf.size() / 2, buf.size() - 1}) {
        Net bad;
        CHECK(parse_net(buf.data(), cut, bad, err) != 0, "truncated net rejected");
      }
      for (size_t at : {(size_t)0, (size_t)5, (size_t)13, (size_t)(buf.size() - 3)}) {
        std::vector<uint8_t> c = buf;
        c[at] ^= 0x5A;
        Net bad;
        (void)parse_net(c.data(), c.size(), bad, err);  // any return code; no crash, no overread
      }
      std::vector<uint8_t> longer = buf;
      longer.push_back(0);
      Net bad;
      CHECK(parse_net(longer.data(), longer.size(), bad, err) != 0, "trailing bytes rejected");

      // ---- oracle: scalar vs SIMD (both ISAs) from scratch and as CHAIN groups ----
      onet* on = nullptr;
      CHECK(oracle_net_load_mem(buf.data(), buf.size(), &on) == 0, "oracle loads the net");
      if (!on) continue;
      const size_t n = pos.size();
      const uint8_t* pk = reinterpret_cast<const uint8_t*>(pos.data());
      std::vector<int32_t> a(n), b(n), c(n), d(n);
      CHECK(oracle_eval_packed(on, pk, n, a.data(), b.data(), 2) == 0, "scalar oracle");
      for (int isa : {0, 1}) {
        cpu_simd_set_isa(isa);
        CHECK(cpu_simd_eval_packed(on, pk, n, c.data(), d.data(), 2) == 0, "simd from scratch");
        CHECK(a == c && b == d, "simd == scalar (from scratch)");
        const uint32_t off[3] = {0, (uint32_t)(n / 2), (uint32_t)n};
        CHECK(cpu_simd_eval_groups(on, pk, off, 2, 0, c.data(), d.data(), 2) == 0, "simd chain");
        CHECK(a == c && b == d, "simd == scalar (chain)");
      }
      oracle_net_free(on);
      std::vector<uint8_t> cut(buf.begin(), buf.begin() + buf.size() / 3);
      onet* on2 = nullptr;
      CHECK(oracle_net_load_mem(cut.data(), cut.size(), &on2) != 0 && !on2, "oracle rejects a truncated net");
    }
  }
  // ---- Fairy-Stockfish variant nets: product parser/writer, variant restatement ----
  for (int variant : {kVariantCrazyhouse, kVariantAtomic}) {
    Net vn;
    synthesize_net(11, 256, 0, vn, variant);
    std::vector<uint8_t> vbuf;
    write_net(vn, variant == kVariantCrazyhouse, vbuf);
    Net back;
    std::string err;
    CHECK(parse_net(vbuf.data(), vbuf.size(), back, err, variant) == 0, "variant net round trip");
    CHECK(parse_net(vbuf.data(), vbuf.size(), back, err, kVariantChess) != 0, "variant net is not a chess net");
    CHECK(accumulator_bound(back.ft_w.data(), back.ft_bias.data(), back.hd, variant) < 32768, "variant bound");
    onet* von = nullptr;
    CHECK(oracle_net_load_variant_mem(vbuf.data(), vbuf.size(), variant, &von) == 0, "variant oracle loads");
    if (!von) continue;
    // start position (white / black to move) and kings only with 15 pieces in each hand (48-B records)
    std::vector<uint8_t> vp(48 * 3, 0);
    const uint8_t start[32] = {0x24, 0x53, 0x36, 0x42, 0x11, 0x11, 0x11, 0x11, 0, 0, 0, 0, 0, 0, 0, 0,
                               0,    0,    0,    0,    0,    0,    0,    0,    0x99, 0x99, 0x99, 0x99,
                               0xAC, 0xDB, 0xBE, 0xCA};
    std::memcpy(vp.data(), start, 32);
    std::memcpy(vp.data() + 48, start, 32);
    vp[48 + 32] = 1;
    vp[96 + 2] = 0x06;   // white king on e1 (square 4 = low nibble of byte 2)
    vp[96 + 30] = 0xE0;  // black king on f8 (square 61 = high nibble of byte 30)
    if (variant == kVariantCrazyhouse)
      for (int i = 0; i < 10; ++i) vp[96 + 33 + i] = i % 5 == 0 ? 7 : 2;
    std::vector<int32_t> a(3), b(3), c(3), d(3);
    (void)voracle_eval_packed(von, vp.data(), 3, a.data(), b.data(), 2);
    const uint32_t off[2] = {0, 3};
    (void)voracle_eval_groups(von, vp.data(), off, 1, 0, c.data(), d.data());
    CHECK(a == c && b == d, "variant incremental == refresh");
    oracle_net_free(von);
  }
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("sanitized host checks ok: %zu positions\n", pos.size());
  return 0;
}
