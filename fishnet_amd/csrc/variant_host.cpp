// variant_host.cpp — host side of the Fairy-Stockfish variant path: FEN with
// crazyhouse holdings -> fnnue_vpos, and seeded random walks that produce
// variant positions for tests and the bench (include/fnnue.h).
#include <cstring>
#include <string>
#include <vector>

#include "board.h"
#include "internal.h"

using namespace fnnue;
using namespace fnnue::detail;

namespace {

struct VState {
  uint8_t b[64];
  int stm;
  uint8_t hand[10];  // white P N B R Q, black P N B R Q
};

fnnue_vpos pack_v(const VState& v) {
  fnnue_vpos p;
  std::memset(&p, 0, sizeof p);
  for (int s = 0; s < 64; ++s) p.sq[s >> 1] |= (uint8_t)(v.b[s] << (4 * (s & 1)));
  p.stm = (uint8_t)v.stm;
  std::memcpy(p.hand, v.hand, 10);
  return p;
}

int piece_of(char c) {
  const char* w = "PNBRQK";
  const char* k = "pnbrqk";
  for (int i = 0; i < 6; ++i) {
    if (c == w[i]) return i + 1;
    if (c == k[i]) return i + 9;
  }
  return 0;
}

void start_position(VState& v) {
  std::memset(&v, 0, sizeof v);
  const int back[8] = {4, 2, 3, 5, 6, 3, 2, 4};
  for (int f = 0; f < 8; ++f) {
    v.b[f] = (uint8_t)back[f];
    v.b[8 + f] = 1;
    v.b[48 + f] = 9;
    v.b[56 + f] = (uint8_t)(back[f] | 8);
  }
}

bool near_king(const VState& v, int sq) {
  for (int dr = -1; dr <= 1; ++dr)
    for (int df = -1; df <= 1; ++df) {
      const int r = (sq >> 3) + dr, f = (sq & 7) + df;
      if (r < 0 || r > 7 || f < 0 || f > 7) continue;
      if ((v.b[r * 8 + f] & 7) == 6) return true;
    }
  return false;
}

// One pseudo-legal step (no chess movement rules: any own piece to any square
// not holding an own piece or a king; kings step to a neighbour).  Feature-wise
// it exercises exactly what real play does: moves, captures, promotions and,
// per variant, pockets (crazyhouse) or explosions (atomic).
void random_step(VState& v, uint64_t& st, int variant) {
  const int us = v.stm;
  uint8_t* hand = v.hand + 5 * us;
  int htot = 0;
  for (int i = 0; i < 5; ++i) htot += hand[i];
  if (variant == kVariantCrazyhouse && htot && splitmix64(st) % 3 == 0) {
    int k = (int)(splitmix64(st) % (uint64_t)htot), pt = 0;
    while (k >= hand[pt]) k -= hand[pt++];
    for (int tries = 0; tries < 64; ++tries) {
      const int sq = (int)(splitmix64(st) % 64);
      if (v.b[sq] || (pt == 0 && (sq < 8 || sq >= 56))) continue;
      v.b[sq] = (uint8_t)((us << 3) | (pt + 1));
      --hand[pt];
      v.stm ^= 1;
      return;
    }
  }
  int own[32], n = 0;
  for (int s = 0; s < 64; ++s)
    if (v.b[s] && (v.b[s] >> 3) == us) own[n++] = s;
  for (int tries = 0; tries < 64; ++tries) {
    const int from = own[splitmix64(st) % (uint64_t)n];
    const int pc = v.b[from];
    int to;
    if ((pc & 7) == 6) {
      const int dr = (int)(splitmix64(st) % 3) - 1, df = (int)(splitmix64(st) % 3) - 1;
      const int r = (from >> 3) + dr, f = (from & 7) + df;
      if ((!dr && !df) || r < 0 || r > 7 || f < 0 || f > 7) continue;
      to = r * 8 + f;
    } else {
      to = (int)(splitmix64(st) % 64);
    }
    const int cap = v.b[to];
    if (to == from || (cap && (cap >> 3) == us) || (cap & 7) == 6) continue;
    int moved = pc;
    if ((pc & 7) == 1 && (to < 8 || to >= 56)) moved = (us << 3) | 5;  // promotion to a queen
    if (cap && variant == kVariantCrazyhouse) {
      const int t = (cap & 7) - 1;  // captured piece joins the capturer's hand
      if (hand[t] >= kVHandSlots) continue;
      ++hand[t];
    }
    if (cap && variant == kVariantAtomic) {
      if ((pc & 7) == 6 || near_king(v, to)) continue;  // an explosion never takes a king here
      v.b[from] = 0;
      v.b[to] = 0;  // the capturer explodes with its victim
      for (int dr = -1; dr <= 1; ++dr)
        for (int df = -1; df <= 1; ++df) {
          const int r = (to >> 3) + dr, f = (to & 7) + df;
          if (r < 0 || r > 7 || f < 0 || f > 7) continue;
          uint8_t& x = v.b[r * 8 + f];
          if (x && (x & 7) != 1) x = 0;  // pawns survive
        }
      v.stm ^= 1;
      return;
    }
    v.b[from] = 0;
    v.b[to] = (uint8_t)moved;
    v.stm ^= 1;
    return;
  }
  v.stm ^= 1;  // nothing found: pass
}

}  // namespace

extern "C" {

int fnnue_vpos_from_fen(int variant, const char* fen, fnnue_vpos* out) {
  if (!fen || !out) return fail(FNNUE_E_ARG, "null argument");
  if (variant != FNNUE_VARIANT_CRAZYHOUSE && variant != FNNUE_VARIANT_ATOMIC)
    return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  VState v;
  std::memset(&v, 0, sizeof v);
  const char* p = fen;
  int rank = 7, file = 0;
  bool holdings = false;
  for (; *p && *p != ' '; ++p) {
    const char c = *p;
    if (c == '[') { holdings = true; continue; }
    if (c == ']') { holdings = false; continue; }
    if (c == '~') continue;  // promoted-piece mark
    if (c == '/') {
      if (--rank < 0) holdings = true;  // a 9th field: holdings
      file = 0;
      continue;
    }
    if (holdings) {
      const int pc = piece_of(c);
      if (!pc || (pc & 7) == 6 || c == '-') {
        if (c == '-') continue;
        return fail(FNNUE_E_FEN, std::string("bad holdings piece '") + c + "'");
      }
      uint8_t& h = v.hand[5 * (pc >> 3) + (pc & 7) - 1];
      if (h >= kVHandSlots) return fail(FNNUE_E_FEN, "too many pieces in hand");
      ++h;
      continue;
    }
    if (c >= '1' && c <= '8') {
      file += c - '0';
      continue;
    }
    const int pc = piece_of(c);
    if (!pc || file > 7 || rank < 0) return fail(FNNUE_E_FEN, "bad placement");
    v.b[rank * 8 + file++] = (uint8_t)pc;
  }
  while (*p == ' ') ++p;
  if (*p != 'w' && *p != 'b') return fail(FNNUE_E_FEN, "missing side to move");
  v.stm = *p == 'b';
  int hand_total = 0, n = 0, wk = 0, bk = 0;
  for (int i = 0; i < 10; ++i) hand_total += v.hand[i];
  for (int s = 0; s < 64; ++s) {
    n += v.b[s] != 0;
    wk += v.b[s] == 6;
    bk += v.b[s] == 14;
  }
  if (wk != 1 || bk != 1) return fail(FNNUE_E_FEN, "needs one king per side");
  if (hand_total && variant != FNNUE_VARIANT_CRAZYHOUSE) return fail(FNNUE_E_FEN, "holdings in a variant without pockets");
  if (n + hand_total > 32) return fail(FNNUE_E_FEN, "more than 32 pieces on board and in hand");
  *out = pack_v(v);
  return FNNUE_OK;
}

int fnnue_random_vpositions(uint64_t seed, int variant, size_t count, uint32_t max_plies, int mode, fnnue_vpos* out,
                            size_t cap, uint32_t* off, size_t off_cap, size_t* n_out, size_t* n_groups) {
  if (!n_out || !n_groups) return fail(FNNUE_E_ARG, "null argument");
  if (variant != FNNUE_VARIANT_CRAZYHOUSE && variant != FNNUE_VARIANT_ATOMIC)
    return fail(FNNUE_E_ARG, "unknown variant " + std::to_string(variant));
  if (mode != FNNUE_PLAYOUT_FINAL && mode != FNNUE_PLAYOUT_PLIES) return fail(FNNUE_E_ARG, "bad mode");
  std::vector<fnnue_vpos> res;
  std::vector<uint32_t> offs{0};
  try {
    for (size_t i = 0; i < count; ++i) {
      uint64_t st = seed ^ (0xD1B54A32D192ED03ull * (i + 1));
      const uint32_t L = (uint32_t)(splitmix64(st) % ((uint64_t)max_plies + 1));
      VState v;
      start_position(v);
      if (mode == FNNUE_PLAYOUT_PLIES) res.push_back(pack_v(v));
      for (uint32_t k = 0; k < L; ++k) {
        random_step(v, st, variant);
        if (mode == FNNUE_PLAYOUT_PLIES) res.push_back(pack_v(v));
      }
      if (mode == FNNUE_PLAYOUT_FINAL) res.push_back(pack_v(v));
      else offs.push_back((uint32_t)res.size());
    }
  } catch (const std::bad_alloc&) {
    return fail(FNNUE_E_OOM, "host allocation failed");
  }
  *n_out = res.size();
  *n_groups = offs.size() - 1;
  if (!out || cap < res.size()) return fail(FNNUE_E_CAPACITY, "output buffer too small");
  if (mode == FNNUE_PLAYOUT_PLIES && (!off || off_cap < offs.size())) return fail(FNNUE_E_CAPACITY, "offset buffer too small");
  std::memcpy(out, res.data(), res.size() * sizeof(fnnue_vpos));
  if (mode == FNNUE_PLAYOUT_PLIES) std::memcpy(off, offs.data(), offs.size() * sizeof(uint32_t));
  return FNNUE_OK;
}

}  // extern "C"
