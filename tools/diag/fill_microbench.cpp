// Host microbenchmark of the engine actor's response fill (backend.cpp fill()):
// a response built on the stack and copied out vs written in place, and the
// cp conversion by integer vs double division (exact over the tested range).
//   g++ -O2 -march=x86-64-v3 -o /tmp/fill tools/diag/fill_microbench.cpp && /tmp/fill
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <emmintrin.h>
#include <cstddef>
#include "../../include/fnnue_backend.h"
static inline int64_t to_cp(int32_t psqt, int32_t positional, int32_t norm) {
  const int64_t v = ((int64_t)psqt + positional) / 16;
  return v * 100 / norm;
}
static inline int64_t to_cp_d(int32_t psqt, int32_t positional, int32_t norm) {
  const int64_t v = ((int64_t)psqt + positional) / 16;
  return (int64_t)((double)(v * 100) / (double)norm);
}
int main() {
  const size_t n = 102400;
  std::vector<fnnue_position_response> out(n);
  std::vector<int32_t> ps(n), po(n);
  for (size_t i = 0; i < n; ++i) { ps[i] = (int)(i * 2654435761u) % 40000 - 20000; po[i] = (int)(i * 40503u) % 30000 - 15000; }
  volatile int32_t nv = 361; int32_t nrm = nv;
  for (int variant = 0; variant < 6; ++variant) {
    double best = 1e9;
    for (int rep = 0; rep < 50; ++rep) {
      auto t0 = std::chrono::steady_clock::now();
      if (variant == 3) {
        for (size_t q = 0; q < n; ++q) {
          fnnue_position_response& r = out[q];
          std::memset(&r, 0, sizeof(r));
          r.position_id = (uint32_t)q;
          r.time_ms = 5; r.nps = 7;
          r.psqt = ps[q]; r.positional = po[q];
          r.score_kind = 1;
          r.score = to_cp(ps[q], po[q], nrm);
          r.nodes = 1;
        }
      } else if (variant == 5) {
        // three 16-byte stores and one 8-byte store per record; the time / nps
        // / best-move bytes are the same for the whole piece
        static_assert(offsetof(fnnue_position_response, score) == 8 && offsetof(fnnue_position_response, psqt) == 16 &&
                      offsetof(fnnue_position_response, time_ms) == 32 && sizeof(fnnue_position_response) == 56, "");
        const __m128i hi = _mm_set_epi64x((long long)7, (long long)5);
        char* base = reinterpret_cast<char*>(out.data());
        for (size_t q = 0; q < n; ++q) {
          char* r = base + 56 * q;
          const int64_t sc = to_cp(ps[q], po[q], nrm);
          _mm_storeu_si128(reinterpret_cast<__m128i*>(r), _mm_set_epi64x(sc, (long long)(uint32_t)q));
          _mm_storeu_si128(reinterpret_cast<__m128i*>(r + 16),
                           _mm_set_epi64x(1, (long long)((uint64_t)(uint32_t)ps[q] | (uint64_t)(uint32_t)po[q] << 32)));
          _mm_storeu_si128(reinterpret_cast<__m128i*>(r + 32), hi);
          _mm_storel_epi64(reinterpret_cast<__m128i*>(r + 48), _mm_setzero_si128());
        }
      } else if (variant == 4) {
        for (size_t q = 0; q < n; ++q) {
          fnnue_position_response r{};
          r.position_id = (uint32_t)q;
          r.time_ms = 5; r.nps = 7;
          r.psqt = ps[q]; r.positional = po[q];
          r.score_kind = 1;
          r.score = to_cp(ps[q], po[q], nrm);
          r.nodes = 1;
          uint64_t w[7]; std::memcpy(w, &r, 56);
          std::memcpy(&out[q], w, 56);
        }
      } else
      for (size_t q = 0; q < n; ++q) {
        fnnue_position_response r;
        std::memset(&r, 0, sizeof(r));
        r.position_id = (uint32_t)q;
        r.time_ms = 5; r.nps = 7; r.matrix = 0;
        r.psqt = ps[q]; r.positional = po[q];
        r.score_kind = 1;
        r.score = variant == 0 ? to_cp(r.psqt, r.positional, nrm) : variant == 1 ? to_cp_d(r.psqt, r.positional, nrm) : 0;
        r.nodes = 1;
        out[q] = r;
      }
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    long chk = 0; for (size_t q = 0; q < n; ++q) chk += out[q].score;
    printf("variant %d: %.3f ms per 102k (single thread) chk %ld\n", variant, best, chk);
  }
  // exactness of the double form over a wide range
  long bad = 0;
  for (int64_t s = -3000000; s <= 3000000; s += 7) for (int32_t nn : {361, 100, 328, 1, 65535}) {
    int64_t v = s / 16; if (v * 100 / nn != (int64_t)((double)(v * 100) / (double)nn)) ++bad; }
  printf("mismatches %ld\n", bad);
}
