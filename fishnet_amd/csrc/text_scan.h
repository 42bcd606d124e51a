// text_scan.h — host-only token scan of the engine actor's move text
// (backend.cpp), kept free of HIP so the sanitizer tests build it with g++
// (tests/sanitize/text_scan_check.cpp).
#pragma once
#include <immintrin.h>

#include <cstddef>
#include <cstdint>

namespace fnnue {

// The builder's rule (replay_wave.h): blanks are ' ', '\t', '\n', '\r'; a
// token starts at a non-blank byte whose predecessor is blank or the string's
// start.  One byte at a time; *len = the string's length.
inline size_t scan_tokens_scalar(const char* s, size_t* len) {
  size_t tokens = 0, i = 0;
  bool prev_ws = true;
  for (; s[i]; ++i) {
    const char c = s[i];
    const bool ws = c == ' ' || c == '\t' || c == '\n' || c == '\r';
    tokens += !ws && prev_ws;
    prev_ws = ws;
  }
  *len = i;
  return tokens;
}

// The same in one pass, 16 bytes at a time.  The loads are aligned, so they
// never leave the page holding the terminator, but they do read bytes before
// s and past the terminator: AddressSanitizer builds take the scalar form.
inline size_t scan_tokens(const char* s, size_t* len) {
#if defined(__SANITIZE_ADDRESS__)
  return scan_tokens_scalar(s, len);
#else
  const char* base = reinterpret_cast<const char*>(reinterpret_cast<uintptr_t>(s) & ~(uintptr_t)15);
  const __m128i sp = _mm_set1_epi8(' '), tab = _mm_set1_epi8('\t'), nl = _mm_set1_epi8('\n'), cr = _mm_set1_epi8('\r');
  uint32_t pre = (1u << (s - base)) - 1;  // bytes before s: blank, not the end
  uint32_t prev_ws = 1;
  size_t tokens = 0;
  for (const char* p = base;; p += 16, pre = 0) {
    const __m128i v = _mm_load_si128(reinterpret_cast<const __m128i*>(p));
    uint32_t z = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(v, _mm_setzero_si128())) & ~pre;
    const __m128i w = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, sp), _mm_cmpeq_epi8(v, tab)),
                                   _mm_or_si128(_mm_cmpeq_epi8(v, nl), _mm_cmpeq_epi8(v, cr)));
    uint32_t ws = (uint32_t)_mm_movemask_epi8(w) | pre;
    if (z) ws |= ~((1u << __builtin_ctz(z)) - 1) & 0xFFFFu;  // the terminator and what follows: blank
    const uint32_t starts = ~ws & ((ws << 1) | prev_ws) & 0xFFFFu;
    tokens += (size_t)__builtin_popcount(starts);
    if (z) {
      *len = (size_t)(p - s) + (size_t)__builtin_ctz(z);
      return tokens;
    }
    prev_ws = (ws >> 15) & 1u;
  }
#endif
}

}  // namespace fnnue
