// The engine actor's move-text scan (fishnet_amd/csrc/text_scan.h) on
// server-shaped text: every string is copied into an allocation of exactly
// its length + 1 at every offset mod 16, and also ending at the last byte of a
// page followed by an inaccessible page.  Built twice by
// tests/test_sanitizers.py: under ASan + UBSan (scan_tokens is then the
// scalar form: every byte read must be inside the allocation) and under UBSan
// alone (the 16-byte form, compared with the scalar one; the guard page
// catches a load past the terminator's page).
#include <sys/mman.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../fishnet_amd/csrc/text_scan.h"

using fnnue::scan_tokens;
using fnnue::scan_tokens_scalar;

static int failures = 0;

static void check(const char* s, const std::string& what) {
  size_t l1 = 0, l2 = 0;
  const size_t a = scan_tokens(s, &l1), b = scan_tokens_scalar(s, &l2);
  if (a != b || l1 != l2) {
    if (++failures < 10)
      std::printf("mismatch (%s): tokens %zu vs %zu, len %zu vs %zu\n", what.c_str(), a, b, l1, l2);
  }
}

int main() {
  std::mt19937_64 rng(7);
  std::vector<std::string> texts = {"", " ", "e2e4", " e2e4", "e2e4 ", "e2e4  e7e5\t\tg1f3\r\nb8c6",
                                    std::string(15, ' '), std::string(16, 'a'), std::string(17, ' ') + "x"};
  const char alpha[] = "abcdefgh12345678qrnb \t\r\n";
  for (int i = 0; i < 3000; ++i) {
    const size_t len = rng() % 300;
    std::string t(len, ' ');
    for (char& c : t) c = alpha[rng() % (sizeof(alpha) - 1)];
    texts.push_back(t);
  }
  // a long lichess-shaped move list
  std::string game;
  for (int i = 0; i < 400; ++i) game += (i ? " " : "") + std::string("e2e4");
  texts.push_back(game);
  size_t n = 0;
  for (const std::string& t : texts) {
    for (size_t off = 0; off < 16; ++off) {
      char* raw = static_cast<char*>(std::malloc(t.size() + 1 + off));
      std::memcpy(raw + off, t.c_str(), t.size() + 1);
      check(raw + off, "heap+" + std::to_string(off));
      std::free(raw);
      ++n;
    }
  }
  // ending at the last byte of a page, the next page inaccessible
  const long pg = sysconf(_SC_PAGESIZE);
  char* two = static_cast<char*>(mmap(nullptr, 2 * pg, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
  if (two == MAP_FAILED || mprotect(two + pg, pg, PROT_NONE) != 0) {
    std::printf("mmap failed\n");
    return 2;
  }
  for (const std::string& t : texts) {
    if ((long)t.size() + 1 > pg) continue;
    char* s = two + pg - (t.size() + 1);
    std::memcpy(s, t.c_str(), t.size() + 1);
    check(s, "page end");
    ++n;
  }
  munmap(two, 2 * pg);
  if (failures) {
    std::printf("%d mismatches\n", failures);
    return 1;
  }
  std::printf("text scan ok: %zu strings\n", n);
  return 0;
}
