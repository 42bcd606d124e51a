// ThreadSanitizer stress of the engine actor's host thread pool
// (fishnet_amd/csrc/workers.h): many runs of every size against the chunk
// grain — each index covered exactly once, every run joined before the next,
// no data race reported.  Built and run by tests/test_sanitizers.py.
#include <cstdio>

#include "../../fishnet_amd/csrc/workers.h"

int main() {
  fnnue::Workers w;
  w.start(16);
  long total = 0;
  for (int it = 0; it < 40000; ++it) {
    const size_t n = 1 + (size_t)(it * 7919) % 3000;
    const size_t grain = it % 5 == 0 ? 512 : 1 + (size_t)(it % 300);
    std::vector<unsigned char> hit(n, 0);
    w.run(n, grain, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) ++hit[i];
    });
    for (size_t i = 0; i < n; ++i)
      if (hit[i] != 1) {
        std::printf("run %d: index %zu covered %d times\n", it, i, hit[i]);
        return 1;
      }
    total += (long)n;
  }
  w.stop();
  std::printf("workers stress ok %ld\n", total);
  return 0;
}
