// xread_bench.hip — how fast can the layer-stack kernel read the x workspace?
// Standalone (no torch): 1M rows of 1024 B, persistent workgroups with
// contiguous 16-row tiles per wave, as stack_kernel.  Access shapes per load
// instruction:
//   mfma   16 rows x 64 B (lane l: row l&15, 16 B chunk 4s + (l>>4)): the
//          MFMA A-operand layout stack_kernel loads today
//   row128 8 rows x 128 B (lane l: row l>>3, chunk l&7), two instructions per
//          pair of K-steps
//   flat   one 1 KiB row per instruction (lane l: chunk l)
// Every variant reads each byte once and folds it into a checksum.
//   build: hipcc --offload-arch=gfx950 -O3 -o /tmp/xread tools/diag/xread_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int HD = 1024, KS = HD / 64;

template <int kShape, int kWaves>
__global__ __launch_bounds__(64 * kWaves) void xread(const uint8_t* __restrict__ x, uint32_t n, int* __restrict__ out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t ntiles = n / 16, nw = gridDim.x * kWaves, wid = blockIdx.x * kWaves + wv;
  const uint32_t per = (ntiles + nw - 1) / nw;
  const uint32_t t0 = wid * per, t1 = min(ntiles, t0 + per);
  v4i acc = (v4i)0;
  for (uint32_t t = t0; t < t1; ++t) {
    const v4i* base = reinterpret_cast<const v4i*>(x + (size_t)t * 16 * HD);
    v4i a[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      int row, chunk;
      if constexpr (kShape == 0) {
        row = lane & 15;
        chunk = 4 * s + (lane >> 4);
      } else if constexpr (kShape == 1) {
        row = (lane >> 3) + 8 * (s & 1);
        chunk = 8 * (s >> 1) + (lane & 7);
      } else {
        row = s;
        chunk = lane;
      }
      a[s] = __builtin_nontemporal_load(base + row * (HD / 16) + chunk);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) acc += a[s];
  }
  const int v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x7F3A5C11) atomicAdd(out, 1);
}

// Fills x the way ft_slices does (every byte written once, 4 B per lane) so
// the read that follows starts with dirty lines in L2 / the Infinity Cache.
__global__ __launch_bounds__(256) void xwrite(uint8_t* __restrict__ x, size_t words, uint32_t v) {
  uint32_t* w = reinterpret_cast<uint32_t*>(x);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
    w[i] = v ^ (uint32_t)i;
}

template <int kShape, int kWaves>
float run_dirty(uint8_t* x, uint32_t n, int* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(xwrite, dim3(4096), dim3(256), 0, 0, x, (size_t)n * HD / 4, (uint32_t)r);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((xread<kShape, kWaves>), dim3(256), dim3(64 * kWaves), 0, 0, x, n, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    tot += ms;
  }
  return tot / reps;
}

template <int kShape, int kWaves>
float run(const uint8_t* x, uint32_t n, int* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = 256;
  hipLaunchKernelGGL((xread<kShape, kWaves>), dim3(blocks), dim3(64 * kWaves), 0, 0, x, n, out);
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((xread<kShape, kWaves>), dim3(blocks), dim3(64 * kWaves), 0, 0, x, n, out);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const uint32_t n = 1u << 20;
  uint8_t* x = nullptr;
  int* out = nullptr;
  if (hipMalloc(&x, (size_t)n * HD) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(x, 3, (size_t)n * HD);
  (void)hipMemset(out, 0, 4);
  const double gb = (double)n * HD / 1e9;
  const char* names[3] = {"mfma 16x64B", "row128 8x128B", "flat 1x1KiB"};
  for (int rep = 0; rep < 2; ++rep) {
    float t[3][3];
    t[0][0] = run<0, 8>(x, n, out, 20);
    t[0][1] = run<0, 12>(x, n, out, 20);
    t[0][2] = run<0, 16>(x, n, out, 20);
    t[1][0] = run<1, 8>(x, n, out, 20);
    t[1][1] = run<1, 12>(x, n, out, 20);
    t[1][2] = run<1, 16>(x, n, out, 20);
    t[2][0] = run<2, 8>(x, n, out, 20);
    t[2][1] = run<2, 12>(x, n, out, 20);
    t[2][2] = run<2, 16>(x, n, out, 20);
    for (int s = 0; s < 3; ++s)
      printf("%-14s waves 8: %.1f us %.2f TB/s | 12: %.1f us %.2f TB/s | 16: %.1f us %.2f TB/s\n", names[s],
             t[s][0] * 1e3, gb / t[s][0], t[s][1] * 1e3, gb / t[s][1], t[s][2] * 1e3, gb / t[s][2]);
  }
  {
    const float d0 = run_dirty<0, 12>(x, n, out, 10), d1 = run_dirty<1, 12>(x, n, out, 10),
                d2 = run_dirty<2, 12>(x, n, out, 10);
    printf("after a 1 GiB write, 12 waves: mfma %.1f us %.2f TB/s | row128 %.1f us %.2f TB/s | flat %.1f us %.2f TB/s\n",
           d0 * 1e3, gb / d0, d1 * 1e3, gb / d1, d2 * 1e3, gb / d2);
  }
  hipError_t e = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(e));
  (void)hipFree(x);
  (void)hipFree(out);
  return e == hipSuccess ? 0 : 1;
}
