// Microbenchmark: VALU issue cost on gfx950 for the instructions of the
// ft_slices inner loop (v_pk_add_u16, v_add_u32_sdwa, v_add_u32), as a
// function of waves per SIMD.  Cycles from s_memtime (shader clock).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void k(unsigned* out, long long* cyc, int iters) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const unsigned b = blockIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#define OP(r)                                                                         \
    if (KIND == 0) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(b));       \
    else if (KIND == 1) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(r) : "v"(b)); \
    else asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));
    OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
    OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned* out;
  long long* cyc;
  hipMalloc(&out, 256u << 20);
  hipMalloc(&cyc, 64u << 20);
  const int iters = 4096;
  const char* names[3] = {"v_pk_add_u16", "v_add_u32_sdwa", "v_add_u32"};
  for (int kind = 0; kind < 3; ++kind)
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: one WG of 4*wps waves per CU
      dim3 grid(cus), block(256 * wps);
      auto launch = [&] {
        if (kind == 0) hipLaunchKernelGGL(k<0>, grid, block, 0, 0, out, cyc, iters);
        else if (kind == 1) hipLaunchKernelGGL(k<1>, grid, block, 0, 0, out, cyc, iters);
        else hipLaunchKernelGGL(k<2>, grid, block, 0, 0, out, cyc, iters);
      };
      launch();
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      long long h; hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
      const double instr_per_wave = 16.0 * iters;
      printf("%-16s waves/SIMD=%d  cycles/instr/wave=%.2f  => SIMD cycles/instr=%.2f  (%.3f ms, %.2f GHz implied)\n",
             names[kind], wps, h / instr_per_wave, h / instr_per_wave / wps, ms, h / (ms * 1e-3) / 1e9);
    }
  return 0;
}
