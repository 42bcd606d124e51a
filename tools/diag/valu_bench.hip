// Microbenchmark: relative VALU issue cost on gfx950 of candidate instructions
// for the ft_slices inner loop, 4 waves per SIMD (one 1024-thread WG per CU),
// 8 independent accumulators per lane.  Reported relative to v_add_u32.
#include <hip/hip_runtime.h>
#include <cstdio>

#define BODY(INSN) \
  OP(INSN, a0) OP(INSN, a1) OP(INSN, a2) OP(INSN, a3) OP(INSN, a4) OP(INSN, a5) OP(INSN, a6) OP(INSN, a7)
#define OP(INSN, r) asm volatile(INSN : "+v"(r) : "v"(b), "v"(c));

#define KERNEL(NAME, INSN)                                                                          \
  __global__ void NAME(unsigned* out, int iters) {                                                  \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
             a6 = a0 + 6, a7 = a0 + 7;                                                              \
    const unsigned b = blockIdx.x, c = threadIdx.x * 3;                                             \
    for (int i = 0; i < iters; ++i) { BODY(INSN) BODY(INSN) }                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
  }

KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_pkadd, "v_pk_add_u16 %0, %0, %1")
KERNEL(k_sdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1")
KERNEL(k_mad16, "v_mad_u32_u16 %0, %1, 16, %0 op_sel:[1,0,0,0]")
KERNEL(k_lshladd, "v_lshl_add_u32 %0, %0, 4, %1")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 16, 16")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_pkmax, "v_pk_max_i16 %0, %0, %1")
KERNEL(k_pkmul, "v_pk_mul_lo_u16 %0, %0, %1")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_mov, "v_mov_b32 %0, %1")

// 64-bit SWAR candidate: one v_lshl_add_u64 adds four
// int16 columns held as one 64-bit word (shift 0), vs two v_add_u32.
#define OP64(INSN, r) asm volatile(INSN : "+v"(r) : "v"(b64));
#define BODY64(INSN) \
  OP64(INSN, a0) OP64(INSN, a1) OP64(INSN, a2) OP64(INSN, a3) OP64(INSN, a4) OP64(INSN, a5) OP64(INSN, a6) OP64(INSN, a7)
#define KERNEL64(NAME, INSN)                                                                        \
  __global__ void NAME(unsigned* out, int iters) {                                                  \
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,        \
                       a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                       \
    const unsigned long long b64 = ((unsigned long long)blockIdx.x << 32) | threadIdx.x;            \
    for (int i = 0; i < iters; ++i) { BODY64(INSN) BODY64(INSN) }                                   \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
  }
KERNEL64(k_lshladd64, "v_lshl_add_u64 %0, %0, 0, %1")

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned* out;
  (void)hipMalloc(&out, 256u << 20);
  const int iters = 8192;
  struct K { const char* name; void (*fn)(unsigned*, int); };
  K ks[] = {{"v_add_u32", k_add}, {"v_add3_u32", k_add3}, {"v_pk_add_u16", k_pkadd}, {"v_add_u32_sdwa", k_sdwa},
            {"v_mad_u32_u16", k_mad16}, {"v_lshl_add_u32", k_lshladd}, {"v_bfe_u32", k_bfe}, {"v_perm_b32", k_perm},
            {"v_pk_max_i16", k_pkmax}, {"v_pk_mul_lo_u16", k_pkmul}, 
            {"v_and_or_b32", k_and_or}, {"v_mov_b32", k_mov},
            {"v_lshl_add_u64", k_lshladd64}};
  for (int wps : {2, 4, 8}) {  // waves per SIMD: wps/4 1024-thread WGs per CU (or one WG of 256*wps)
  printf("--- %d waves per SIMD\n", wps);
  const dim3 grid(wps <= 4 ? cus : cus * (wps / 4)), block(wps <= 4 ? 256 * wps : 1024);
  double base = 0;
  for (auto& k : ks) {
    if (!k.fn) continue;
    hipLaunchKernelGGL(k.fn, grid, block, 0, 0, out, iters);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k.fn, grid, block, 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = (double)wps * 16 * iters;  // waves x 16 instr x iters
    const double ns = ms * 1e6 / per_simd;
    if (base == 0) base = ns;
    printf("%-18s %.3f ns/instr/SIMD  (%.2fx v_add_u32; %.2f cyc @2.4GHz)\n", k.name, ns, ns / base, ns * 2.4);
  }
  }
  return 0;
}
