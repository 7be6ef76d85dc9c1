// Issue cost of single VALU instructions on gfx950: each kernel runs 8 independent chains of one
// instruction in a loop on a full grid; reports SIMD cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(ins)                                                                                   \
  asm volatile(ins ins ins ins ins ins ins ins : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4),  \
               "+v"(a5), "+v"(a6), "+v"(a7)::);

constexpr int kIters = 4096;

#define KERNEL(name, body)                                                  \
  __global__ __launch_bounds__(256) void name(unsigned* out, unsigned s) {  \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;       \
    unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;            \
    for (int i = 0; i < kIters; i++) {                                      \
      body                                                                  \
    }                                                                       \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
  }

// 8 instructions per body (one per chain)
#define ONE(op) \
  op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)

KERNEL(k_xor, asm volatile("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_fma, asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_mullo, asm volatile("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_mulhi, asm volatile("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_mul24, asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_rcp, asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_sqrt, asm volatile("v_sqrt_f32 %0, %0\n v_sqrt_f32 %1, %1\n v_sqrt_f32 %2, %2\n v_sqrt_f32 %3, %3\n v_sqrt_f32 %4, %4\n v_sqrt_f32 %5, %5\n v_sqrt_f32 %6, %6\n v_sqrt_f32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
KERNEL(k_cndmask, asm volatile("v_cmp_gt_u32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %0, vcc\n v_cndmask_b32 %2, %2, %0, vcc\n v_cndmask_b32 %3, %3, %0, vcc\n v_cndmask_b32 %4, %4, %0, vcc\n v_cndmask_b32 %5, %5, %0, vcc\n v_cndmask_b32 %6, %6, %0, vcc\n v_cndmask_b32 %7, %7, %0, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");)
KERNEL(k_readlane, asm volatile("v_readlane_b32 s0, %0, 3\n v_readlane_b32 s1, %1, 5\n v_readlane_b32 s2, %2, 3\n v_readlane_b32 s3, %3, 3\n v_readlane_b32 s4, %4, 3\n v_readlane_b32 s5, %5, 3\n v_readlane_b32 s6, %6, 3\n v_readlane_b32 s7, %7, 3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "s0","s1","s2","s3","s4","s5","s6","s7");)
KERNEL(k_salu, asm volatile("s_xor_b32 s0, s0, %8\n s_xor_b32 s1, s1, %8\n s_xor_b32 s2, s2, %8\n s_xor_b32 s3, s3, %8\n s_xor_b32 s4, s4, %8\n s_xor_b32 s5, s5, %8\n s_xor_b32 s6, s6, %8\n s_xor_b32 s7, s7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "s0","s1","s2","s3","s4","s5","s6","s7");)

__global__ __launch_bounds__(256) void k_mad64(unsigned* out, unsigned s) {
  unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
                     a7 = a0 + 7;
  unsigned b = threadIdx.x * 7u + 1u;
  for (int i = 0; i < kIters; i++) {
    asm volatile(
        "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %9, %1\n v_mad_u64_u32 %2, vcc, %8, %9, %2\n"
        " v_mad_u64_u32 %3, vcc, %8, %9, %3\n v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %9, %5\n"
        " v_mad_u64_u32 %6, vcc, %8, %9, %6\n v_mad_u64_u32 %7, vcc, %8, %9, %7"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "s"(s), "v"(b)
        : "vcc");
  }
  out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

typedef void (*Fn)(unsigned*, unsigned);

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  int cus = prop.multiProcessorCount;
  double clk_ghz = prop.clockRate / 1e6;
  int blocks = cus * 8;  // 8 blocks x 4 waves = 8 waves per SIMD
  unsigned* out;
  (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
  struct {
    const char* n;
    Fn f;
  } ks[] = {{"v_xor_b32", k_xor},         {"v_fma_f32", k_fma},   {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
            {"v_mul_u32_u24", k_mul24},   {"v_rcp_f32", k_rcp},   {"v_sqrt_f32", k_sqrt},    {"v_cndmask_b32", k_cndmask},
            {"v_readlane_b32", k_readlane}, {"s_xor_b32", k_salu}, {"v_mad_u64_u32", k_mad64}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("CUs %d clock %.3f GHz (prop)\n", cus, clk_ghz);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double waves_per_simd = blocks * 4.0 / (cus * 4.0);
    double ins_per_simd = 5.0 * waves_per_simd * kIters * 8;
    double cycles = ms * 1e-3 * clk_ghz * 1e9;
    printf("%-16s %.3f ms  %.2f cycles per wave-instruction (at %.2f GHz)\n", k.n, ms, cycles / ins_per_simd, clk_ghz);
  }
  return 0;
}
