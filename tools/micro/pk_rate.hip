// Issue rate of packed vs scalar f32 adds on gfx950 (one-off microbenchmark, round 5):
//   hipcc --offload-arch=gfx950 -O3 -o pk_rate pk_rate.hip && ./pk_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

__global__ void __launch_bounds__(256) scalar_add(float* out, float s) {
  float a[16];
  for (int j = 0; j < 16; j++) a[j] = threadIdx.x * 0.5f + j;
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int j = 0; j < 16; j++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
  }
  float r = 0;
  for (int j = 0; j < 16; j++) r += a[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) packed_add(float* out, float s) {
  f2 a[8];
  const f2 sv = {s, s};
  for (int j = 0; j < 8; j++) a[j] = f2{threadIdx.x * 0.5f + 2 * j, threadIdx.x * 0.5f + 2 * j + 1};
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(sv));
  }
  float r = 0;
  for (int j = 0; j < 8; j++) r += a[j].x + a[j].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) packed_fma(float* out, float s) {
  f2 a[8];
  const f2 sv = {s, s};
  for (int j = 0; j < 8; j++) a[j] = f2{threadIdx.x * 0.5f + 2 * j, threadIdx.x * 0.5f + 2 * j + 1};
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(sv));
  }
  float r = 0;
  for (int j = 0; j < 8; j++) r += a[j].x + a[j].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 1024 * 64 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8 * 4;  // 8 waves per SIMD
  for (int rep = 0; rep < 2; rep++) {
    for (int k = 0; k < 3; k++) {
      hipEventRecord(e0);
      if (k == 0) scalar_add<<<blocks, 256>>>(out, 1e-7f);
      if (k == 1) packed_add<<<blocks, 256>>>(out, 1e-7f);
      if (k == 2) packed_fma<<<blocks, 256>>>(out, 1e-7f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double lane_adds = (double)blocks * 256 * kIters * 16;  // f32 adds (or fmas) per launch
      std::printf("%s: %.3f ms, %.1f T f32 lane-ops/s\n", k == 0 ? "v_add_f32 " : (k == 1 ? "v_pk_add_f32" : "v_pk_fma_f32"), ms,
                  lane_adds / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
