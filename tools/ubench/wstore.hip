// Calibration of rocprofv3 WRITE_SIZE for the store shapes the render kernel's sample buffer can
// use (MI355X_MICROARCH.md: only 16-B-per-lane streaming stores are calibrated). Each kernel writes
// exactly kBytes; run under `rocprofv3 --pmc WRITE_SIZE` and divide.
//   hipcc --offload-arch=gfx950 -O3 -o wstore wstore.hip && ./wstore
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr unsigned kN = 1u << 24;               // samples (16.7 M)
constexpr size_t kBytes = size_t(kN) * 12;      // 12 B per sample: 201 MB

// 12 B per lane, lanes contiguous (one frame plane, every lane at once)
__global__ void plane12(float* out) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  out[3 * i] = (float)i;
  out[3 * i + 1] = 1.0f;
  out[3 * i + 2] = 2.0f;
}

// 96 B per lane (8 samples), lanes' blocks contiguous: six 16-B stores per lane
__global__ void octet96(float* out) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;  // kN / 8 lanes
  float4* b = reinterpret_cast<float4*>(out + 24ull * i);
#pragma unroll
  for (int k = 0; k < 6; k++) b[k] = make_float4((float)i, (float)k, 1.0f, 2.0f);
}

// 12 B per lane into frame planes, but a line's samples written by different waves far apart in
// time: sample s goes to pixel (s % kW) * kSpread + s / kW of a plane (each 128-B line of 10.7
// samples gets them from kSpread-separated lanes)
constexpr unsigned kSpread = 4096;
__global__ void spread12(float* out) {
  const unsigned s = blockIdx.x * 256u + threadIdx.x;
  const unsigned w = kN / kSpread;
  const unsigned p = (s % w) * kSpread + s / w;
  out[3 * p] = (float)s;
  out[3 * p + 1] = 1.0f;
  out[3 * p + 2] = 2.0f;
}

// 96-B lane blocks written one 12-B sample at a time, 8 passes in time order (lane-contiguous
// octets filled slot by slot, as direct stores without LDS staging would)
__global__ void octet_slots(float* out, int slot) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  float* b = out + 24ull * i + 3 * slot;
  b[0] = (float)i;
  b[1] = 1.0f;
  b[2] = 2.0f;
}

int main() {
  float* d;
  if (hipMalloc(&d, kBytes + 4096) != hipSuccess) return 1;
  hipMemset(d, 0, kBytes);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 2; rep++) {
    plane12<<<kN / 256, 256>>>(d);
    octet96<<<kN / 8 / 256, 256>>>(d);
    spread12<<<kN / 256, 256>>>(d);
    for (int s = 0; s < 8; s++) octet_slots<<<kN / 8 / 256, 256>>>(d, s);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"bytes_per_kernel\": %zu, \"octet_slot_bytes\": %zu}\n", kBytes, kBytes / 8);
  hipFree(d);
  return 0;
}
