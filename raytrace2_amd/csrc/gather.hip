// gather.hip — root side of the multi-GPU image gather.
//
// Every GPU renders the interleaved row bands of its rank (rt2_layout.h BandRank) into a compact
// band stack; the stacks, padded to the same height, arrive on the root one after another
// ([world][max_rows][W] float3, by ncclGather or device-local copies). This kernel writes them
// back to image order and derives Pixels() = ToColor(clamp(accum / frame_idx, 0, 1))
// (RayTracer.cpp:16-18,65-66) with the same operations as accumulate_kernel, so the gathered image
// is bit-identical to a one-GPU render.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt2_layout.h"

namespace rt2 {
namespace dev {

// glm's scalar min/max (func_common.inl): max(x, y) = x < y ? y : x, min(x, y) = y < x ? y : x
__device__ __forceinline__ float gmax1(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float gmin1(float x, float y) { return y < x ? y : x; }

// One thread per image pixel: coalesced reads of one band-stack row, coalesced writes of one image row.
__global__ __launch_bounds__(256) void deinterleave_kernel(const float* __restrict__ stacks, float* __restrict__ image,
                                                           float* __restrict__ image_nc,
                                                           uint32_t* __restrict__ pixels, uint32_t width,
                                                           uint32_t npix, uint32_t band_h, uint32_t world,
                                                           uint32_t max_rows, int frame_idx) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= npix) return;
  const uint32_t y = i / width, x = i - y * width;
  const BandRow src = BandSource((int)y, (int)band_h, (int)world);  // rt2_layout.h
  const float* s = stacks + 3ull * (((unsigned long long)src.rank * max_rows + (uint32_t)src.row) * width + x);
  const float a0 = s[0], a1 = s[1], a2 = s[2];
  image[3ull * i] = a0;
  image[3ull * i + 1] = a1;
  image[3ull * i + 2] = a2;
  // NonConvertedPixels() (RayTracer.cpp:108-109): accumulation / frame_idx_ in float
  const float fi = (float)frame_idx;
  const float cc[3] = {a0 / fi, a1 / fi, a2 / fi};
  image_nc[3ull * i] = cc[0];
  image_nc[3ull * i + 1] = cc[1];
  image_nc[3ull * i + 2] = cc[2];
  uint32_t rgba = 0u;  // Reset() state: nothing rendered yet
  if (frame_idx > 0) {
    rgba = 0xFF000000u;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float v = gmin1(gmax1(cc[k], 0.0f), 1.0f);
      rgba |= ((uint32_t)(uint8_t)floor((double)v * 255.999)) << (8 * k);
    }
  }
  pixels[i] = rgba;
}

}  // namespace dev

hipError_t LaunchDeinterleave(const float* stacks, float* image, float* image_nc, uint8_t* pixels, int width,
                              int height, int band_h, int world, int max_rows, int frame_idx, hipStream_t stream) {
  const uint32_t npix = (uint32_t)width * (uint32_t)height;
  if (npix == 0) return hipSuccess;
  hipLaunchKernelGGL(dev::deinterleave_kernel, dim3((npix + 255u) / 256u), dim3(256), 0, stream, stacks, image,
                     image_nc, reinterpret_cast<uint32_t*>(pixels), (uint32_t)width, npix, (uint32_t)band_h, (uint32_t)world,
                     (uint32_t)max_rows, frame_idx);
  return hipGetLastError();
}

}  // namespace rt2
