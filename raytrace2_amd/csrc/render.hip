// render.hip — the hot path: RayTracer::Update (RayTracer.cpp:55-70) → Camera::GetRay
// (Camera.hpp:50-67) → RayColor (RayTracer.cpp:20-45) → closest-hit traversal (BVH.cpp:50-55,
// HittableList.cpp:8-22, Quad.cpp:19-43, Sphere.cpp:7-37, Transform.cpp:75-88,
// ConstantMedium.cpp:14-58) → Scatter/Emit (Material.cpp:10-83, Texture.cpp:7-22,
// PerlinNoiseGen.cpp:54-88), as one persistent gfx950 kernel.
//
// Execution model (MI355X):
//  * persistent lanes take work items = (pixel, chunk of consecutive frames of the launch); a lane
//    renders its chunk's frames back to back and writes each frame's sample (float3) to the
//    sample buffer (octets: a pixel's 8 consecutive frames are 96 contiguous bytes, rt2_layout.h);
//    accumulate_kernel then adds a launch's samples to the accumulation in frame order, so the
//    float sum is the reference's `accumulation_data_[i] += c` sequence (RayTracer.cpp:64)
//    whatever the chunking;
//  * one loop iteration = one bounce for every live lane; a lane whose path ends starts its next
//    frame in the same iteration (path regeneration), so lanes never idle inside a wave until
//    their chunk is done;
//  * items are numbered chunk-major over 8x8 pixel tiles and handed out by a wave-aggregated
//    atomic: __ballot of the lanes that need work, one atomicAdd per wave batch (guided sizes), a
//    popcount prefix for each lane's slot;
//  * small scenes run a threaded (stackless) pre-order program walked in lockstep by the wave, so
//    step kinds are wave-uniform and records come through scalar loads; larger ones use a stack
//    traversal with the stack in LDS (lane-major columns: a wave's push/pop is one conflict-free
//    ds_write/ds_read) and the scene, or the top of its BVH, staged in LDS beside it;
//  * traversal carries only (t, primitive ref, transform ref) of the closest hit; the hit point,
//    normal and material are computed once for the winning primitive (bit-identical to computing
//    them at every candidate hit, as the reference does);
//  * the kernel is instantiated per scene feature set (rt2_layout.h Feature), so code for absent
//    primitive / material / texture kinds costs no registers in the variant that runs.
//
// Numerics: compiled with -ffp-contract=off; fp32 division and sqrt are correctly rounded (HIP
// default). Every expression repeats the reference's operation order, so results match the
// CPU restatement bit for bit except the radiance product, which is accumulated front to back
// (thr *= att) instead of the reference's recursion order (att0*(att1*(...*E))).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "rt2_layout.h"
#define RT2_BOXAA_FN __device__ __forceinline__
#include "boxaa.h"

namespace rt2 {
namespace dev {

constexpr int kBlock = 256;

// Diagnostic builds (tools/: cost probes, wave-step counts, section times, launch-tail times); all
// default off. The product kernel is the build with none of them.
#ifndef RT2_EXP_TRACE_TWICE
#define RT2_EXP_TRACE_TWICE 0  // cost probe: every ray is traced a second time (result discarded)
#endif
#ifndef RT2_EXP_TWICE
#define RT2_EXP_TWICE 0  // cost probes (bits): 1 resolve_hit, 2 rand_unit_vec3, 4 camera_ray, 8 slab test,
                         // 16 quad-run test, 32 threaded medium step, 64 its log, 128 its two boundary
                         // queries, 256 a Philox block (at every refill), 512 the sample store /
                         // staging, 2048 a threaded transform entry (ray into model space, its reciprocal),
                         // 4096 an accelerated list's lane walk, 8192 the box-level test of a MakeBox run
#endif
#ifndef RT2_EXP_WAVESTEPS
#define RT2_EXP_WAVESTEPS 0  // diagnostic build: per-wave linear-traversal step counts into diag slots
#endif
#ifndef RT2_EXP_STAMPS
#define RT2_EXP_STAMPS 0  // diagnostic build: per-section s_memtime sums into the stamp slots
#endif
#ifndef RT2_EXP_ENDTIME
#define RT2_EXP_ENDTIME 0  // diagnostic build: per-wave start / first-idle / end times (s_memrealtime) into diag
#endif
// Occupancy targets (waves per SIMD) per kernel variant; overridable for sweeps (tools/build_variants.sh).
#ifndef RT2_MIN_WAVES_CORNELL
#define RT2_MIN_WAVES_CORNELL 8
#endif
#ifndef RT2_MIN_WAVES_BOOK1
#define RT2_MIN_WAVES_BOOK1 8
#endif
#ifndef RT2_MIN_WAVES_VOL
#define RT2_MIN_WAVES_VOL 8  // round 3, with box boundaries as one block: 7 / 8 waves 19.9 k / 20.6 k Mray/s
#endif
#ifndef RT2_MIN_WAVES_B2LIN
#define RT2_MIN_WAVES_B2LIN 8  // book 2 threaded (2000 spp): 6/7/8 waves 1685/1788/1887 Mray/s since its tree steps run in
                               // the BVH-step loop (round 1, before: 3/4/5/6/7/8 waves 934/938/1091/1183/1297/508)
#endif
#ifndef RT2_MIN_WAVES_ALL
#define RT2_MIN_WAVES_ALL 6
#endif
#ifndef RT2_MIN_WAVES_PER_EU
#define RT2_MIN_WAVES_PER_EU 0  // 0: per-variant occupancy targets (kMinWaves below)
#endif

extern __shared__ float4 s_dyn[];  // [lds_nodes scene records][stack_depth * kBlock stack words]

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) {
  float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
  return (px + py) + pz;
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
// IEEE-exact 1/x and sqrt(x) without the range-scaling steps of the full sequences: equal to them
// (v_div_scale / v_div_fixup and the sqrt rescale are identities there) for 2^-95 <= |x| <= 2^126
// (reciprocal) and 2^-96 <= x <= 2^126 (sqrt); callers check the range wave-uniformly and take
// the full sequence otherwise. rt2_selftest which 2 checks both on the GPU.
// rcp_nr: the hardware reciprocal and two Newton steps, each as fma(fma(-x, r, 1), r, r); equal to
// IEEE 1/x for every float in its range (rt2_selftest which 5 checks all 3.7e9 of them; a third
// step, used before round 4, changes nothing)
__device__ __forceinline__ float rcp_nr(float x) {
  const float r0 = __builtin_amdgcn_rcpf(x);
  const float r1 = fmaf(fmaf(-x, r0, 1.0f), r0, r0);
  return fmaf(fmaf(-x, r1, 1.0f), r1, r1);
}
__device__ __forceinline__ float sqrt_nr(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
  const float rdn = fmaf(-sdn, s, x), rup = fmaf(-sup, s, x);
  const float r = rdn <= 0.0f ? sdn : s;
  return rup > 0.0f ? sup : r;
}
__device__ __forceinline__ bool rcp_in_range(float x) { return fabsf(x) >= 0x1p-95f && fabsf(x) <= 0x1p126f; }
// glm::normalize = v * inversesqrt(dot(v, v)) = v * (1 / sqrt(dot(v, v)))
__device__ __forceinline__ f3 normalize(f3 v) {
  const float l2 = dot(v, v);
  if (__all(l2 >= 0x1p-96f && l2 <= 0x1p126f)) return v * rcp_nr(sqrt_nr(l2));
  return v * (1.0f / sqrtf(l2));
}
// (1/d.x, 1/d.y, 1/d.z), IEEE
__device__ __forceinline__ f3 recip3(f3 d) {
  if (__all(rcp_in_range(d.x) && rcp_in_range(d.y) && rcp_in_range(d.z)))
    return mk(rcp_nr(d.x), rcp_nr(d.y), rcp_nr(d.z));
  return mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
}
// d = normalize(v), inv = (1/d.x, 1/d.y, 1/d.z) (IEEE) and whether inv is finite. When the whole wave
// takes normalize's fast path (dot(v, v) in [2^-96, 2^126]), every component of d is a NaN or has
// |x| <= 1 + 2^-21, so only the lower end of rcp_nr's range needs a check (a NaN fails it) and the
// reciprocal is finite by construction (|1 / x| <= 2^95). normalize's slow path can give components of
// any size (+-inf for a v so short that dot(v, v) underflows), and there the reciprocal is
// IEEE division.
__device__ __forceinline__ void normalize_recip3(f3 v, f3& d, f3& inv, bool& fin) {
  const float l2 = dot(v, v);
  if (__all(l2 >= 0x1p-96f && l2 <= 0x1p126f)) {
    d = v * rcp_nr(sqrt_nr(l2));
    if (__all(fabsf(d.x) >= 0x1p-95f && fabsf(d.y) >= 0x1p-95f && fabsf(d.z) >= 0x1p-95f)) {
      inv = mk(rcp_nr(d.x), rcp_nr(d.y), rcp_nr(d.z));
      fin = true;
      return;
    }
  } else {
    d = v * (1.0f / sqrtf(l2));
  }
  inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  fin = __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z);
}
__device__ __forceinline__ f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }
// floor(n / d) for n < 2^31 by the host's multiplier (rt2_layout.h Magic): v_mad_u64_u32 + shift
__device__ __forceinline__ uint32_t udiv(uint32_t n, Magic d) { return (uint32_t)(((uint64_t)n * d.m) >> d.s); }
__device__ __forceinline__ uint32_t bits(float f) { return __float_as_uint(f); }
// glm scalar max/min
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }
__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }

template <uint32_t F, uint32_t B>
constexpr bool Has() {
  return (F & B) != 0;
}

// Scene-record source: the LDS copy (kModeStackLds) or global memory. Loads go through a
// __restrict__ parameter so wave-uniform indices (linear mode) become scalar loads.
__device__ __forceinline__ float4 ldg4(const float4* __restrict__ p, uint32_t i) { return p[i]; }
__device__ __forceinline__ uint32_t ldg1(const uint32_t* __restrict__ p, uint32_t i) { return p[i]; }

template <int kMode>
struct Nodes {
  const float4* g;
  uint32_t lds_n;  // kModeStackHybrid: records [0, lds_n) are in LDS
  __device__ __forceinline__ float4 operator[](uint32_t i) const {
    if constexpr (kMode == kModeStackLds) {
      return s_dyn[i];
    } else if constexpr (kMode == kModeStackHybrid) {
      return i < lds_n ? s_dyn[i] : ldg4(g, i);
    } else {
      return ldg4(g, i);
    }
  }
  __device__ __forceinline__ uint32_t word(uint32_t rec, uint32_t k) const {  // 32-bit word k after record rec
    if constexpr (kMode == kModeStackLds) {
      return bits(reinterpret_cast<const float*>(s_dyn + rec)[k]);
    } else if constexpr (kMode == kModeStackHybrid) {
      // k may run past record rec (list children, the leaf-list cursor's word(0, k)): the record
      // that holds the word decides where it lives
      const uint32_t w = 4u * rec + k;
      return (w >> 2) < lds_n ? bits(reinterpret_cast<const float*>(s_dyn)[w])
                              : ldg1(reinterpret_cast<const uint32_t*>(g), w);
    } else {
      return ldg1(reinterpret_cast<const uint32_t*>(g + rec), k);
    }
  }
};

// Scalar (SMEM) loads of wave-uniform data: the linear traversal's program entries and records
// land in SGPRs. Inline asm because the compiler will not prove these loads unclobbered (the
// kernel stores the accumulation buffer inside the same loop). Base and byte offset must be
// wave-uniform; each helper waits for its own loads. Helpers issuing several loads mark their
// outputs early-clobber: a later load's base/offset must not share registers with an earlier
// load's destination (its data can land before the later load reads its operands).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
// (offsets are wave-uniform by construction; readfirstlane keeps them in SGPRs even where the
// compiler could not prove it, and costs nothing where it could)
__device__ __forceinline__ uint32_t sld1(const void* base, uint32_t off) {
  off = __builtin_amdgcn_readfirstlane(off);
  uint32_t v;
  asm("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(base), "s"(off));
  return v;
}
__device__ __forceinline__ u32x8 sld8(const void* base, uint32_t off) {
  off = __builtin_amdgcn_readfirstlane(off);
  u32x8 v;
  asm("s_load_dwordx8 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(base), "s"(off));
  return v;
}
__device__ __forceinline__ u32x16 sld16(const void* base, uint32_t off) {
  off = __builtin_amdgcn_readfirstlane(off);
  u32x16 v;
  asm("s_load_dwordx16 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(base), "s"(off));
  return v;
}
// 20 dwords (one quad record) at off
__device__ __forceinline__ void sld20(const void* base, uint32_t off, u32x16& a, u32x4& b) {
  off = __builtin_amdgcn_readfirstlane(off);
  asm("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx4 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
      : "=&s"(a), "=&s"(b)
      : "s"(base), "s"(off), "s"(off + 64u));
}
__device__ __forceinline__ float uf(uint32_t u) { return __uint_as_float(u); }

// Launch parameters re-read from the kernel-argument segment where they are used (one scalar load)
// instead of being held in SGPRs across the render loop: the loop keeps more wave-uniform values
// live than there are SGPRs, and the compiler's spill of them to VGPR lanes costs one v_readlane (a
// VALU instruction) per value at every use. Volatile, so the load is not hoisted back out of the
// loop. The kernel's only argument is its RenderParams, at offset 0 of the segment.
template <uint32_t kOff>
__device__ __forceinline__ u32x16 karg16() {
  static_assert(kOff % 4 == 0, "dword-aligned");
  u32x16 v;
  asm volatile("s_load_dwordx16 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(v)
               : "s"(__builtin_amdgcn_kernarg_segment_ptr()), "n"(kOff));
  return v;
}
template <uint32_t kOff>
__device__ __forceinline__ u32x8 karg8() {
  static_assert(kOff % 4 == 0, "dword-aligned");
  u32x8 v;
  asm volatile("s_load_dwordx8 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(v)
               : "s"(__builtin_amdgcn_kernarg_segment_ptr()), "n"(kOff));
  return v;
}
template <uint32_t kOff>
__device__ __forceinline__ u32x4 karg4() {
  static_assert(kOff % 4 == 0, "dword-aligned");
  u32x4 v;
  asm volatile("s_load_dwordx4 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(v)
               : "s"(__builtin_amdgcn_kernarg_segment_ptr()), "n"(kOff));
  return v;
}
template <uint32_t kOff>
__device__ __forceinline__ unsigned long long karg2() {
  static_assert(kOff % 4 == 0, "dword-aligned");
  unsigned long long v;
  asm volatile("s_load_dwordx2 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(v)
               : "s"(__builtin_amdgcn_kernarg_segment_ptr()), "n"(kOff));
  return v;
}

#define RT2_KOFF(f) ((uint32_t)offsetof(RenderParams, f))
template <typename T, int k>
__device__ __forceinline__ T kword(const u32x16& v) {  // a 4- or 8-byte field of a loaded block
  static_assert(k >= 0 && k + (int)sizeof(T) / 4 <= 16, "field outside the block");
  // (the element is copied out first: __builtin_bit_cast of a vector-element lvalue reads element 0
  // with this compiler)
  if constexpr (sizeof(T) == 4) {
    const uint32_t x = v[k];
    return __builtin_bit_cast(T, x);
  } else {
    static_assert(sizeof(T) == 8, "field size");
    const unsigned long long x = (unsigned long long)v[k] | ((unsigned long long)v[k + 1] << 32);
    return __builtin_bit_cast(T, x);
  }
}

// The render loop's launch constants (image, partition, work items, chunk table, magic divisors,
// seed, sample buffer): two 64-byte blocks and the width, one wait.
struct LoopArgs {
  static constexpr uint32_t kA = 144, kB = 212;  // [144, 208) height .. chunks, [212, 276) div_tile_items .. local_pixels
  static_assert(RT2_KOFF(height) == kA && RT2_KOFF(chunks) + 8 == kA + 64 && RT2_KOFF(div_tile_items) == kB &&
                    RT2_KOFF(local_pixels) + 4 == kB + 64 &&
                    RT2_KOFF(width) == kA - 4,
                "RenderParams layout");
  u32x16 a, b;
  uint32_t w;
  template <typename T, uint32_t kOff>
  __device__ __forceinline__ T get() const {
    if constexpr (kOff < kB) {
      return kword<T, (int)(kOff - kA) / 4>(a);
    } else {
      return kword<T, (int)(kOff - kB) / 4>(b);
    }
  }
#define RT2_LA(name, T, f) \
  __device__ __forceinline__ T name() const { return get<T, RT2_KOFF(f)>(); }
  RT2_LA(local_rows, int, local_rows)
  RT2_LA(band_h, int, band_h)
  RT2_LA(rank, int, rank)
  RT2_LA(world, int, world)
  RT2_LA(tile_shift, uint32_t, tile_shift)
  RT2_LA(tiles_x, int, tiles_x)
  RT2_LA(tile_items, uint32_t, tile_items)
  RT2_LA(n_items, uint32_t, n_items)
  RT2_LA(batch_max, uint32_t, batch_max)
  RT2_LA(batch_div, uint32_t, batch_div)
  RT2_LA(frame_begin, int, frame_begin)
  RT2_LA(n_frames, int, n_frames)
  RT2_LA(max_depth, int, max_depth)
  RT2_LA(chunks, const uint32_t*, chunks)
  RT2_LA(div_tile_items, Magic, div_tile_items)
  RT2_LA(div_tiles_x, Magic, div_tiles_x)
  RT2_LA(div_band_h, Magic, div_band_h)
  RT2_LA(div_band_w, Magic, div_band_w)
  RT2_LA(div_world, Magic, div_world)
  RT2_LA(samples, float*, samples)
  RT2_LA(local_pixels, uint32_t, local_pixels)
#undef RT2_LA
  __device__ __forceinline__ int width() const { return (int)w; }
};
__device__ __forceinline__ LoopArgs loop_args() {
  LoopArgs r;
  asm volatile(
      "s_load_dwordx16 %0, %3, %4\n\ts_load_dwordx16 %1, %3, %5\n\ts_load_dword %2, %3, %6\n\ts_waitcnt lgkmcnt(0)"
      : "=&s"(r.a), "=&s"(r.b), "=&s"(r.w)
      : "s"(__builtin_amdgcn_kernarg_segment_ptr()), "n"(LoopArgs::kA), "n"(LoopArgs::kB), "n"(LoopArgs::kA - 4));
  return r;
}

// Scene tables used by shading: materials, textures, Perlin vectors and permutations (one load).
struct ShadeArgs {
  const float4* materials;
  const float4* textures;
  const float4* perlin_vec;
  const int* perlin_perm;
};
__device__ __forceinline__ ShadeArgs shade_args() {
  static_assert(RT2_KOFF(materials) == 8 && RT2_KOFF(perlin_perm) == 32, "RenderParams layout");
  const u32x8 v = karg8<8>();
  auto ptr = [&](int k) { return (unsigned long long)v[k] | ((unsigned long long)v[k + 1] << 32); };
  return ShadeArgs{reinterpret_cast<const float4*>(ptr(0)), reinterpret_cast<const float4*>(ptr(2)),
                   reinterpret_cast<const float4*>(ptr(4)), reinterpret_cast<const int*>(ptr(6))};
}


// Philox keys, one scalar load.
__device__ __forceinline__ void seed_args(uint32_t& k0, uint32_t& k1) {
  static_assert(RT2_KOFF(seed_hi) == RT2_KOFF(seed_lo) + 4, "RenderParams layout");
  const unsigned long long k = karg2<RT2_KOFF(seed_lo)>();
  k0 = (uint32_t)k;
  k1 = (uint32_t)(k >> 32);
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 path stream keyed by (seed, pixel, frame). Draws are taken in groups of K <= 4
// consecutive values; `n` counts draws and the buffer holds the block of the last value drawn
// ((n - 1) >> 2), so a group needs at most ONE Philox call (one refill site per call site instead
// of one per value: under divergence every refill site executes for the whole wave).
__device__ __forceinline__ void philox(uint32_t k0, uint32_t k1, uint32_t pixel, uint32_t frame, uint32_t block,
                                       uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t& r3) {
  uint32_t c0 = pixel, c1 = frame, c2 = block, c3 = 0x52543250u;
  // The keys are wave-uniform: opaque here so the 20 round keys are recomputed with SALU adds at
  // each call instead of being hoisted out of the render loop (and spilled to VGPR lanes).
  uint32_t key0 = k0, key1 = k1;
  asm volatile("" : "+s"(key0), "+s"(key1));
  const uint32_t m0 = 0xD2511F53u, m1 = 0xCD9E8D57u;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    // one v_mad_u64_u32 gives both halves of each 32x32 product; xor3 is one v_bitop3_b32
    uint64_t p0, p1;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p0) : "s"(m0), "v"(c0) : "vcc");
    asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p1) : "s"(m1), "v"(c2) : "vcc");
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(c0) : "v"(hi1), "v"(c1), "s"(key0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(c2) : "v"(hi0), "v"(c3), "s"(key1));
    c1 = lo1;
    c3 = lo0;
    key0 += 0x9E3779B9u;
    key1 += 0xBB67AE85u;
  }
  r0 = c0;
  r1 = c1;
  r2 = c2;
  r3 = c3;
}

// philox() with the path streams' round keys from the launch parameters (RenderParams::philox_keys,
// two scalar loads): the same rounds and values, no scalar adds (kRK; Cornell +0.5 %, volume +0.7 %;
// the sphere kernels keep the adds: the 20 key SGPRs cost book 1 SGPR spills, -0.4 %).
template <bool kRK>
__device__ __forceinline__ void philox_path(uint32_t pixel, uint32_t frame, uint32_t block, uint32_t& r0,
                                            uint32_t& r1, uint32_t& r2, uint32_t& r3) {
  if constexpr (!kRK) {
    uint32_t key0, key1;
    seed_args(key0, key1);
    philox(key0, key1, pixel, frame, block, r0, r1, r2, r3);
    return;
  }
  static_assert(RT2_KOFF(philox_keys) % 4 == 0, "RenderParams layout");
  const u32x16 ka = karg16<RT2_KOFF(philox_keys)>();
  const u32x4 kb = karg4<RT2_KOFF(philox_keys) + 64u>();
  uint32_t c0 = pixel, c1 = frame, c2 = block, c3 = 0x52543250u;
  const uint32_t m0 = 0xD2511F53u, m1 = 0xCD9E8D57u;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t key0 = r < 8 ? ka[2 * r] : kb[2 * r - 16], key1 = r < 8 ? ka[2 * r + 1] : kb[2 * r - 15];
    uint64_t p0, p1;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p0) : "s"(m0), "v"(c0) : "vcc");
    asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p1) : "s"(m1), "v"(c2) : "vcc");
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(c0) : "v"(hi1), "v"(c1), "s"(key0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(c2) : "v"(hi0), "v"(c3), "s"(key1));
    c1 = lo1;
    c3 = lo0;
  }
  r0 = c0;
  r1 = c1;
  r2 = c2;
  r3 = c3;
}

__device__ __forceinline__ uint32_t sel4(uint32_t i, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3) {
  return i == 0u ? r0 : (i == 1u ? r1 : (i == 2u ? r2 : r3));
}
__device__ __forceinline__ float to_unit(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// Per-lane LDS planes: word k of a lane at p[64 k] (p = the wave's plane block + the lane id), so a
// wave's access to one plane is one conflict-free ds_read / ds_write. The render kernel gives every
// wave one block of planes (render_kernel: Philox block, sample staging, box-boundary candidates,
// parked path state) and keeps one per-lane address for all of them: the planes differ by
// immediate offsets.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) float lds_f32;

// The per-lane path context the samplers need. kLdsRng: the lane's current Philox block lives in
// four LDS planes (word k at rb[64 k]) instead of four VGPRs that stay live across the whole render
// loop. kRing: eight planes hold two consecutive blocks (draw j at rb[64 (j & 7)]), so the next block
// can be computed before the current one is used up: the render loop computes, in ONE place per
// bounce, the block each lane will draw from next (prefetch: a scattering lane's next block, or
// block 0 of the next frame for a lane starting its next path). Without it the wave runs the Philox
// code at every draw site where any lane refills: the scatter site and the camera site of the
// lanes that start a path, both in nearly every bounce (profiles/r04_c2_cost_probes.json). The
// draws are the same values in the same order.
template <bool kLdsRng, bool kRing = false, bool kRK = false>
struct PathT {
  static constexpr bool kLds = kLdsRng;
  uint32_t frame;
  uint32_t pix;  // global pixel index y * width + x (the stream's pixel word)
  uint32_t sij;  // stratum s_i | s_j << 16 of `frame` (RayTracer.cpp:59-60), advanced per frame
  uint32_t n;    // draws taken in this frame; kRing: | (draws loaded and not taken) << 28
  uint32_t r0, r1, r2, r3;  // the block (kLdsRng false)
  lds_u32* rb;              // the lane's Philox planes (kLdsRng true)
  __device__ __forceinline__ void start(uint32_t f) {
    frame = f;
    n = 0;  // buffer holds block -1: the first group refills
  }
  // kRing: the next frame's block 0 is already in the ring (prefetch with restart)
  __device__ __forceinline__ void start_loaded(uint32_t f) {
    frame = f;
    n = 4u << 28;
  }
  __device__ __forceinline__ void block(uint32_t b, uint32_t& w0, uint32_t& w1, uint32_t& w2, uint32_t& w3) const {
    philox_path<kRK>(pix, frame, b, w0, w1, w2, w3);  // keys re-read at the refill (see karg16)
  }
  // kRing: block b of frame f into the ring (half b & 1)
  __device__ __forceinline__ void ring_put(uint32_t f, uint32_t b) {
    uint32_t w0, w1, w2, w3;
    philox_path<kRK>(pix, f, b, w0, w1, w2, w3);
#if RT2_EXP_TWICE & 256
    {
      uint32_t key0, key1;
      seed_args(key0, key1);
      uint32_t q0, q1, q2, q3, fr = f;
      asm volatile("" : "+v"(fr));
      philox(key0, key1, pix, fr, b + 7u, q0, q1, q2, q3);
      asm volatile("" ::"v"(q0), "v"(q1), "v"(q2), "v"(q3));
    }
#endif
    lds_u32* h = rb + 256u * (b & 1u);
    h[0] = w0;
    h[64] = w1;
    h[128] = w2;
    h[192] = w3;
  }
  // kRing: the one refill site of a bounce. scatter: the lane will take up to 2 draws of this frame;
  // restart: the lane's path is done and its next frame starts (block 0 of frame + 1).
  __device__ __forceinline__ void prefetch(bool scatter, bool restart) {
    const uint32_t nn = n & 0x0FFFFFFFu, ah = n >> 28;
    const bool more = scatter && ah < 2u;
    if (more || restart) {
      ring_put(restart ? frame + 1u : frame, restart ? 0u : (nn + ah) >> 2);
      if (more) n += 4u << 28;
    }
  }
  // K consecutive uniforms in [0,1) (24-bit mantissa), in stream order
  template <int K>
  __device__ __forceinline__ void take(float* out) {
    if constexpr (kRing) {
      static_assert(kLdsRng && K <= 4, "ring draws");
      const uint32_t nn = n & 0x0FFFFFFFu;
      uint32_t ah = n >> 28;
      if (ah < (uint32_t)K) {  // not prefetched (a path's first camera ray after a work fetch)
        ring_put(frame, (nn + ah) >> 2);
        ah += 4u;
      }
#pragma unroll
      for (int j = 0; j < K; j++) out[j] = to_unit(rb[64u * ((nn + (uint32_t)j) & 7u)]);
      n = (nn + (uint32_t)K) | ((ah - (uint32_t)K) << 28);
      return;
    }
    uint32_t i = n & 3u;
    bool fresh = i == 0u;
    uint32_t v[K];
    if constexpr (kLdsRng) {
#pragma unroll
      for (int j = 0; j < K; j++) v[j] = rb[64u * ((i + (uint32_t)j) & 3u)];
      if (fresh || i + (uint32_t)K > 4u) {
        uint32_t w0, w1, w2, w3;
        block((n >> 2) + (fresh ? 0u : 1u), w0, w1, w2, w3);
#if RT2_EXP_TWICE & 256
        {
          uint32_t q0, q1, q2, q3, fr = frame;
          asm volatile("" : "+v"(fr));
          uint32_t key0, key1;
          seed_args(key0, key1);
          philox(key0, key1, pix, fr, (n >> 2) + 7u, q0, q1, q2, q3);
          asm volatile("" ::"v"(q0), "v"(q1), "v"(q2), "v"(q3));
        }
#endif
#pragma unroll
        for (int j = 0; j < K; j++)
          if (fresh || i + (uint32_t)j >= 4u) v[j] = sel4((i + (uint32_t)j) & 3u, w0, w1, w2, w3);
        rb[0] = w0;
        rb[64] = w1;
        rb[128] = w2;
        rb[192] = w3;
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; j++) v[j] = sel4((i + (uint32_t)j) & 3u, r0, r1, r2, r3);
      if (fresh || i + (uint32_t)K > 4u) {
        block((n >> 2) + (fresh ? 0u : 1u), r0, r1, r2, r3);
#pragma unroll
        for (int j = 0; j < K; j++)
          if (fresh || i + (uint32_t)j >= 4u) v[j] = sel4((i + (uint32_t)j) & 3u, r0, r1, r2, r3);
      }
    }
    n += (uint32_t)K;
#pragma unroll
    for (int j = 0; j < K; j++) out[j] = to_unit(v[j]);
  }
  __device__ __forceinline__ float uniform() {
    float u[1];
    take<1>(u);
    return u[0];
  }
};

// Path state parked in LDS while a ray is traced (render_kernel kPark): the lane's world ray and
// the path context sit in planes of the wave's park block (word k of the lane at pk[64 k]), so the
// registers that held them are free for the traversal. The only path-state use inside a trace is
// the medium step's free-flight draw: it reads the stream position from the planes and writes the
// advanced count back. Volatile accesses: neither hoisted into registers nor forwarded from the
// stores.
enum ParkWord : uint32_t { kPkThr = 0, kPkDl = 3, kPkSij = 4, kPkFrame = 5, kPkPix = 6, kPkN = 7, kPkO = 8,
                           kPkD = 11, kParkWords = 14 };
__device__ __forceinline__ void pk_st(lds_u32* pk, uint32_t w, uint32_t v) {
  *reinterpret_cast<volatile lds_u32*>(pk + 64u * w) = v;
}
__device__ __forceinline__ uint32_t pk_ld(const lds_u32* pk, uint32_t w) {
  return *reinterpret_cast<const volatile lds_u32*>(pk + 64u * w);
}
__device__ __forceinline__ void pk_st3(lds_u32* pk, uint32_t w, f3 v) {
  pk_st(pk, w, bits(v.x));
  pk_st(pk, w + 1u, bits(v.y));
  pk_st(pk, w + 2u, bits(v.z));
}
__device__ __forceinline__ f3 pk_ld3(const lds_u32* pk, uint32_t w) {
  return mk(uf(pk_ld(pk, w)), uf(pk_ld(pk, w + 1u)), uf(pk_ld(pk, w + 2u)));
}
struct ParkedPath {
  static constexpr bool kLds = true;
  lds_u32* rb;  // the lane's Philox planes (PathT<true>)
  lds_u32* pk;    // this lane's park planes
  template <int K>
  __device__ __forceinline__ void take(float* out) {
    PathT<true> p;
    p.rb = rb;
    p.frame = pk_ld(pk, kPkFrame);
    p.pix = pk_ld(pk, kPkPix);
    p.n = pk_ld(pk, kPkN);
    p.template take<K>(out);
    pk_st(pk, kPkN, p.n);
  }
  __device__ __forceinline__ float uniform() {
    float u[1];
    take<1>(u);
    return u[0];
  }
};
// The world ray a trace starts from: in registers, or (kPark) read back from the park planes at the
// steps that need it again (the exit of a transform, the end of the trace).
struct RegRay {
  f3 o, d;
  __device__ __forceinline__ f3 wo() const { return o; }
  __device__ __forceinline__ f3 wd() const { return d; }
};
struct ParkRay {
  const lds_u32* pk;
  __device__ __forceinline__ f3 wo() const { return pk_ld3(pk, kPkO); }
  __device__ __forceinline__ f3 wd() const { return pk_ld3(pk, kPkD); }
};

// Math.hpp:15 RandReal(min, max) = min + RandReal() * (max - min)
__device__ __forceinline__ float rand_range(float u, float mn, float mx) { return mn + u * (mx - mn); }

// (cos 2 pi v, sin 2 pi v), v in [0, 1): exact quarter-turn split 4v = q + x and polynomials in x;
// the oracle's CosSin2Pi evaluates the same operations in the same order.
__device__ __forceinline__ void cos_sin_2pi(float v, float& c, float& s) {
  const float t = v * 4.0f;
  const int q = (int)t;
  const float x = t - (float)q;
  const float x2 = x * x;
  // Horner steps as fused multiply-adds (one rounding each; the oracle evaluates the same fmas)
  const float sp = fmaf(fmaf(fmaf(fmaf(1.509560242993757e-4f, x2, -4.672547802329063e-3f), x2, 7.968873530626297e-2f), x2,
                             -6.459634304046631e-1f), x2, 1.570796251296997f) * x;
  const float cp = fmaf(fmaf(fmaf(fmaf(8.59465915709734e-4f, x2, -2.0813362672924995e-2f), x2, 2.536526620388031e-1f), x2,
                             -1.2336987257003784f), x2, 1.0f);
  const bool odd = (q & 1) != 0, neg_c = q == 1 || q == 2, neg_s = q >= 2;
  const float cc = odd ? sp : cp, ss = odd ? cp : sp;
  c = neg_c ? -cc : cc;
  s = neg_s ? -ss : ss;
}
// sin(x) in float for the marble texture (Texture.cpp:16, std::sin of a float): x - k pi/2 with
// k = rint(x 2/pi) by a three-part Cody-Waite split in fmas, then the quarter-turn polynomials of r in
// [-pi/4, pi/4] (Horner steps as fmas); within 9e-8 of sin for |x| <= 5000 (the marble's arguments stay
// below a few hundred). |x| >= 2^24 (no fractional part left) gives x - x: 0, or NaN for +-inf and NaN.
// The oracle's SinF evaluates the same operations in the same order. (Round 5 took a double-precision
// sin here, whose hoisted coefficients held 72 of book 2's 92 bytes of register-spill scratch.)
__device__ __forceinline__ float sin_f(float x) {
  if (!(fabsf(x) < 0x1p24f)) return x - x;
  const float k = __builtin_rintf(x * 0.636619772f);
  float r = fmaf(-k, 1.57079637f, x);
  r = fmaf(-k, -4.37113883e-08f, r);
  r = fmaf(-k, -1.71512451e-15f, r);
  const float z = r * r;
  const float s = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
  const float c = fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f), z * z,
                       fmaf(-0.5f, z, 1.0f));
  const int q = (int)(k - 4.0f * floorf(k * 0.25f));  // k mod 4, exact for |k| < 2^25
  const float v = (q & 1) ? c : s;
  return q >= 2 ? -v : v;
}
// ln(u) of a 24-bit uniform (ConstantMedium.cpp:38 std::log(RandReal())): -inf at 0, else
// e ln2 + log1p(f), u = 2^e (1 + f), 1 + f in [sqrt(1/2), sqrt(2)), log1p = f + f^2 Q(f) (degree-8 Q),
// ln2 split so that e ln2_hi is exact; within 0.87 ulp of ln for every uniform. The oracle's LogU
// evaluates the same operations in the same order (about 20 VALU instead of a double-precision log's
// 40 plus its range handling).
__device__ __forceinline__ float log_u(float u) {
  if (u == 0.0f) return -__builtin_inff();
  const uint32_t b = __float_as_uint(u);
  int e = (int)(b >> 23) - 127;
  float m = __uint_as_float((b & 0x007FFFFFu) | 0x3F800000u);
  if (m > 1.41421354f) {
    m = m * 0.5f;
    e += 1;
  }
  const float f = m - 1.0f;
  float q = -0.07477458566427231f;
  q = fmaf(q, f, 0.12822002172470093f);
  q = fmaf(q, f, -0.13261467218399048f);
  q = fmaf(q, f, 0.1419624537229538f);
  q = fmaf(q, f, -0.16608606278896332f);
  q = fmaf(q, f, 0.2000119835138321f);
  q = fmaf(q, f, -0.2500157654285431f);
  q = fmaf(q, f, 0.3333333730697632f);
  q = fmaf(q, f, -0.49999988079071045f);
  const float l1p = fmaf(f * f, q, f);
  const float ef = (float)e;
  return fmaf(ef, 0.693145751953125f, fmaf(ef, 1.42860677e-06f, l1p));
}

// Math.hpp:26-43 RandUnitVec3 (uniform on the unit sphere) by the inverse-CDF map z = 1 - 2u,
// phi = 2 pi v: two uniforms and no rejection loop, so a wave never waits on its unluckiest
// lane's retries (the oracle draws the same map; DESIGN.md "Sampling").
template <class G>
__device__ __forceinline__ f3 rand_unit_vec3(G& g) {
  float u[2];
  g.template take<2>(u);
  const float z = 1.0f - 2.0f * u[0];
  // 1 - z^2 is 0 or >= 2^-22 for every 24-bit uniform, where sqrt_nr is the IEEE square root
  // (rt2_selftest which 9 checks all 2^24 inputs)
  const float r = sqrt_nr(1.0f - z * z);
  float c, s;
  cos_sin_2pi(u[1], c, s);
  return mk(r * c, r * s, z);
}
// NearZero: |x| < 1e-8 (double) <=> |x| <= 1e-8f for floats
__device__ __forceinline__ bool near_zero(f3 v) {
  return fabsf(v.x) <= 1e-8f && fabsf(v.y) <= 1e-8f && fabsf(v.z) <= 1e-8f;
}
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return v - (2.0f * dot(v, n)) * n; }
__device__ __forceinline__ f3 refract(f3 uv, f3 n, float etai_over_etat) {
  float cos_theta = fminf(dot(-uv, n), 1.0f);
  f3 perp = etai_over_etat * (uv + cos_theta * n);
  f3 par = (-sqrtf(fabsf(1.0f - dot(perp, perp)))) * n;
  return perp + par;
}

struct Counters {
  uint32_t bvh, quad, sphere, xform, medium, list;
  uint32_t box, box_cert, box_wave, box_wave_run;  // box-level test (counting kernels)
#if RT2_EXP_WAVESTEPS
  // wave-level (counted by the first active lane): trace calls, steps, bvh + acc-bvh steps, quad
  // runs, sphere + acc-sphere steps, media, extra trips of the min-index search, active lanes at
  // trace (summed by every lane)
  uint32_t wd[8];
#endif
};
#if RT2_EXP_WAVESTEPS
#define RT2_WAVE(k)                                                           \
  do {                                                                        \
    if ((int)__lane_id() == __builtin_amdgcn_readfirstlane((int)__lane_id())) \
      cnt.wd[k]++;                                                            \
  } while (0)
#else
#define RT2_WAVE(k) \
  do {              \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------
// Primitive tests: return whether the primitive is hit inside the interval and its t.

// AABB::Hit (AABB.hpp:34-47); inv = 1/d per axis (the same value the reference computes per node)
__device__ __forceinline__ bool aabb_hit(float4 lo, float4 hi, f3 o, f3 inv, float tmin, float tmax) {
  float t0 = (lo.x - o.x) * inv.x, t1 = (hi.x - o.x) * inv.x;
  if (t1 < t0) { float s = t0; t0 = t1; t1 = s; }
  tmin = gmax(t0, tmin);
  tmax = gmin(t1, tmax);
  if (tmax <= tmin) return false;
  t0 = (lo.y - o.y) * inv.y;
  t1 = (hi.y - o.y) * inv.y;
  if (t1 < t0) { float s = t0; t0 = t1; t1 = s; }
  tmin = gmax(t0, tmin);
  tmax = gmin(t1, tmax);
  if (tmax <= tmin) return false;
  t0 = (lo.z - o.z) * inv.z;
  t1 = (hi.z - o.z) * inv.z;
  if (t1 < t0) { float s = t0; t0 = t1; t1 = s; }
  tmin = gmax(t0, tmin);
  tmax = gmin(t1, tmax);
  return !(tmax <= tmin);
}

// aabb_hit when no slab value can be NaN (inv finite, so (bound - o) * inv is finite or +-inf):
// the swap + glm::max/min chain with early exits then equals min/max of all axes at once.
// min / max of the slab tests as single instructions. fminf / fmaxf (IEEE minNum / maxNum) make the
// compiler quiet possible signalling NaNs first (a v_max_f32 x, x per operand it cannot prove
// canonical: loop-carried tmax, values from another block); every operand here comes out of a
// VALU operation or is a finite record bound, so it is never a signalling NaN, and v_min_f32 /
// v_max_f32 already return the other operand for a quiet NaN: the same values, minNum / maxNum
// semantics included (the padded slab test relies on NaN being ignored).
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// t0 = max(min(ax, bx), min(ay, by), min(az, bz), tmin), t1 likewise: max and min are associative
// and commutative on these operands (NaN aside, which the callers exclude or which minNum ignores
// in any grouping), so the grouping below gives the reference's values.
__device__ __forceinline__ void slab_t(float ax, float bx, float ay, float by, float az, float bz, float tmin,
                                       float tmax, float& t0, float& t1) {
  t0 = vmax3(vmin(ax, bx), vmin(ay, by), vmax(vmin(az, bz), tmin));
  t1 = vmin3(vmax(ax, bx), vmax(ay, by), vmin(vmax(az, bz), tmax));
}

__device__ __forceinline__ bool aabb_hit_fin(float4 lo, float4 hi, f3 o, f3 inv, float tmin, float tmax) {
  const float ax = (lo.x - o.x) * inv.x, bx = (hi.x - o.x) * inv.x;
  const float ay = (lo.y - o.y) * inv.y, by = (hi.y - o.y) * inv.y;
  const float az = (lo.z - o.z) * inv.z, bz = (hi.z - o.z) * inv.z;
  float t0, t1;
  slab_t(ax, bx, ay, by, az, bz, tmin, tmax, t0, t1);
  return !(t1 <= t0);  // AABB::Hit: a miss when t1 <= t0 (AABB.hpp)
}
// The padded box test of an accelerated list's tree (the library's own conservative cull, not the
// reference's AABB::Hit): bounds lo - pad, hi + pad as fma(bound - o, inv, -+pinv) with pinv = pad * inv
// computed once per ray (inv from acc_slab_inv, rt2_layout.h). rt2_selftest which 4 checks on the
// GPU that it never rejects a box the ray's exact (double-precision) padded slab accepts.
__device__ __forceinline__ bool acc_slab(f3 lo, f3 hi, f3 o, f3 inv, f3 pinv, float tmin, float tmax) {
  const float ax = fmaf(lo.x - o.x, inv.x, -pinv.x), bx = fmaf(hi.x - o.x, inv.x, pinv.x);
  const float ay = fmaf(lo.y - o.y, inv.y, -pinv.y), by = fmaf(hi.y - o.y, inv.y, pinv.y);
  const float az = fmaf(lo.z - o.z, inv.z, -pinv.z), bz = fmaf(hi.z - o.z, inv.z, pinv.z);
  float t0, t1;
  slab_t(ax, bx, ay, by, az, bz, tmin, tmax, t0, t1);
  return t0 <= t1;
}
__device__ __forceinline__ bool finite3(f3 v) {
  return __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z);
}

// a / b, correctly rounded, from inv = fl(1 / b) (correctly rounded): q0 = a * inv and one fma
// correction q0 + (a - b q0) inv. Equal to IEEE a / b for every pair of significands
// (rt2_selftest which 6 checks all 2^46 pairs; the algorithm and the quotient scale exactly with the
// exponents) whenever no intermediate under/overflows; the callers reject every case where one
// could (|b| <= 1e-8 or a quotient below tmin), and selftests 0 and 3 check their ranges.
__device__ __forceinline__ float div_by_inv(float a, float b, float inv) {
  const float q = a * inv;
  return fmaf(fmaf(-b, q, a), inv, q);
}

// The box-level MakeBox test (boxaa.h, shared with its host proof harness) with the kernel's exact
// arithmetic: division by the ray's correctly rounded reciprocal, single-instruction min / max / med3.
struct BoxMath {
  static __device__ __forceinline__ float div(float a, float b, float inv) { return div_by_inv(a, b, inv); }
  static __device__ __forceinline__ float min(float a, float b) { return vmin(a, b); }
  static __device__ __forceinline__ float max(float a, float b) { return vmax(a, b); }
  static __device__ __forceinline__ float min3(float a, float b, float c) { return vmin3(a, b, c); }
  static __device__ __forceinline__ float max3(float a, float b, float c) { return vmax3(a, b, c); }
  // min / max of the magnitudes, the |.| as source modifiers
  static __device__ __forceinline__ float amin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, |%1|, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  }
  static __device__ __forceinline__ float amax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  }
  static __device__ __forceinline__ float med3(float a, float b, float c) { return __builtin_amdgcn_fmed3f(a, b, c); }
  static __device__ __forceinline__ float fma(float a, float b, float c) { return fmaf(a, b, c); }
  static __device__ __forceinline__ float abs(float a) { return fabsf(a); }
  static __device__ __forceinline__ uint32_t bits(float a) { return __float_as_uint(a); }
};

// Quad::Hit (Quad.cpp:19-43): inclusive interval (Contains)
template <int kMode>
__device__ __forceinline__ bool quad_t(const Nodes<kMode>& N, uint32_t off, f3 o, f3 d, float tmin, float tmax,
                                       float& t_out) {
  float4 r0 = N[off];
  f3 n = xyz(r0);
  float n_dot = dot(n, d);
  if (fabsf(n_dot) <= 1e-8f) return false;  // |n.d| < 1e-8 (double)
  float t = (r0.w - dot(n, o)) / n_dot;
  if (!(tmin <= t && t <= tmax)) return false;
  float4 r1 = N[off + 1], r2 = N[off + 2], r3 = N[off + 3], r4 = N[off + 4];
  f3 p = o + d * t;
  f3 pv = p - xyz(r1);
  float alpha = dot(xyz(r4), cross(pv, xyz(r3)));
  float beta = dot(xyz(r4), cross(xyz(r2), pv));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return false;
  t_out = t;
  return true;
}

// The range in which a sphere root (hh -+ sq) / a may be taken as div_by_inv(num, a, fl(1/a)): every
// intermediate normal and finite. 2^-60 <= a <= 2^60 and |hh| + sq <= 2^60 bound the quotient and the
// products; each numerator is +0 (exact: 0 * inv = +0 = +0 / a) or has |num| >= max(2^-70, 2^-60 a),
// so the quotient is >= 2^-60 and the fma residual (about 2^-24 |num|) stays above 2^-126. A cancelled
// numerator below that (a medium's boundary queries accept every root, ConstantMedium.cpp:18) or -0
// (IEEE gives -0 / a = -0, the correction +0) takes the IEEE division. rt2_selftest which 8 checks the
// fast roots against IEEE division on rays from near a sphere's surface (cancelled numerators down to
// the subnormal range) at every interval kind.
__device__ __forceinline__ bool sphere_fast_ok(float a, float hh, float sq) {
  const float n1 = hh - sq, n2 = hh + sq;
  const float lo = fmaxf(0x1p-70f, 0x1p-60f * a);
  const bool ok1 = fabsf(n1) >= lo || __float_as_uint(n1) == 0u;
  const bool ok2 = fabsf(n2) >= lo || __float_as_uint(n2) == 0u;
  return a >= 0x1p-60f && a <= 0x1p60f && fabsf(hh) + sq <= 0x1p60f && ok1 && ok2;
}
// The same for a query on [tmin, tmax] with tmin >= 0.001 (every query but a medium's boundary
// queries): an accepted root then has |num| >= 0.001 a >= 2^-70 (the residual stays normal), and a
// root whose numerator is below that range, computed to within a few ulps, is far below tmin on either
// path, so it is rejected either way; only a and the products' range need the check.
__device__ __forceinline__ bool sphere_fast_ok_pos(float a, float hh, float sq) {
  return a >= 0x1p-60f && a <= 0x1p60f && fabsf(hh) + sq <= 0x1p60f;
}
// Sphere::Hit (Sphere.cpp:7-37): exclusive interval (Surrounds); uv is dead output. kDiv 0: the fast
// roots when every lane of the wave is in sphere_fast_ok_pos's range (queries with tmin >= 0.001);
// 4: in sphere_fast_ok's (any interval: a medium's boundary queries); 1 / 3: when this lane is in
// sphere_fast_ok's / sphere_fast_ok_pos's range (selftest); 2: IEEE division only (selftest reference).
// kMotion false (kernels for scenes whose spheres all stand still, kFeatMotion): center(time) = c0.
template <int kDiv = 0, bool kMotion = true>
__device__ __forceinline__ bool sphere_t_rec(float4 r0, float4 r1, f3 o, f3 d, float time, float tmin, float tmax,
                                             float& t_out) {
  const f3 center = kMotion ? xyz(r0) + xyz(r1) * time : xyz(r0);
  f3 oc = center - o;
  float a = dot(d, d);
  float hh = dot(d, oc);
  float c = dot(oc, oc) - r0.w * r0.w;
  float disc = hh * hh - a * c;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  // The two roots (hh -+ sq) / a: by the correctly rounded 1/a with one fma correction
  // (div_by_inv, equal to IEEE division for every pair of significands) in sphere_fast_ok's range;
  // IEEE division otherwise.
  bool fast = false;
  if constexpr (kDiv == 0) fast = __all(sphere_fast_ok_pos(a, hh, sq));
  if constexpr (kDiv == 4) fast = __all(sphere_fast_ok(a, hh, sq));
  if constexpr (kDiv == 1) fast = sphere_fast_ok(a, hh, sq);
  if constexpr (kDiv == 3) fast = sphere_fast_ok_pos(a, hh, sq);
  const float inv_a = fast ? rcp_nr(a) : 0.0f;
  float root = fast ? div_by_inv(hh - sq, a, inv_a) : (hh - sq) / a;
  if (!(tmin < root && root < tmax)) {
    root = fast ? div_by_inv(hh + sq, a, inv_a) : (hh + sq) / a;
    if (!(tmin < root && root < tmax)) return false;
  }
  t_out = root;
  return true;
}
template <int kMode, int kDiv = 0, bool kMotion = true>
__device__ __forceinline__ bool sphere_t(const Nodes<kMode>& N, uint32_t off, f3 o, f3 d, float time, float tmin,
                                         float tmax, float& t_out) {
  return sphere_t_rec<kDiv, kMotion>(N[off], N[off + 1], o, d, time, tmin, tmax, t_out);
}

// Quad::Hit split in two: the candidate (pure function of the ray) and the interval test. The
// reference tests the interval before the interior; both are side-effect free, so testing the
// interior first and applying the interval afterwards gives the same hit.
template <int kMode>
__device__ __forceinline__ bool quad_cand(const Nodes<kMode>& N, uint32_t off, f3 o, f3 d, float& t_out) {
  float4 r0 = N[off];
  f3 n = xyz(r0);
  float n_dot = dot(n, d);
  float t = (r0.w - dot(n, o)) / n_dot;
  float4 r1 = N[off + 1], r2 = N[off + 2], r3 = N[off + 3], r4 = N[off + 4];
  f3 p = o + d * t;
  f3 pv = p - xyz(r1);
  float alpha = dot(xyz(r4), cross(pv, xyz(r3)));
  float beta = dot(xyz(r4), cross(xyz(r2), pv));
  t_out = t;
  return !(fabsf(n_dot) <= 1e-8f) && (0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f);
}

// quad_cand on a record held in registers: w[0..19] = (n, D) (q, mat) (u, -) (v, -) (w, -)
__device__ __forceinline__ bool quad_cand_w(const float* w, f3 o, f3 d, float& t_out) {
  f3 n = mk(w[0], w[1], w[2]);
  float n_dot = dot(n, d);
  float t = (w[3] - dot(n, o)) / n_dot;
  f3 p = o + d * t;
  f3 pv = p - mk(w[4], w[5], w[6]);
  f3 ww = mk(w[16], w[17], w[18]);
  float alpha = dot(ww, cross(pv, mk(w[12], w[13], w[14])));
  float beta = dot(ww, cross(mk(w[8], w[9], w[10]), pv));
  t_out = t;
  return !(fabsf(n_dot) <= 1e-8f) && (0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f);
}

// Axis-aligned Quad::Hit (record axis code K + 1): with n and w exactly zero off axis K,
// dot(n, d), dot(n, o) and dot(w, cross(., .)) equal the single axis-K products in value (the
// other terms are signed zeros, which no comparison distinguishes), so this returns the same
// decision and t as quad_cand_w at a third of the arithmetic.
// The float above 1e-8f: |n.d| > 1e-8f, the quads' parallel-ray rejection (Quad.cpp:22, |denom| < 1e-8
// in double, is |denom| <= 1e-8f for a float denom), as |n.d| >= kAboveDenomMin
constexpr float kAboveDenomMin = 0x1.5798f0p-27f;
static_assert(kAboveDenomMin > 1e-8f && 0x1.5798eep-27f == 1e-8f, "the float after 1e-8f");
template <int K>
__device__ __forceinline__ float comp(f3 v) {
  return K == 0 ? v.x : (K == 1 ? v.y : v.z);
}
template <int K>
__device__ __forceinline__ bool quad_cand_aa(const float* w, f3 o, f3 d, float& t_out) {
  constexpr int A = (K + 1) % 3, B = (K + 2) % 3;
  const float nk = w[K], wk = w[16 + K];
  float n_dot = nk * comp<K>(d);
  float t = (w[3] - nk * comp<K>(o)) / n_dot;
  float pva = (comp<A>(o) + comp<A>(d) * t) - w[4 + A];
  float pvb = (comp<B>(o) + comp<B>(d) * t) - w[4 + B];
  float alpha = wk * (pva * w[12 + B] - w[12 + A] * pvb);  // w . cross(pv, v)
  float beta = wk * (w[8 + A] * pvb - pva * w[8 + B]);    // w . cross(u, pv)
  t_out = t;
  return !(fabsf(n_dot) <= 1e-8f) && (0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f);
}
// Unit-normal axis-aligned Quad::Hit (axis code K + 4, n[K] = s = +-1): n_dot = s * d[K] and
// t = (D - s * o[K]) / (s * d[K]) = (sD - o[K]) / d[K] exactly (negation commutes with rounding),
// computed from the ray's inv[K] = fl(1 / d[K]) with div_by_inv.
template <int K>
__device__ __forceinline__ bool quad_cand_unit(const float* w, f3 o, f3 d, f3 inv, float& t_out) {
  constexpr int A = (K + 1) % 3, B = (K + 2) % 3;
  const float wk = w[16 + K];
  const float dk = comp<K>(d);
  float t = div_by_inv(w[19] - comp<K>(o), dk, comp<K>(inv));
  float pva = (comp<A>(o) + comp<A>(d) * t) - w[4 + A];
  float pvb = (comp<B>(o) + comp<B>(d) * t) - w[4 + B];
  float alpha = wk * (pva * w[12 + B] - w[12 + A] * pvb);  // w . cross(pv, v)
  float beta = wk * (w[8 + A] * pvb - pva * w[8 + B]);    // w . cross(u, pv)
  t_out = t;
  return !(fabsf(dk) <= 1e-8f) && (0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f);
}
// lo <= t <= hi (IEEE compares) for 0 < lo <= hi <= FLT_MAX <=> bits(t) - bits(lo) <= bits(hi) -
// bits(lo) (unsigned, wrapping): positive floats order as their bits; a t below lo, a negative t,
// -0, +inf or a NaN lands above the largest right side bits(FLT_MAX) - bits(lo).
__device__ __forceinline__ bool in_interval(float t, float lo, float hi) {
  return __float_as_uint(t) - __float_as_uint(lo) <= __float_as_uint(hi) - __float_as_uint(lo);
}
// Unit-normal axis-aligned Quad::Hit from a QUADAA record r = (sD, lo[A], hi[A], lo[B], hi[B]): t as
// quad_cand_unit computes it, the hit point's coordinates p[A], p[B] as Quad::Hit computes them
// (r.at(t)), and the interior test alpha, beta in [0, 1] as lo <= p <= hi on each coordinate: the
// compiler records rectangles only, whose alpha depends on p[A] alone through monotone rounded
// operations and beta on p[B] alone, and the bounds are the first and last floats it accepts
// (compile.cpp CoordRange), so the decision is the same for every finite p.
// Returned as a rejection word whose sign bit is set when the quad is not hit: the sign of a rounded
// difference is the sign of the exact one (a zero only for equal operands, +0 then; lo is stored as -0
// where it is 0, so p = -0 passes as p = +0 does), so p - lo, hi - p, ... are all >= 0 exactly when p
// is inside, and |d_K| - (the float above 1e-8f) >= 0 exactly when |d_K| > 1e-8f (Quad.cpp:22:
// |denom| < 1e-8, in double). One OR of the words and one sign test instead of five compare masks
// and their scalar ANDs: the lockstep kernels' scalar unit is as busy as their vector pipes. (The ray's
// o and d are finite, so t and p are: compile.cpp RectAAWords bounds the scene.)
template <int K>
__device__ __forceinline__ uint32_t quad_aa(const float* r, f3 o, f3 d, f3 inv, float& t_out) {
  constexpr int A = (K + 1) % 3, B = (K + 2) % 3;
  const float dk = comp<K>(d);
  const float t = div_by_inv(r[0] - comp<K>(o), dk, comp<K>(inv));
  const float pa = comp<A>(o) + comp<A>(d) * t;
  const float pb = comp<B>(o) + comp<B>(d) * t;
  t_out = t;
  return (__float_as_uint(pa - r[1]) | __float_as_uint(r[2] - pa) | __float_as_uint(pb - r[3])) |
         (__float_as_uint(r[4] - pb) | __float_as_uint(fabsf(dk) - kAboveDenomMin));
}
__device__ __forceinline__ uint32_t quad_aa_k(uint32_t k, const float* r, f3 o, f3 d, f3 inv, float& t) {
  if (k == 0u) return quad_aa<0>(r, o, d, inv, t);
  if (k == 1u) return quad_aa<1>(r, o, d, inv, t);
  return quad_aa<2>(r, o, d, inv, t);
}

// quad candidate dispatched on a wave-uniform axis code
__device__ __forceinline__ bool quad_cand_u(uint32_t axis, const float* w, f3 o, f3 d, f3 inv, float& t) {
  switch (axis) {
    case 1: return quad_cand_aa<0>(w, o, d, t);
    case 2: return quad_cand_aa<1>(w, o, d, t);
    case 3: return quad_cand_aa<2>(w, o, d, t);
    case 4: return quad_cand_unit<0>(w, o, d, inv, t);
    case 5: return quad_cand_unit<1>(w, o, d, inv, t);
    case 6: return quad_cand_unit<2>(w, o, d, inv, t);
    default: return quad_cand_w(w, o, d, t);
  }
}

// (kBoundary: a medium's boundary query, on any interval)
template <uint32_t F, int kMode, bool kBoundary = false>
__device__ __forceinline__ bool prim_t(const Nodes<kMode>& N, uint32_t ref, f3 o, f3 d, float time, float tmin,
                                       float tmax, float& t, Counters& cnt) {
  uint32_t off = ref & kOffsetMask;
  if constexpr (Has<F, kFeatSphere>()) {
    if ((ref >> 28) == kSphere) {
      cnt.sphere++;
      return sphere_t<kMode, kBoundary ? 4 : 0, Has<F, kFeatMotion>()>(N, off, o, d, time, tmin, tmax, t);
    }
  }
  cnt.quad++;
  return quad_t(N, off, o, d, tmin, tmax, t);
}

// Closest t of a ConstantMedium boundary (quad, sphere or a leaf-only list) on [lo, hi]
template <uint32_t F, int kMode>
__device__ __forceinline__ bool boundary_t(const Nodes<kMode>& N, uint32_t ref, f3 o, f3 d, float time, float lo,
                                           float hi, float& t_out, Counters& cnt) {
  if ((ref >> 28) != kList) return prim_t<F, kMode, true>(N, ref, o, d, time, lo, hi, t_out, cnt);
  uint32_t off = ref & kOffsetMask;
  uint32_t n = N.word(off, 0);
  bool any = false;
  for (uint32_t k = 0; k < n; k++) {
    float t;
    if (prim_t<F, kMode, true>(N, N.word(off + 1, k), o, d, time, lo, hi, t, cnt)) {
      any = true;
      hi = t;
    }
  }
  if (any) t_out = hi;
  return any;
}

// Parent space -> model space of one XFORM (Transform.cpp:13-20)
template <int kMode>
__device__ __forceinline__ void to_model(const Nodes<kMode>& N, uint32_t off, f3& o, f3& d) {
  float4 c0 = N[off], c1 = N[off + 1], c2 = N[off + 2], c3 = N[off + 3];
  f3 no = mk((c0.x * o.x + c1.x * o.y) + (c2.x * o.z + c3.x), (c0.y * o.x + c1.y * o.y) + (c2.y * o.z + c3.y),
             (c0.z * o.x + c1.z * o.y) + (c2.z * o.z + c3.z));
  f3 nd = mk(c0.x * d.x + c1.x * d.y + c2.x * d.z, c0.y * d.x + c1.y * d.y + c2.y * d.z,
             c0.z * d.x + c1.z * d.y + c2.z * d.z);
  o = no;
  d = normalize(nd);
}

// Ray in the space of XFORM `xref` (kRefNone = world), rebuilt from the world ray through the chain
// of enclosing transforms; recomputing gives the same bits as the traversal's incremental path.
template <int kMode>
__device__ __forceinline__ void ray_in_space(const Nodes<kMode>& N, uint32_t xref, f3 wo, f3 wd, f3& o, f3& d) {
  o = wo;
  d = wd;
  if (xref == kRefNone) return;
  uint32_t parent = N.word((xref & kOffsetMask) + 1, 3);
  if (parent == kRefNone) {  // the common single-level case
    to_model(N, xref & kOffsetMask, o, d);
    return;
  }
  uint32_t chain[8];
  int n = 0;
  for (uint32_t x = xref; x != kRefNone && n < 8; x = N.word((x & kOffsetMask) + 1, 3)) chain[n++] = x;
  for (int k = n - 1; k >= 0; k--) to_model(N, chain[k] & kOffsetMask, o, d);
}

// ConstantMedium::Hit (ConstantMedium.cpp:14-58) on [tmin, tmax]: two boundary queries, then one
// random number for the free-flight distance. Returns the medium's t.
template <uint32_t F, int kMode, class G>
__device__ __forceinline__ bool medium_t(const Nodes<kMode>& N, uint32_t off, f3 o, f3 d, float time, float tmin,
                                         float tmax, G& path, float& t_out, Counters& cnt) {
  float4 r0 = N[off];
  uint32_t bref = bits(r0.z);
  float t1, t2;
  if (!boundary_t<F>(N, bref, o, d, time, -FLT_MAX, FLT_MAX, t1, cnt)) return false;
  if (!boundary_t<F>(N, bref, o, d, time, (float)((double)t1 + 0.0001), FLT_MAX, t2, cnt)) return false;
  t1 = fmaxf(t1, tmin);
  t2 = fminf(t2, tmax);
  if (t1 >= t2) return false;
  t1 = fmaxf(t1, 0.0f);
  float len = sqrtf(dot(d, d));
  float inside = (t2 - t1) * len;
  float hit_dist = r0.x * log_u(path.uniform());
  if (hit_dist > inside) return false;
  t_out = t1 + hit_dist / len;
  return true;
}

// ConstantMedium boundary in the threaded traversal: the medium step is wave-uniform, so its
// boundary records are scalar loads, and an axis-aligned boundary quad (every box face) takes the
// axis-aligned test with IEEE division (quad_cand_aa, the same decision and t as Quad::Hit).
template <uint32_t F>
__device__ __forceinline__ bool boundary_prim_lin(const void* recs, uint32_t ref, f3 o, f3 d, float time, float lo,
                                                  float hi, float& t_out, Counters& cnt) {
  const uint32_t off = ref & kOffsetMask;
  if (Has<F, kFeatSphere>() && (ref >> 28) == kSphere) {
    cnt.sphere++;
    return sphere_t<kModeLinear, 4, Has<F, kFeatMotion>()>(Nodes<kModeLinear>{reinterpret_cast<const float4*>(recs), 0u},
                                                             off, o, d, time, lo, hi, t_out);
  }
  cnt.quad++;
  u32x16 a;
  u32x4 b2;
  sld20(recs, off * 16u, a, b2);
  float w[20];
#pragma unroll
  for (int j = 0; j < 16; j++) w[j] = uf(a[j]);
#pragma unroll
  for (int j = 0; j < 4; j++) w[16 + j] = uf(b2[j]);
  const uint32_t code = a[11];  // axis code (compile.cpp): k + 1, or k + 4 for a unit normal
  float t;
  bool ok;
  if (code == 1u || code == 4u) {
    ok = quad_cand_aa<0>(w, o, d, t);
  } else if (code == 2u || code == 5u) {
    ok = quad_cand_aa<1>(w, o, d, t);
  } else if (code == 3u || code == 6u) {
    ok = quad_cand_aa<2>(w, o, d, t);
  } else {
    ok = quad_cand_w(w, o, d, t);
  }
  if (!(ok && lo <= t && t <= hi)) return false;  // Quad::Hit: Contains (inclusive)
  t_out = t;
  return true;
}

template <uint32_t F>
__device__ __forceinline__ bool boundary_t_lin(const void* recs, uint32_t ref, f3 o, f3 d, float time, float lo,
                                               float hi, float& t_out, Counters& cnt) {
  if ((ref >> 28) != kList) return boundary_prim_lin<F>(recs, ref, o, d, time, lo, hi, t_out, cnt);
  const uint32_t off = ref & kOffsetMask;
  const uint32_t n = sld1(recs, off * 16u);
  bool any = false;
  for (uint32_t k = 0; k < n; k++) {  // HittableList::Hit (HittableList.cpp:8-22)
    float t;
    if (boundary_prim_lin<F>(recs, sld1(recs, (off + 1u) * 16u + 4u * k), o, d, time, lo, hi, t, cnt)) {
      any = true;
      hi = t;
    }
  }
  if (any) t_out = hi;
  return any;
}

// A box boundary (rt2_layout.h MEDIUM, kBoundaryAAFlag): the closest of its quads on [lo, hi], list
// order, each by the unit-normal test with IEEE division: t = (sD - o_K) / d_K is exactly
// Quad::Hit's (D - n.o) / (n.d) for n = +-e_K (negation commutes with rounding), the interior test is
// quad_aa's (the QUADAA bounds), and the interval test is Contains (inclusive).
// (div_by_inv with the ray's reciprocal instead of the division: +0.7 % at 7 waves, -0.6 % at 8;
// not used)
template <int K>
__device__ __forceinline__ bool quad_aa_div(const uint32_t* r, f3 o, f3 d, float& t_out) {
  constexpr int A = (K + 1) % 3, B = (K + 2) % 3;
  const float dk = comp<K>(d);
  const float t = (uf(r[0]) - comp<K>(o)) / dk;
  const float pa = comp<A>(o) + comp<A>(d) * t;
  const float pb = comp<B>(o) + comp<B>(d) * t;
  t_out = t;
  return (int)((__float_as_uint(pa - uf(r[1])) | __float_as_uint(uf(r[2]) - pa) | __float_as_uint(pb - uf(r[3]))) |
               (__float_as_uint(uf(r[4]) - pb) | __float_as_uint(fabsf(dk) - kAboveDenomMin))) >= 0;
}
// Both boundary queries of ConstantMedium::Hit (ConstantMedium.cpp:14-58) on a box in one pass:
// each quad's t and interior decision do not depend on the query's interval, so its quads are
// tested once and the two answers selected from the candidates — t1 = the smallest candidate in
// [-FLT_MAX, FLT_MAX] (Interval::universe, kInfinity = FLT_MAX), t2 = the smallest in
// [fl(t1 + 0.0001), FLT_MAX] — which is what the two HittableList queries return (the closest hit in
// the interval; only its t is used). Half the quad tests of the two queries.
// The candidates wait in LDS planes of the wave (word k of the lane at cand[64 k]) between the two
// selections: held in six VGPRs they pushed the 8-wave kernel into 25 spilled VGPRs (round 3: 56 B
// of scratch per lane, 32 HBM bytes per ray); only the running minimum stays in a register.
__device__ __forceinline__ bool boundary_aa_pair(const void* recs, uint32_t off, uint32_t hdr, f3 o, f3 d, float& t1,
                                                 float& t2, lds_u32* cand, Counters& cnt) {
  const uint32_t n = (hdr >> 24) & 7u;
  float m = INFINITY;  // candidate t, +inf when the quad is missed (no interval accepts it)
  for (uint32_t k = 0; k < n; k += 2u) {  // wave-uniform
    const u32x16 w = sld16(recs, off + 32u * k);
#pragma unroll
    for (uint32_t j = 0; j < 2u; j++) {
      if (k + j < n) {
        uint32_t r[8];
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = w[8 * j + i];
        const uint32_t code = (hdr >> (3u * (k + j))) & 7u;
        float t;
        bool ok;
        if (code == 0u) {
          ok = quad_aa_div<0>(r, o, d, t);
        } else if (code == 1u) {
          ok = quad_aa_div<1>(r, o, d, t);
        } else {
          ok = quad_aa_div<2>(r, o, d, t);
        }
        cnt.quad += 2;  // the two queries' tests
        const float c = (ok && -FLT_MAX <= t && t <= FLT_MAX) ? t : INFINITY;
        m = fminf(m, c);
        pk_st(cand, k + j, bits(c));
      }
    }
  }
  if (!(m <= FLT_MAX)) return false;
  t1 = m;
  const float lb = (float)((double)m + 0.0001);
  float m2 = INFINITY;
  for (uint32_t k = 0; k < n; k++) {
    const float c = uf(pk_ld(cand, k));
    m2 = (lb <= c && c < m2) ? c : m2;
  }
  if (!(m2 <= FLT_MAX)) return false;
  t2 = m2;
  return true;
}

// medium_t with the boundary queries above (same operations, same random draw)
template <uint32_t F, class G>
__device__ __forceinline__ bool medium_t_lin(const void* recs, uint32_t moff, const u32x4 r0, f3 o, f3 d, f3 inv,
                                             float time, float tmin, float tmax, G& path, lds_u32* cand, float& t_out,
                                             Counters& cnt) {
  const uint32_t bref = r0.z;
  float t1, t2;
  // a box (the sphere scenes' kernels keep the general path: the 48 words cost them SGPRs)
  if (!Has<F, kFeatSphere>() && (r0.w & kBoundaryAAFlag)) {
    const uint32_t off = (moff + 1u) * 16u;
    // a MakeBox boundary: the box-level test of both queries (boxaa.h BoxAAPair); the lanes it cannot
    // certify take the six faces
    bool cert = false, ok = false;
    if (r0.w & kBoundaryBoxFlag) {
      const u32x8 bwr = sld8(recs, off + 32u * kBoundaryAAMax);
      float bw[kBoxAAWords];
#pragma unroll
      for (int j = 0; j < kBoxAAWords; j++) bw[j] = uf(bwr[j]);
      const BoxAAPairResult r = BoxAAPair<BoxMath>(bw, uf(bwr[6]), o.x, o.y, o.z, d.x, d.y, d.z, inv.x, inv.y, inv.z);
      // stats counters (flushed by the counting kernels only; dead code elsewhere)
      cnt.box++;
      const bool lead = (int)__lane_id() == __builtin_amdgcn_readfirstlane((int)__lane_id());
      cnt.box_wave += lead ? 1u : 0u;
      cnt.box_wave_run += (lead && !__all(r.cert)) ? 1u : 0u;
      if (r.cert) {
        cert = true;
        cnt.box_cert++;
        cnt.quad += 2u * kBoundaryAAMax;  // the two queries' face tests (the reference's count)
        // the second query's interval starts at fl(t1 + 0.0001): t1 itself for a large t1 (its face
        // then answers both queries), else past it (the exit face answers)
        const float lb = (float)((double)r.tin + 0.0001);
        t1 = r.tin;
        t2 = lb <= r.tin ? r.tin : r.tout;
        ok = r.through && t2 >= lb;
      }
    }
    if (!cert) ok = boundary_aa_pair(recs, off, r0.w, o, d, t1, t2, cand, cnt);
    if (!ok) return false;
  } else {
#if RT2_EXP_TWICE & 128
  {
    f3 o2 = o;
    asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
    Counters c2 = cnt;
    float u1 = 0.0f, u2 = 0.0f;
    const bool b1 = boundary_t_lin<F>(recs, bref, o2, d, time, -FLT_MAX, FLT_MAX, u1, c2);
    const bool b2 = b1 && boundary_t_lin<F>(recs, bref, o2, d, time, (float)((double)u1 + 0.0001), FLT_MAX, u2, c2);
    asm volatile("" ::"v"(u1), "v"(u2), "v"((int)b2));
  }
#endif
  if (!boundary_t_lin<F>(recs, bref, o, d, time, -FLT_MAX, FLT_MAX, t1, cnt)) return false;
  if (!boundary_t_lin<F>(recs, bref, o, d, time, (float)((double)t1 + 0.0001), FLT_MAX, t2, cnt)) return false;
  }
  t1 = fmaxf(t1, tmin);
  t2 = fminf(t2, tmax);
  if (t1 >= t2) return false;
  t1 = fmaxf(t1, 0.0f);
  float len = sqrtf(dot(d, d));
  float inside = (t2 - t1) * len;
  const float u = path.uniform();
#if RT2_EXP_TWICE & 64
  {
    float u2 = u;
    asm volatile("" : "+v"(u2));
    const float l2 = log_u(u2);
    asm volatile("" ::"v"(l2));
  }
#endif
  float hit_dist = uf(r0.x) * log_u(u);
  if (hit_dist > inside) return false;
  t_out = t1 + hit_dist / len;
  return true;
}

// The closest hit's world-space record and its material (resolve_hit + the material table)
struct HitShade {
  f3 hp, hn;
  bool front;
  float4 m0, m1;
  uint32_t type;
};

struct HitRef {
  float t;
  uint32_t prim;  // ref of the quad / sphere / medium that produced the closest hit
  uint32_t xf;    // innermost enclosing transform of that primitive (kRefNone = world)
};

// ------------------------------------------------------------------------------------------
// Closest hit over the scene program (HittableList{BVHNode} at the root, App.cpp:126).
// Reference semantics preserved: left-then-right, right subtree pruned by the current closest t,
// model-space t of transformed children compared as-is (Transform.cpp:82), span-1 media tested
// twice with fresh random numbers, media boundaries queried on (-FLT_MAX, FLT_MAX).

// Stack traversal (any scene): each lane walks its own steps — LDS stack pops, or the next child of
// a leaf list through a per-lane cursor — one step per loop trip.
template <uint32_t F, int kMode, bool kStats, class G>
__device__ __forceinline__ bool trace_stack(const RenderParams& P, const Nodes<kMode>& N, f3 wo, f3 wd, float time,
                                            G& path, HitRef& h, uint32_t* stk, Counters& cnt, bool& overflow) {
  f3 o = wo, d = wd;
  const f3 winv = recip3(wd);
  f3 inv = winv;
  const float tmin = 0.001f;  // Interval{0.001, kInfinity}
  float tmax = FLT_MAX;
  bool any = false;
  uint32_t cur_xf = kRefNone;
  const int cap = P.stack_depth;
  int sp = 0;
  uint32_t lword = 0, lrem = 0;  // leaf-list cursor: next child-ref word, children left
  uint32_t cur = P.root;         // next step
  float acc_pad = 0.0f;          // accelerated list: this ray's box padding
  uint32_t acc_best = kRefNone;  // accelerated list: record of its current closest child
  while (cur != kRefNone) {
    uint32_t kind = cur >> 28, off = cur & kOffsetMask;
    if (kind == kQuad || (Has<F, kFeatSphere>() && kind == kSphere)) {
      float t;
      if (prim_t<F>(N, cur, o, d, time, tmin, tmax, t, cnt)) {
        tmax = t;
        any = true;
        h.prim = cur;
        h.xf = cur_xf;
      }
    } else if (kind == kBvh) {
      if (kStats) cnt.bvh++;
      float4 lo = N[off], hi = N[off + 1];
      if (aabb_hit(lo, hi, o, inv, tmin, tmax)) {
        uint32_t right = bits(hi.w);
        if (right != kRefNone) {
          if (sp + 1 > cap) {
            overflow = true;
          } else {
            stk[(sp++) * kBlock] = right;
          }
        }
        cur = bits(lo.w);
        continue;  // the left child is the next step (no stack round trip)
      }
    } else if (kind == kList) {
      if (kStats) cnt.list++;
      uint32_t n = N.word(off, 0);
      bool leaf_only = true;
      if constexpr (Has<F, kFeatGenList>()) leaf_only = (N.word(off, 1) & kListLeafOnly) != 0u;
      if (leaf_only) {
        lword = 4u * (off + 1u);
        lrem = n;
      } else if (sp + (int)n > cap) {
        overflow = true;
      } else {
        for (int k = (int)n - 1; k >= 0; k--) stk[(sp++) * kBlock] = N.word(off + 1, (uint32_t)k);
      }
    } else if (Has<F, kFeatXform>() && kind == kXform) {
      if (kStats) cnt.xform++;
      if (sp + 1 > cap) {
        overflow = true;
      } else {
        to_model(N, off, o, d);
        inv = recip3(d);
        cur_xf = cur;
        stk[(sp++) * kBlock] = make_ref(kXformExit, off);
        cur = N.word(off, 3);  // the transformed child is the next step
        continue;
      }
    } else if (Has<F, kFeatXform>() && kind == kXformExit) {
      cur_xf = N.word(off + 1, 3);  // parent transform
      if (cur_xf == kRefNone) {
        o = wo;
        d = wd;
        inv = winv;
      } else {
        ray_in_space(N, cur_xf, wo, wd, o, d);
        inv = recip3(d);
      }
    } else if (Has<F, kFeatMedium>() && kind == kMedium) {
      if (kStats) cnt.medium++;
      float t;
      if (medium_t<F>(N, off, o, d, time, tmin, tmax, path, t, cnt)) {
        tmax = t;
        any = true;
        h.prim = cur;
        h.xf = cur_xf;
      }
    } else if (Has<F, kFeatSphere>() && kind == kListAcc) {
      // HittableList::Hit over many spheres through its exact acceleration tree (rt2_layout.h)
      if (kStats) cnt.list++;
      const float4 r0 = N[off], r1 = N[off + 1];
      const f3 dc = o - xyz(r0);
      const float L = sqrtf(dot(dc, dc)) * 1.0001f + r0.w;
      acc_pad = (r1.x * L + r1.y) * L + r1.z;
      acc_best = kRefNone;
      cur = bits(r1.w);
      continue;
    } else if (Has<F, kFeatSphere>() && is_acc_bvh(kind)) {
      if (kStats) cnt.bvh++;
      const float4 lo = N[off], hi = N[off + 1];
      // padded slab test; NaN from 0 * inf is ignored by fminf/fmaxf (a ray in a padded face
      // plane with zero direction component stays >= pad away from every child)
      const float ax = ((lo.x - acc_pad) - o.x) * inv.x, bx = ((hi.x + acc_pad) - o.x) * inv.x;
      const float ay = ((lo.y - acc_pad) - o.y) * inv.y, by = ((hi.y + acc_pad) - o.y) * inv.y;
      const float az = ((lo.z - acc_pad) - o.z) * inv.z, bz = ((hi.z + acc_pad) - o.z) * inv.z;
      const float t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
      const float t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax));
      if (t0 <= t1) {
        const uint32_t axis = kind - kAccBvh;
        const float dax = axis == 0u ? d.x : (axis == 1u ? d.y : d.z);
        const uint32_t nr = bits(lo.w), fr = bits(hi.w);
        const bool flip = dax < 0.0f;  // visit the child nearer along the split axis first
        if (sp + 1 > cap) {
          overflow = true;
        } else {
          stk[(sp++) * kBlock] = flip ? nr : fr;
        }
        cur = flip ? fr : nr;
        continue;
      }
    } else if (Has<F, kFeatSphere>() && kind == kAccSphere) {
      // smallest root wins; an equal root goes to the lower child index = lower record offset
      if (kStats) cnt.sphere++;
      float t;
      if (sphere_t<kMode, 0, Has<F, kFeatMotion>()>(N, off, o, d, time, tmin, FLT_MAX, t) &&
          (t < tmax || (t == tmax && acc_best != kRefNone && off < acc_best))) {
        tmax = t;
        any = true;
        h.prim = make_ref(kSphere, off);
        h.xf = cur_xf;
        acc_best = off;
      }
    }
    // next step: the leaf-list cursor first, then the stack
    if (lrem != 0u) {
      cur = N.word(0, lword++);
      lrem--;
    } else if (sp > 0) {
      cur = stk[(--sp) * kBlock];
    } else {
      cur = kRefNone;
    }
  }
  h.t = tmax;
  return any;
}

// Threaded traversal (small scenes): all lanes of the wave walk the pre-order program in lockstep.
// Each lane keeps the index of its next step; the wave executes the smallest pending index, so the
// step kind is wave-uniform (no divergence between kinds) and the step's 64 bytes (program entry +
// the first 48 bytes of its record, P.lin_wide) are one scalar load into SGPRs. A lane whose AABB
// test misses jumps to the node's skip index. Per lane the visit order is exactly the stack
// traversal's.
// Smallest `next` over the wave's active lanes (one ballot per distinct smaller value).
__device__ __forceinline__ uint32_t wave_min_next(uint32_t next) {
  uint32_t i = __builtin_amdgcn_readfirstlane(next);
  unsigned long long lower;
  while ((lower = __ballot(next < i)) != 0ull) i = __builtin_amdgcn_readlane(next, __ffsll((long long)lower) - 1);
  return i;
}

// The box-level test of box-flagged MakeBox runs (boxaa.h), in every kernel with quads (the compiler flags
// the runs: book 2's ground boxes, the Cornell box's two boxes; DESIGN.md §4 "Box-level test").
template <uint32_t F>
constexpr bool BoxOn() {
  return true;
}
template <uint32_t F, bool kStats, class W, class G>
__device__ __forceinline__ bool trace_linear(const RenderParams& P, const W& wray, float time, G& path, HitRef& h,
                                             lds_u32* cand, lds_u32* xray, Counters& cnt) {
  const Nodes<kModeLinear> N{reinterpret_cast<const float4*>(P.lind)};  // boundaries / nested xforms
  const void* recs = P.lind;
  // the world ray's reciprocal stays in registers for the transforms' exits to world space (three
  // VGPRs live across the trace), except with the parked ray (book 2), which recomputes it there
  constexpr bool kKeepW = !__is_same(W, ParkRay);
  f3 o = wray.wo(), d = wray.wd();
  f3 inv = recip3(d);
  const f3 winv = inv;
  bool fin = finite3(inv);  // inv finite: the NaN-free slab test applies
  const bool wfin = fin;
  const float tmin = 0.001f;
  float tmax = FLT_MAX;
  uint32_t prim = kRefNone;  // closest primitive so far (h.xf: its transform, quads: from the record)
  uint32_t cur_xf = kRefNone;
  f3 acc_pinv = mk(0.0f, 0.0f, 0.0f);  // accelerated list: this ray's box padding x inv
  uint32_t acc_best = kRefNone;  // accelerated list: child index of its current closest sphere
  uint32_t next = 0;  // this lane's next step
  RT2_WAVE(0);
#if RT2_EXP_WAVESTEPS
  cnt.wd[7]++;
#endif
  uint32_t i = wave_min_next(next);  // wave-uniform step = min over live lanes of `next`
  // (i reaches P.lin_len when every lane is done: the wide program's entry there is kProgramEnd)
  while (true) {
    u32x16 sw = sld16(P.lin_wide, i * 64u);  // entry + the first 48 bytes of its record
    if (sw[0] == kBvh) {
      // A run of BVH steps in a loop of their own: only `next` changes from step to step, so
      // nothing else is carried (no register copies between kinds) and the step costs the slab
      // test, the next-index update and the wave-minimum search. A paired step (compile.cpp: word
      // 2 is not i + 1; sphere scenes only) also tests its near child's box (words 7, 11-15), with
      // the tmax that child's own step would see (nothing runs between the two in pre-order), and
      // jumps past it. (Accelerated-list trees are walked lane by lane at their LISTACC step.)
      const bool allfin = __all(fin);
      do {
        RT2_WAVE(1);
        RT2_WAVE(2);
        // kSel: every lane evaluates the step (the same VALU issue: masked lanes cost their slots
        // anyway) and the lanes at it take the result by a select, no exec-mask branch per step
        // (Cornell +0.4 %; the sphere kernels keep the branch: book 1 -0.4 % with the select)
        constexpr bool kSel = !Has<F, kFeatSphere>();
        const bool act = next == i;
        if (kSel || act) {
          if (kStats && act) cnt.bvh++;
          const float4 lo = make_float4(uf(sw[4]), uf(sw[5]), uf(sw[6]), 0.0f);
          const float4 hi = make_float4(uf(sw[8]), uf(sw[9]), uf(sw[10]), 0.0f);
          const bool in = allfin ? aabb_hit_fin(lo, hi, o, inv, tmin, tmax) : aabb_hit(lo, hi, o, inv, tmin, tmax);
          uint32_t nx = in ? i + 1u : sw[1];
          if (Has<F, kFeatSphere>() && sw[2] != i + 1u) {
            const float4 lo2 = make_float4(uf(sw[7]), uf(sw[11]), uf(sw[12]), 0.0f);
            const float4 hi2 = make_float4(uf(sw[13]), uf(sw[14]), uf(sw[15]), 0.0f);
            const bool in2 =
                allfin ? aabb_hit_fin(lo2, hi2, o, inv, tmin, tmax) : aabb_hit(lo2, hi2, o, inv, tmin, tmax);
            if (kStats && act && in) cnt.bvh++;
            nx = in ? (in2 ? sw[2] : sw[3]) : sw[1];
          }
#if RT2_EXP_TWICE & 8
          {
            f3 o2 = o;
            asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
            const bool in2 = allfin ? aabb_hit_fin(lo, hi, o2, inv, tmin, tmax) : aabb_hit(lo, hi, o2, inv, tmin, tmax);
            asm volatile("" ::"v"((int)in2));
          }
#endif
          next = kSel && !act ? next : nx;
        }
        i = wave_min_next(next);
        sw = sld16(P.lin_wide, i * 64u);
      } while (sw[0] == kBvh);
    }
    const u32x4 st = {sw[0], sw[1], sw[2], sw[3]};
    const uint32_t kind = st.x, off = st.z;
    if (kind == kProgramEnd) break;
    RT2_WAVE(1);
    if (kind == kQuad) RT2_WAVE(3);
    if (is_acc_bvh(kind)) RT2_WAVE(2);
    if (kind == kSphere) RT2_WAVE(4);
    if (kind == kMedium) RT2_WAVE(5);
    const uint32_t at = i;
    i = kRefNone;  // computed after the step
    if (next == at) {
    next = at + 1u;
    if (kind == kQuad) {
      // a run of st.w quads with contiguous records, axis codes in st.y (3 bits each), tested in
      // order (issue-bound: one candidate at a time beats two interleaved, measured)
      const uint32_t run = st.w & kRunLenMask;
      // A MakeBox run with a box record (aux bit 31; compile.cpp, every scene unless RT2_BOX_AA=0): the box-level
      // test (boxaa.h) first. A certified lane takes the candidate face's answer and skips the run; the
      // wave runs the six faces only for the lanes it could not certify. The box record (six planes and
      // the margin constant, 2 records) lies right before the run's first face record; aux = run | flag
      // (compile.cpp BoxAAWordsOf).
      bool boxed = false;
      if constexpr (BoxOn<F>()) {
        if ((int)st.w < 0) {
          const u32x8 bwr = sld8(recs, (off - (uint32_t)kBoxAARecords) * 16u);
          float bw[kBoxAAWords];
#pragma unroll
          for (int j = 0; j < kBoxAAWords; j++) bw[j] = uf(bwr[j]);
          const uint32_t kmax0 = bits(tmax) - bits(tmin);
          const BoxAAResult r =
              BoxAATest<BoxMath>(bw, uf(bwr[6]), o.x, o.y, o.z, d.x, d.y, d.z, inv.x, inv.y, inv.z, tmin);
#if RT2_EXP_TWICE & 8192
          {
            float ox2 = o.x;
            asm volatile("" : "+v"(ox2));
            const BoxAAResult r2 =
                BoxAATest<BoxMath>(bw, uf(bwr[6]), ox2, o.y, o.z, d.x, d.y, d.z, inv.x, inv.y, inv.z, tmin);
            asm volatile("" ::"v"(r2.x), "v"(r2.t), "v"(r2.face), "v"((int)r2.cert));
          }
#endif
          if (kStats) {
            cnt.box++;
            const bool lead = (int)__lane_id() == __builtin_amdgcn_readfirstlane((int)__lane_id());
            cnt.box_wave += lead ? 1u : 0u;
            cnt.box_wave_run += (lead && !__all(r.cert)) ? 1u : 0u;
          }
          if (r.cert) {
            if (kStats) {
              cnt.quad += 6;  // the run's six Quad::Hit tests (the reference's count)
              cnt.box_cert++;
            }
            if (r.x <= kmax0) {
              tmax = r.t;
              prim = make_ref(kQuadAA, off + r.face * (uint32_t)kQuadRecords);
            }
            boxed = true;
          }
        }
      }
      if (!boxed) {
      uint32_t codes = st.y;  // 3 bits per quad, then a 1 bit (compile.cpp)
      // the run's interval test in_interval(t, tmin, tmax) as key(t) <= kmax with key(x) = bits(x) -
      // bits(tmin) (kmax = key(tmax), updated with the accepted t's key; tmax = its float after the run)
      uint32_t kmax = bits(tmax) - bits(tmin);
      uint32_t boff = off * 16u;  // byte offset of the quad's record
      // the quad's QUADAA ref, counted in a VGPR (one VALU add per quad instead of two scalar
      // instructions and a copy to build each accepted ref: the scalar unit is the busier pipe)
      uint32_t vref = make_ref(kQuadAA, off);
      asm volatile("" : "+v"(vref));
      for (bool first = true;; first = false) {
        const uint32_t c0 = codes & 7u;
        float t0;
        // kmax < 2^31 (a key of a t in [tmin, FLT_MAX]): a candidate whose key or rejection word has
        // the sign bit set is never <= kmax
        if (c0 >= 4u) {
          const u32x8 a = first ? u32x8{sw[4], sw[5], sw[6], sw[7], sw[8], sw[9], sw[10], sw[11]} : sld8(recs, boff);
          float ra[8];
#pragma unroll
          for (int j = 0; j < 8; j++) ra[j] = uf(a[j]);
          const uint32_t rej = quad_aa_k(c0 - 4u, ra, o, d, inv, t0);  // sign bit set: no candidate
          // kt with the rejection's sign bit: <= kmax (< 2^31) exactly for an accepted candidate
          const uint32_t x = (bits(t0) - bits(tmin)) | (rej & 0x80000000u);
          if (x <= kmax) prim = vref;
          kmax = min(kmax, x);
        } else {
          u32x16 a;
          u32x4 b2;
          sld20(recs, boff, a, b2);
          float w0[20];
#pragma unroll
          for (int j = 0; j < 16; j++) w0[j] = uf(a[j]);
#pragma unroll
          for (int j = 0; j < 4; j++) w0[16 + j] = uf(b2[j]);
          const bool ok0 = quad_cand_u(c0, w0, o, d, inv, t0);
          const uint32_t kt = bits(t0) - bits(tmin);
          if (ok0 && kt <= kmax) {
            kmax = kt;
            prim = vref ^ ((kQuadAA ^ kQuad) << 28);  // the QUAD layout's kind
          }
        }
        if (kStats) cnt.quad += 1;
#if RT2_EXP_TWICE & 16
        {
          f3 o2 = o;
          asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
          float t2 = 0.0f;
          bool ok2 = false;
          if (c0 >= 4u) {
            const u32x8 a = sld8(recs, boff);
            float ra[8];
#pragma unroll
            for (int j = 0; j < 8; j++) ra[j] = uf(a[j]);
            ok2 = (int)quad_aa_k(c0 - 4u, ra, o2, d, inv, t2) >= 0;
          }
          asm volatile("" ::"v"(t2), "v"((int)ok2));
        }
#endif
        codes >>= 3;
        if (codes == 1u) break;
        boff += 16u * (uint32_t)kQuadRecords;
        vref += (uint32_t)kQuadRecords;
      }
      tmax = uf(kmax + bits(tmin));
      }  // !boxed
      next = at + run;
    } else if (Has<F, kFeatSphere>() && kind == kSphere) {
      float t;
      uint32_t ref = make_ref(kind, off);
      // the sphere record (c0, r | disp, mat) is the step's inline words: no load
      if (kStats) cnt.sphere++;
      const bool hs = sphere_t_rec<0, Has<F, kFeatMotion>()>(make_float4(uf(sw[4]), uf(sw[5]), uf(sw[6]), uf(sw[7])),
                                   make_float4(uf(sw[8]), uf(sw[9]), uf(sw[10]), uf(sw[11])), o, d, time, tmin, tmax, t);
      if (hs) {
        tmax = t;
        prim = ref;
        h.xf = cur_xf;
      }
    } else if (Has<F, kFeatXform>() && kind == kXform) {
      if (kStats) cnt.xform++;
      const u32x16 m = sld16(recs, off * 16u);  // inverse-model columns
      f3 no, nd;
      if (m[11] == kXformYAxis) {
        // a transform about y (compile.cpp YAxisPattern): the products of the +-0 entries col0.y,
        // col1.x, col1.z, col2.y are left out of the sums below (DESIGN.md §4 "Transforms about y")
        no = mk(uf(m[0]) * o.x + (uf(m[8]) * o.z + uf(m[12])), uf(m[5]) * o.y + uf(m[13]),
                uf(m[2]) * o.x + (uf(m[10]) * o.z + uf(m[14])));
        nd = mk(uf(m[0]) * d.x + uf(m[8]) * d.z, uf(m[5]) * d.y, uf(m[2]) * d.x + uf(m[10]) * d.z);
      } else {
        no = mk((uf(m[0]) * o.x + uf(m[4]) * o.y) + (uf(m[8]) * o.z + uf(m[12])),
                (uf(m[1]) * o.x + uf(m[5]) * o.y) + (uf(m[9]) * o.z + uf(m[13])),
                (uf(m[2]) * o.x + uf(m[6]) * o.y) + (uf(m[10]) * o.z + uf(m[14])));
        nd = mk(uf(m[0]) * d.x + uf(m[4]) * d.y + uf(m[8]) * d.z, uf(m[1]) * d.x + uf(m[5]) * d.y + uf(m[9]) * d.z,
                uf(m[2]) * d.x + uf(m[6]) * d.y + uf(m[10]) * d.z);
      }
      o = no;
      normalize_recip3(nd, d, inv, fin);
#if RT2_EXP_TWICE & 2048
      {
        f3 o2 = o;
        asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
        f3 n2, e2;
        if (m[11] == kXformYAxis) {
          n2 = mk(uf(m[0]) * o2.x + (uf(m[8]) * o2.z + uf(m[12])), uf(m[5]) * o2.y + uf(m[13]),
                  uf(m[2]) * o2.x + (uf(m[10]) * o2.z + uf(m[14])));
          e2 = mk(uf(m[0]) * o2.x + uf(m[8]) * o2.z, uf(m[5]) * o2.y, uf(m[2]) * o2.x + uf(m[10]) * o2.z);
        } else {
          n2 = mk((uf(m[0]) * o2.x + uf(m[4]) * o2.y) + (uf(m[8]) * o2.z + uf(m[12])),
                  (uf(m[1]) * o2.x + uf(m[5]) * o2.y) + (uf(m[9]) * o2.z + uf(m[13])),
                  (uf(m[2]) * o2.x + uf(m[6]) * o2.y) + (uf(m[10]) * o2.z + uf(m[14])));
          e2 = mk(uf(m[0]) * o2.x + uf(m[4]) * o2.y + uf(m[8]) * o2.z, uf(m[1]) * o2.x + uf(m[5]) * o2.y + uf(m[9]) * o2.z,
                  uf(m[2]) * o2.x + uf(m[6]) * o2.y + uf(m[10]) * o2.z);
        }
        f3 d2, i2;
        bool f2;
        normalize_recip3(e2, d2, i2, f2);
        asm volatile("" ::"v"(n2.x), "v"(n2.y), "v"(n2.z), "v"(i2.x), "v"(i2.y), "v"(i2.z), "v"((int)f2));
      }
#endif
      cur_xf = make_ref(kXform, off);
    } else if (Has<F, kFeatXform>() && kind == kXformExit) {
      // kept model-space ray (xray planes, flat transforms): the closest primitive so far lies under
      // this transform (its record in [off + 8, skip)), so this space's ray is what resolve_hit needs
      if (xray != nullptr && P.flat_xforms != 0u && prim - make_ref(prim >> 28, off + (uint32_t)kXformRecords) <
                                                       st.y - (off + (uint32_t)kXformRecords)) {
        pk_st3(xray, 0u, o);
        pk_st3(xray, 3u, d);
      }
      cur_xf = st.w;
      if (cur_xf == kRefNone) {
        o = wray.wo();
        d = wray.wd();
        if constexpr (kKeepW) {
          inv = winv;
          fin = wfin;
        } else {
          inv = recip3(d);
          fin = finite3(inv);
        }
      } else {
        ray_in_space(N, cur_xf, wray.wo(), wray.wd(), o, d);
        inv = recip3(d);
        fin = finite3(inv);
      }
    } else if (Has<F, kFeatAccList>() && kind == kListAcc) {
      const u32x16& aw = sw;
      // an accelerated HittableList (rt2_layout.h LISTACC): this ray's box padding; its tree's
      // steps follow in pre-order, near child first
      if (kStats) cnt.list++;
      const f3 dc = o - mk(uf(aw[4]), uf(aw[5]), uf(aw[6]));
      const float L = sqrtf(dot(dc, dc)) * 1.0001f + uf(aw[7]);
      // The walk's padded slab bound is fma(bound - o, inv, -+pad inv), one rounding per bound. An
      // infinite inv (a direction component exactly 0) would give NaN or -inf there and cull a box
      // the ray passes inside the padding; the walk takes +-2^100 for it instead (acc_slab_inv,
      // rt2_layout.h: conservative), and the exact inv is restored after the walk.
      const bool clamp = !__all(fin);  // wave-uniform, rare
      if (clamp) inv = mk(acc_slab_inv(inv.x), acc_slab_inv(inv.y), acc_slab_inv(inv.z));
      acc_pinv = ((uf(aw[8]) * L + uf(aw[9])) * L + uf(aw[10])) * inv;  // inv: the list's space
      acc_best = kRefNone;
      // The tree's steps (at + 1 .. skip) are walked lane by lane: each lane follows its own
      // pre-order path (skip on a miss, paired child boxes), the steps a lockstep walk would have
      // taken for it, in the same order (the same tests, the same hit), so the wave pays its
      // longest lane's walk instead of the union of its lanes' walks (rays enter the list from
      // every direction: book 2 +30 %). Steps come by vector loads of the wide program (64 B each;
      // the tree is L2-resident).
      {
        const uint32_t end = st.y;
        const uint4* wide = reinterpret_cast<const uint4*>(P.lin_wide);
        uint32_t j = at + 1u;
        // eight copies of the tree (compile.cpp): the one ordered nearer-first for this ray's octant
        if (end - j > st.w) j += st.w * ((d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u));
        const uint32_t stop = j + st.w;
#if RT2_EXP_TWICE & 4096
        {  // cost probe: the same walk on copies of the lane's state, result discarded
          f3 o2 = o;
          asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
          float tmax2 = tmax;
          uint32_t prim2 = prim, best2 = acc_best, j2 = j;
          while (j2 < stop) {
            const uint4 e0 = wide[4u * j2], e1 = wide[4u * j2 + 1u], e2 = wide[4u * j2 + 2u], e3 = wide[4u * j2 + 3u];
            if (e0.x == kAccBvh) {
              const bool in = acc_slab(mk(uf(e1.x), uf(e1.y), uf(e1.z)), mk(uf(e2.x), uf(e2.y), uf(e2.z)), o2, inv,
                                       acc_pinv, tmin, tmax2);
              uint32_t nx = in ? j2 + 1u : e0.y;
              if (e0.z != j2 + 1u) {
                const bool in2 = acc_slab(mk(uf(e1.w), uf(e2.w), uf(e3.x)), mk(uf(e3.y), uf(e3.z), uf(e3.w)), o2, inv,
                                          acc_pinv, tmin, tmax2);
                nx = in ? (in2 ? e0.z : e0.w) : e0.y;
              }
              j2 = nx;
            } else {
              float t;
              if (sphere_t_rec<0, Has<F, kFeatMotion>()>(make_float4(uf(e1.x), uf(e1.y), uf(e1.z), uf(e1.w)),
                                                         make_float4(uf(e2.x), uf(e2.y), uf(e2.z), uf(e2.w)), o2, d,
                                                         time, tmin, FLT_MAX, t) &&
                  (t < tmax2 || (t == tmax2 && best2 != kRefNone && e0.w < best2))) {
                tmax2 = t;
                prim2 = make_ref(kSphere, e0.z);
                best2 = e0.w;
              }
              j2++;
            }
          }
          asm volatile("" ::"v"(tmax2), "v"(prim2), "v"(best2));
        }
#endif
        while (j < stop) {
          // e0 = (kind, skip, after a hit, after a paired miss), e1..e3 = words 4..15
          const uint4 e0 = wide[4u * j], e1 = wide[4u * j + 1u], e2 = wide[4u * j + 2u], e3 = wide[4u * j + 3u];
          if (e0.x == kAccBvh) {
            if (kStats) cnt.bvh++;
            const bool in = acc_slab(mk(uf(e1.x), uf(e1.y), uf(e1.z)), mk(uf(e2.x), uf(e2.y), uf(e2.z)), o, inv,
                                     acc_pinv, tmin, tmax);
            uint32_t nx = in ? j + 1u : e0.y;
            if (e0.z != j + 1u) {  // paired with its near child (words 7, 11-15)
              const bool in2 = acc_slab(mk(uf(e1.w), uf(e2.w), uf(e3.x)), mk(uf(e3.y), uf(e3.z), uf(e3.w)), o, inv,
                                        acc_pinv, tmin, tmax);
              if (kStats && in) cnt.bvh++;
              nx = in ? (in2 ? e0.z : e0.w) : e0.y;
            }
            j = nx;
          } else {  // ACCSPHERE: the record's words inline, aux = list position
            if (kStats) cnt.sphere++;
            float t;
            if (sphere_t_rec<0, Has<F, kFeatMotion>()>(make_float4(uf(e1.x), uf(e1.y), uf(e1.z), uf(e1.w)),
                             make_float4(uf(e2.x), uf(e2.y), uf(e2.z), uf(e2.w)), o, d, time, tmin, FLT_MAX, t) &&
                (t < tmax || (t == tmax && acc_best != kRefNone && e0.w < acc_best))) {
              tmax = t;
              prim = make_ref(kSphere, e0.z);
              h.xf = cur_xf;
              acc_best = e0.w;
            }
            j++;
          }
        }
        next = end;
        if (clamp) inv = recip3(d);
      }
    } else if (Has<F, kFeatMedium>() && kind == kMedium) {
      if (kStats) cnt.medium++;
      float t;
      const u32x4 mr = {sw[4], sw[5], sw[6], sw[7]};  // the medium record, inline
#if RT2_EXP_TWICE & 32
      if constexpr (!G::kLds) {
        f3 o2 = o;
        asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
        G p2 = path;
        Counters c2 = cnt;
        float t2 = 0.0f;
        const bool h2 = medium_t_lin<F>(recs, off, mr, o2, d, inv, time, tmin, tmax, p2, cand, t2, c2);
        asm volatile("" ::"v"(t2), "v"((int)h2));
      }
#endif
      if (medium_t_lin<F>(recs, off, mr, o, d, inv, time, tmin, tmax, path, cand, t, cnt)) {
        tmax = t;
        prim = make_ref(kMedium, off);
        h.xf = cur_xf;
      }
    }
    }  // next == at
    i = wave_min_next(next);
  }
  h.t = tmax;
  h.prim = prim;
  if constexpr (Has<F, kFeatXform>()) {
    if (prim != kRefNone && (prim >> 28) == kQuad) h.xf = N.word((prim & kOffsetMask) + 3u, 3);
    if (prim != kRefNone && (prim >> 28) == kQuadAA) h.xf = N.word((prim & kOffsetMask) + 4u, 1);
  }
  return prim != kRefNone;
}

// The closest hit's record in world space (what the reference's rec holds after the chain of
// TransformedHittable::Hit returns): point, normal, front_face, material.
template <uint32_t F, int kMode>
__device__ __forceinline__ void resolve_hit(const Nodes<kMode>& N, const HitRef& h, f3 wo, f3 wd, float time, f3& p,
                                            f3& n, bool& front, uint32_t& mat, const lds_u32* xray = nullptr,
                                            bool flat = false) {
  f3 o = wo, d = wd;
  if constexpr (Has<F, kFeatXform>()) {
    if (xray != nullptr && flat && h.xf != kRefNone) {  // the trace kept the hit's model-space ray
      o = pk_ld3(xray, 0u);
      d = pk_ld3(xray, 3u);
    } else {
      ray_in_space(N, h.xf, wo, wd, o, d);
    }
  }
  uint32_t kind = h.prim >> 28, off = h.prim & kOffsetMask;
  bool wnormal = false;  // n is already the world normal (QUADAA under transforms)
  p = o + d * h.t;
  if (Has<F, kFeatMedium>() && kind == kMedium) {
    n = mk(1.0f, 0.0f, 0.0f);
    front = true;
    mat = N.word(off, 1);
  } else if (Has<F, kFeatSphere>() && kind == kSphere) {
    float4 r0 = N[off], r1 = N[off + 1];
    const f3 center = Has<F, kFeatMotion>() ? xyz(r0) + xyz(r1) * time : xyz(r0);
    f3 outward = (p - center) / r0.w;
    front = dot(d, outward) < 0.0f;
    n = front ? outward : -outward;
    mat = bits(r1.w);
  } else if (kMode == kModeLinear && kind == kQuadAA) {
    f3 qn = xyz(N[off + 2]);
    front = dot(d, qn) < 0.0f;
    n = front ? qn : -qn;
    const float4 r3 = N[off + 3];
    mat = bits(r3.w);
    if (Has<F, kFeatXform>() && h.xf != kRefNone) {
      // the quad's world normal from the record (compile.cpp WorldNormal: the same operations as the
      // loop below on the same values); the loop then moves only the point
      const f3 wn = xyz(r3);
      n = front ? wn : -wn;
      wnormal = true;
    }
  } else {
    f3 qn = xyz(N[off]);
    front = dot(d, qn) < 0.0f;
    n = front ? qn : -qn;
    mat = N.word(off + 1, 3);
  }
  if constexpr (Has<F, kFeatXform>()) {
    // back through every enclosing transform, innermost first (Transform.cpp:85-86)
    for (uint32_t x = h.xf; x != kRefNone;) {
      uint32_t xo = x & kOffsetMask;
      // (the parent link with M: the loop's exit test does not wait on a load of its own)
      const float4 c1 = N[xo + 1];
      float4 m0 = N[xo + 4], m1 = N[xo + 5], m2 = N[xo + 6], m3 = N[xo + 7];
      // (c2.w: the transform's pattern in the threaded program's copy, 0 in the node array)
      if (kMode == kModeLinear && N.word(xo + 2, 3) == kXformYAxis) {  // M's +-0 products left out
        p = mk(m0.x * p.x + (m2.x * p.z + m3.x), m1.y * p.y + m3.y, m0.z * p.x + (m2.z * p.z + m3.z));
      } else {
        p = mk((m0.x * p.x + m1.x * p.y) + (m2.x * p.z + m3.x), (m0.y * p.x + m1.y * p.y) + (m2.y * p.z + m3.y),
               (m0.z * p.x + m1.z * p.y) + (m2.z * p.z + m3.z));
      }
      // (a medium's hit normal is never read: Isotropic::Scatter ignores it, Material.cpp:76-83)
      if (!(Has<F, kFeatMedium>() && kind == kMedium) && !wnormal) {
        const float4 c0 = N[xo], c2 = N[xo + 2];
        n = normalize(mk(c0.x * n.x + c0.y * n.y + c0.z * n.z, c1.x * n.x + c1.y * n.y + c1.z * n.z,
                         c2.x * n.x + c2.y * n.y + c2.z * n.z));
      }
      x = bits(c1.w);  // the parent transform
    }
  }
}

// ------------------------------------------------------------------------------------------
// Textures (Texture.cpp:7-22, PerlinNoiseGen.cpp:10-88)
__device__ __forceinline__ float perlin_noise(const ShadeArgs& S, uint32_t voff, uint32_t poff, uint32_t pc, f3 p) {
  const float4* V = S.perlin_vec + voff;
  const int* Px = S.perlin_perm + poff;
  const int* Py = Px + pc;
  const int* Pz = Py + pc;
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int i = (int)fx, j = (int)fy, k = (int)fz;
  float uu = u * u * (3.0f - 2.0f * u);
  float vv = v * v * (3.0f - 2.0f * v);
  float ww = w * w * (3.0f - 2.0f * w);
  float accum = 0.0f;
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++) {
        int idx = Px[(i + di) & 255] ^ Py[(j + dj) & 255] ^ Pz[(k + dk) & 255];
        f3 g = xyz(V[idx]);
        f3 wv = mk(u - (float)di, v - (float)dj, w - (float)dk);
        float fi = di ? uu : (1.0f - uu);
        float fj = dj ? vv : (1.0f - vv);
        float fk = dk ? ww : (1.0f - ww);
        accum += ((fi * fj) * fk) * dot(g, wv);
      }
  return accum;
}

template <uint32_t F>
__device__ __forceinline__ f3 tex_value(const ShadeArgs& S, uint32_t idx, f3 p) {
  const float4* T = S.textures;
  for (int guard = 0; guard < 32; guard++) {
    float4 t0 = T[3 * idx];
    uint32_t type = bits(t0.x);
    if (!(Has<F, kFeatChecker>() || Has<F, kFeatNoise>()) || type == kTexSolid) return mk(t0.y, t0.z, t0.w);
    float4 t1 = T[3 * idx + 1];
    if constexpr (Has<F, kFeatChecker>()) {
      if (type == kTexChecker) {
        f3 sp = t1.x * p;
        int ix = (int)floorf(sp.x), iy = (int)floorf(sp.y), iz = (int)floorf(sp.z);
        idx = ((ix + iy + iz) % 2 == 0) ? bits(t1.y) : bits(t1.z);
        continue;
      }
    }
    if constexpr (Has<F, kFeatNoise>()) {
      float4 t2 = T[3 * idx + 2];
      uint32_t voff = bits(t2.x), poff = bits(t2.y), pc = bits(t2.z);
      f3 alb = mk(t0.y, t0.z, t0.w) * 0.5f;
      if (bits(t1.w) == 1u) {  // NoiseType::kMarble: turbulence, 7 octaves
        float acc = 0.0f, weight = 1.0f;
        f3 tp = p;
        for (int k = 0; k < 7; k++) {
          acc += weight * perlin_noise(S, voff, poff, pc, tp);
          weight *= 0.5f;
          tp = tp * 2.0f;
        }
        float arg = t1.x * p.z + 10.0f * fabsf(acc);
        return alb * (1.0f + sin_f(arg));
      }
      return alb * (1.0f + perlin_noise(S, voff, poff, pc, t1.x * p));
    }
    break;
  }
  return mk(0.0f, 0.0f, 0.0f);  // checker cycle (the reference recurses forever)
}

// ------------------------------------------------------------------------------------------
// Camera::GetRay for global pixel (x, y) at the path's stratum
template <uint32_t F, class G>
__device__ __forceinline__ void camera_ray(const RenderParams& P, G& g, uint32_t x, uint32_t y, f3& o, f3& d,
                                           float& time) {
  const CameraParams& C = P.cam;
  const int s_i = (int)(g.sij & 0xFFFFu), s_j = (int)(g.sij >> 16);
  float u[3];
  bool defocus = Has<F, kFeatDefocus>() && !(C.defocus_angle <= 0.0f);
  if (defocus) {
    g.template take<2>(u);
  } else {
    g.template take<3>(u);  // px, py, time
  }
  // pixel00, du, dv, center (words 0-11) and recip_sqrt_spp (word 19) from the argument segment
  constexpr uint32_t kCam = (uint32_t)offsetof(RenderParams, cam);
  static_assert(offsetof(CameraParams, recip_sqrt_spp) == 19 * 4, "CameraParams layout");
  const u32x16 ca = karg16<kCam>();
  const u32x8 cb = karg8<kCam + 48u>();  // words 12-19
  const float rs = uf(cb[7]);
  f3 p00 = mk(uf(ca[0]), uf(ca[1]), uf(ca[2]));
  f3 du = mk(uf(ca[3]), uf(ca[4]), uf(ca[5]));
  f3 dv = mk(uf(ca[6]), uf(ca[7]), uf(ca[8]));
  f3 c = mk(uf(ca[9]), uf(ca[10]), uf(ca[11]));
  float px = ((float)s_i + u[0]) * rs - 0.5f;
  float py = ((float)s_j + u[1]) * rs - 0.5f;
  f3 pc = (p00 + (((float)x + px) * du)) + (((float)y + py) * dv);
  if constexpr (Has<F, kFeatDefocus>()) {
    if (defocus) {
      // RandInUnitDisk (uniform in the unit disk) by the inverse-CDF map r = sqrt(u), phi = 2 pi v
      float w[2];
      g.template take<2>(w);
      const float rr = sqrt_nr(w[0]);  // (every 24-bit uniform: rt2_selftest which 9)
      float cd, sd;
      cos_sin_2pi(w[1], cd, sd);
      const float dx = rr * cd, dy = rr * sd;
      c = (c + (dx * mk(C.defocus_u[0], C.defocus_u[1], C.defocus_u[2]))) +
          (dy * mk(C.defocus_v[0], C.defocus_v[1], C.defocus_v[2]));
      u[2] = g.uniform();
    }
  }
  time = u[2];
  o = c;
  d = normalize(pc - c);
}

// Global pixel index -> (x, y) by the host's multiplier for the width (rt2_layout.h Magic; the
// index is below 2^31, capi.cpp OnResize)
__device__ __forceinline__ void pix_xy(const LoopArgs& A, uint32_t pix, uint32_t& x, uint32_t& y) {
  const unsigned long long dw = karg2<RT2_KOFF(div_width)>();
  y = udiv(pix, Magic{(uint32_t)dw, (uint32_t)(dw >> 32)});
  x = pix - y * (uint32_t)A.width();
}
// Local (row-band) pixel index of global pixel (x, y): global row y lies in band y / band_h of period
// y / (band_h * world) and is stored as local row (y / (band_h * world)) * band_h + y % band_h
// (rt2_layout.h BandRank). One GPU: the global index.
__device__ __forceinline__ uint32_t local_index(const LoopArgs& A, uint32_t x, uint32_t y) {
  const uint32_t bh = (uint32_t)A.band_h();
  const uint32_t r = udiv(y, A.div_band_w()) * bh + (y - udiv(y, A.div_band_h()) * bh);
  return r * (uint32_t)A.width() + x;
}

// Occupancy target (waves per SIMD the register allocation must allow), chosen per variant by
// measurement (threaded kernels): Cornell 8 (7: -3 %), Cornell volume 8 (round 3, with box boundaries
// as one block: 7 / 8 waves 19.9 k / 20.6 k Mray/s), book 1 8, book 2 8 (6 / 7: -11 / -5 %; spills
// VGPRs, but its scalar loads are latency bound), the book 2 / all-features stack kernels 6. Other
// stack and the counting kernels keep the compiler's own allocation.
template <uint32_t F, int kMode, bool kStats>
constexpr int MinWaves() {
  if (RT2_MIN_WAVES_PER_EU > 0) return RT2_MIN_WAVES_PER_EU;
  constexpr uint32_t kBook2 = kFeatSphere | kFeatMedium | kFeatXform | kFeatNoise | kFeatSpecular | kFeatAccList | kFeatMotion;
  if ((F == kFeatAll || F == kBook2) && !kStats && (kMode == kModeStackGlobal || kMode == kModeStackHybrid))
    return RT2_MIN_WAVES_ALL;  // book 2
  if (F == kBook2 && !kStats && kMode == kModeLinear) return RT2_MIN_WAVES_B2LIN;
  if (kStats || kMode != kModeLinear) return 1;
  if (F == kFeatXform) return RT2_MIN_WAVES_CORNELL;  // Cornell: 64 VGPRs at 8
  if (F == (kFeatXform | kFeatMedium)) return RT2_MIN_WAVES_VOL;  // Cornell volume
  if (F == kFeatAll) return 1;
  return RT2_MIN_WAVES_BOOK1;                     // book 1
}

// Samples staged in LDS (rt2_layout.h kOctet): a lane keeps the first samples of a group of
// consecutive frames in LDS planes and writes the group with 16-B stores when its last sample is
// done; a chunk edge inside a group writes its samples one by one. Groups of 8 (an octet: 96 B,
// three whole 32-B sectors; 5.25 KB of LDS per wave, so at most 7 waves per SIMD) or, for kernels
// at 8 waves, of 4 (48 B; 2.25 KB per wave; the middle sector of an octet is written in two halves,
// 4/3 of the sample bytes reach memory). Returns the group size, 0 = direct 12-B stores.
// The threaded product kernels at 8 waves per SIMD keep the Philox block in LDS (PathT; 1 KB per
// wave): four VGPRs fewer live across the loop, which removed the Cornell kernel's spills at 8
// waves (12 VGPRs; +1 %). Kernels at 7 waves or fewer keep it in VGPRs and stage whole sample
// octets instead.
template <uint32_t F, int kMode, bool kStats>
constexpr bool LdsRng() {
  return kMode == kModeLinear && !kStats && MinWaves<F, kMode, kStats>() >= 8;
}
// Book 2's threaded kernel parks the path state in LDS while a ray is traced (ParkedPath): its
// trace needs more registers than 8 waves per SIMD leave. Its samples are stored directly (12-B
// stores: staging measured no faster for it), which leaves the LDS room for the park planes.
template <uint32_t F, int kMode, bool kStats>
constexpr bool Park() {
  constexpr uint32_t kBook2 = kFeatSphere | kFeatMedium | kFeatXform | kFeatNoise | kFeatSpecular | kFeatAccList | kFeatMotion;
  return F == kBook2 && kMode == kModeLinear && !kStats && LdsRng<F, kMode, kStats>();
}
// Kernels whose threaded medium step takes both box-boundary queries in one pass (boundary_aa_pair):
// their LDS holds the candidates.
template <uint32_t F, int kMode>
constexpr bool BoxPair() {
  return kMode == kModeLinear && Has<F, kFeatMedium>() && !Has<F, kFeatSphere>();
}

// Kernels with the two-block Philox ring (PathT kRing): 8 Philox planes, where the LDS room allows it (not
// beside the Cornell volume kernel's candidate planes or book 2's park planes).
template <uint32_t F, int kMode, bool kStats>
constexpr bool Ring() {
  return LdsRng<F, kMode, kStats>() && !Park<F, kMode, kStats>() && !BoxPair<F, kMode>();
}
template <uint32_t F, int kMode, bool kStats>
constexpr uint32_t StageGroup() {
  if (kMode != kModeLinear || kStats || Park<F, kMode, kStats>()) return 0u;
  // the ring kernels (Cornell, book 1) store samples directly: their staging logic cost more time than
  // the write traffic it saves (round 4, same box: C2 +0.9 %, book 1 +1 %; 12-B stores write the
  // octets' sectors partially, about 3x the sample bytes, 2.5 % of HBM bandwidth at the headline)
  if (Ring<F, kMode, kStats>()) return 0u;
  // octets need 5.25 KB per wave: with the LDS Philox blocks beside them they fit no occupancy >= 7
  return MinWaves<F, kMode, kStats>() <= 7 && !LdsRng<F, kMode, kStats>() ? 8u : 4u;
}

template <uint32_t F, int kMode, bool kStats>
__global__ __launch_bounds__(kBlock, (MinWaves<F, kMode, kStats>())) void render_kernel(const RenderParams P) {
  constexpr bool kLds = kMode == kModeStackLds || kMode == kModeStackHybrid;
  constexpr uint32_t kGroup = StageGroup<F, kMode, kStats>();
  constexpr uint32_t kPlanes = kGroup ? 3u * (kGroup - 1u) : 1u;  // [slot][component] planes of 64 lanes
  Nodes<kMode> N{reinterpret_cast<const float4*>(P.nodes), P.lds_nodes};
  if constexpr (kLds) {
    const float4* src = reinterpret_cast<const float4*>(P.nodes);
    for (uint32_t i = threadIdx.x; i < P.lds_nodes; i += kBlock) s_dyn[i] = src[i];
    __syncthreads();
  }
  uint32_t* stk = reinterpret_cast<uint32_t*>(s_dyn + (kLds ? P.lds_nodes : 0u)) + threadIdx.x;
  const int lane = (int)__lane_id();
  constexpr bool kLdsRng = LdsRng<F, kMode, kStats>();
  constexpr bool kPark = Park<F, kMode, kStats>();
  // the wave's LDS planes (lds_u32): Philox block, sample staging, box-boundary candidates, parked path
  constexpr uint32_t kRngP = 0u,
                     kOctP = kRngP + (kLdsRng ? (Ring<F, kMode, kStats>() ? 8u : 4u) : 0u),
                     kCandP = kOctP + (kGroup ? kPlanes : 0u);
  constexpr uint32_t kParkP = kCandP + (BoxPair<F, kMode>() ? kBoundaryAAMax : 0u);
  // the model-space ray of the transform holding the closest hit, kept by the trace for resolve_hit
  // (the ring kernels with transforms: the Cornell box)
  constexpr bool kXray = Ring<F, kMode, kStats>() && Has<F, kFeatXform>();
  constexpr uint32_t kXrayP = kParkP + (kPark ? (uint32_t)kParkWords : 0u);
  constexpr uint32_t kWavePlanes = kXrayP + (kXray ? 6u : 0u);
  lds_u32* lp = nullptr;  // this lane's word of plane 0
  if constexpr (kWavePlanes != 0u) {
    __shared__ uint32_t s_planes[(kBlock / 64) * kWavePlanes * 64];
    lp = (lds_u32*)(s_planes) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (kWavePlanes * 64u) + lane;
  }
  const f3 bg = mk(P.background[0], P.background[1], P.background[2]);
  bool need = true;   // lane wants a work item
  bool idle = false;  // no work left for this lane: it stays in the loop, masked, until the wave ends,
                      // so the loop head is a convergence point and wave totals stay in SGPRs
  unsigned long long rays = 0;  // rays cast by the wave (popcounts of a ballot at the loop head)
  uint32_t bnext = 0, bend = 0;  // the wave's reserved batch of work items (wave-uniform)
  uint32_t item_rays = 0;
  constexpr bool kRing = Ring<F, kMode, kStats>();  // two-block Philox ring
  PathT<kLdsRng, kRing, !Has<F, kFeatSphere>()> path;
  path.rb = lp + 64u * kRngP;
  lds_u32* pk = lp + 64u * kParkP;  // this lane's park planes (kPark)
  path.pix = 0;
  path.start(0);
  path.r0 = path.r1 = path.r2 = path.r3 = 0;
  f3 ro = mk(0, 0, 0), rd = mk(0, 0, 1), thr = mk(1, 1, 1);
  float rtime = 0.0f;
  // depth_left (RayColor's depth, bits 0-15) | frames of the lane's chunk after this one (bits 16-26)
  // | the lane's first octet slot in the current octet (bits 27-31, sample staging)
  uint32_t dl = 0;
  Counters cnt = {};
  bool overflow = false;
  // the launch's first-wave start (RenderParams::launch_clock; minimum as the maximum of complements)
  if (lane == 0 && P.launch_clock != nullptr) atomicMax(P.launch_clock, ~__builtin_amdgcn_s_memrealtime());
#if RT2_EXP_ENDTIME
  const unsigned long long et_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long et_idle = 0;  // first loop head at which a lane of this wave found no work
#endif

#if RT2_EXP_STAMPS
  unsigned long long st_fetch = 0, st_trace = 0, st_shade = 0, st_finish = 0, st_t;
#define RT2_STAMP(acc)                                   \
  do {                                                   \
    unsigned long long _n = __builtin_amdgcn_s_memtime(); \
    acc += _n - st_t;                                    \
    st_t = _n;                                           \
  } while (0)
#else
#define RT2_STAMP(acc) \
  do {                 \
  } while (0)
#endif
  while (true) {
#if RT2_EXP_STAMPS
    st_t = __builtin_amdgcn_s_memtime();
#endif
    // ---- hand out work items. A wave reserves a batch [bnext, bend) with one atomic and its
    // lanes take items from it as they finish (popcount prefix); the batch size shrinks with the
    // work left (guided self-scheduling), so the counter sees few atomics early and the last
    // items still spread over all waves.
    unsigned long long mask = __ballot(need && !idle);
    // a lane of this wave found the items exhausted (handed out in order: none are left); the
    // others stop asking (no more atomics on the work counter in the launch's tail)
    if (mask != 0ull && __ballot(idle) != 0ull) {
      if (need) idle = true;
    } else if (mask != 0ull) {
      const LoopArgs A = loop_args();
      const uint32_t max_depth = (uint32_t)A.max_depth();  // <= 0xFFFF (rt2_tracer_set_max_depth)
      const uint32_t count = (uint32_t)__popcll(mask);
      const uint32_t avail = bend - bnext;
      const uint32_t old = bnext;
      uint32_t fresh = 0;
      if (count > avail) {
        const uint32_t want = count - avail;
        // work left as of this wave's last reservation (stale, so an overestimate)
        const uint32_t left = A.n_items() > bend ? A.n_items() - bend : 0u;
        const uint32_t size = max(want, min(A.batch_max(), left / A.batch_div()));
        uint32_t b = 0;
        if (lane == __builtin_amdgcn_readfirstlane(lane)) b = atomicAdd(P.work_counter, size);
        fresh = __builtin_amdgcn_readfirstlane(b);
        bnext = fresh + want;
        bend = fresh + size;
      } else {
        bnext = old + count;
      }
      if (need && !idle) {
        // lanes of `mask` below this one (v_mbcnt: no lane mask held in registers)
        const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        const uint32_t item = k < avail ? old + k : fresh + (k - avail);
        // (no `continue` here: every lane reaches the loop-head ballots below)
        if (item >= A.n_items()) {
          idle = true;  // no work left for this lane
        } else {
          uint32_t chunk;
          int x, r;
          static_assert(RT2_KOFF(frame_tile) == RT2_KOFF(frame_tiles) + 4 &&
                            RT2_KOFF(div_frame_tile) == RT2_KOFF(frame_tiles) + 8, "RenderParams layout");
          const u32x4 ft = karg4<RT2_KOFF(frame_tiles)>();  // frame_tiles, frame_tile, div_frame_tile
          if (ft[0] != 0u) {  // frame tiles: one pixel x 64 consecutive one-frame chunks per 64 items
            const unsigned long long dw = karg2<RT2_KOFF(div_width)>();
            const uint32_t g = udiv(item, Magic{ft[2], ft[3]});
            const uint32_t rem = item - g * ft[1];
            const uint32_t pix = rem >> 6;
            chunk = g * 64u + (rem & 63u);
            r = (int)udiv(pix, Magic{(uint32_t)dw, (uint32_t)(dw >> 32)});
            x = (int)(pix - (uint32_t)r * (uint32_t)A.width());
          } else {
            chunk = udiv(item, A.div_tile_items());  // chunk-major: every tile's chunk 0 first
            const uint32_t titem = item - chunk * A.tile_items();
            const uint32_t tile = titem >> 6, within = titem & 63u;
            const uint32_t trow = udiv(tile, A.div_tiles_x());
            // tiles of (64 >> tile_shift) local rows x (1 << tile_shift) pixels
            const uint32_t tsh = A.tile_shift(), tw = 1u << tsh;
            x = (int)((tile - trow * (uint32_t)A.tiles_x()) * tw + (within & (tw - 1u)));
            r = (int)(trow * (64u >> tsh) + (within >> tsh));
          }
          // the chunk's first frame and its stratum (RayTracer.cpp:59-60, from the host's table),
          // and the next chunk's first frame (<= first + kChunkMaxFrames)
          const uint32_t* ce = A.chunks() + 2u * chunk;
          const int f = (int)ce[0];
          const int fstop = (int)ce[2];
          // else: a lane of a partial edge tile, or a padding chunk of the frame tiles
          if (x < A.width() && r < A.local_rows() && f < A.frame_begin() + A.n_frames()) {
            uint32_t y = (uint32_t)r;
            const uint32_t world = (uint32_t)A.world();
            if (world > 1u) {  // local row -> global row (rt2_layout.h BandRank)
              const uint32_t bh = (uint32_t)A.band_h(), rank = (uint32_t)A.rank();
              const uint32_t per = udiv((uint32_t)r, A.div_band_h());  // the rank's band in period `per`
              const uint32_t pm = per - udiv(per, A.div_world()) * world;
              const uint32_t phase = rank >= pm ? rank - pm : rank + world - pm;
              y = (per * world + phase) * bh + ((uint32_t)r - per * bh);
            }
            path.pix = y * (uint32_t)A.width() + (uint32_t)x;
            item_rays = 0;
            need = false;
            path.start((uint32_t)f);
            path.sij = ce[1];  // then advanced per frame below
            camera_ray<F>(P, path, (uint32_t)x, y, ro, rd, rtime);
            thr = mk(1, 1, 1);
            const uint32_t s0 = (uint32_t)(f - A.frame_begin()) & (kOctet - 1u);
            dl = max_depth | ((uint32_t)(fstop - f - 1) << 16) | (s0 << 27);
          }
        }
      }
    }
#if RT2_EXP_ENDTIME
    if (et_idle == 0ull && __ballot(idle) != 0ull) et_idle = __builtin_amdgcn_s_memrealtime();
#endif
    if (__ballot(!idle) == 0ull) break;  // the wave is done (uniform exit)
    rays += (unsigned long long)__popcll(__ballot(!need && (dl & 0xFFFFu) != 0u));  // RayColor casts below
    if (need) continue;
    RT2_STAMP(st_fetch);

    // ---- one bounce (RayColor, RayTracer.cpp:20-45)
    bool done = false;
    f3 color = mk(0, 0, 0);
    HitRef h;
    bool hit = false;
    // the closest hit's record and material, then its emission or scatter (RayColor,
    // RayTracer.cpp:26-44)
    auto resolve = [&](const ShadeArgs& S) {
        f3 hp, hn;
        bool front;
        uint32_t mat;
        if constexpr (kMode == kModeLinear) {
          resolve_hit<F>(Nodes<kModeLinear>{reinterpret_cast<const float4*>(P.lind)}, h, ro, rd, rtime, hp, hn, front,
                         mat, kXray ? lp + 64u * kXrayP : nullptr, kXray && P.flat_xforms != 0u);
#if RT2_EXP_TWICE & 1
          {
            f3 ro2 = ro, hp2, hn2;
            bool fr2;
            uint32_t m2;
            asm volatile("" : "+v"(ro2.x), "+v"(ro2.y), "+v"(ro2.z));
            resolve_hit<F>(Nodes<kModeLinear>{reinterpret_cast<const float4*>(P.lind)}, h, ro2, rd, rtime, hp2, hn2,
                           fr2, m2);
            asm volatile("" ::"v"(hp2.x), "v"(hp2.y), "v"(hp2.z), "v"(hn2.x), "v"(hn2.y), "v"(hn2.z), "v"(m2),
                         "v"((int)fr2));
          }
#endif
        } else {
          resolve_hit<F>(N, h, ro, rd, rtime, hp, hn, front, mat);
        }
        const float4 m0 = S.materials[2 * mat], m1 = S.materials[2 * mat + 1];
        return HitShade{hp, hn, front, m0, m1, bits(m0.x)};
    };
    auto shade = [&](const HitShade& hs, const ShadeArgs& S) {
        const f3 hp = hs.hp, hn = hs.hn;
        const bool front = hs.front;
        const float4 m0 = hs.m0, m1 = hs.m1;
        const uint32_t type = hs.type;
        if (type == kMatDiffuseLight) {
          color = thr * tex_value<F>(S, bits(m1.z), hp);
          done = true;
        } else {
          f3 att, dir;
          bool dielectric = Has<F, kFeatSpecular>() && type == kMatDielectric;
          f3 ru = mk(0.0f, 0.0f, 0.0f);
          if (!dielectric) ru = rand_unit_vec3(path);  // one sampling site for every other material
#if RT2_EXP_TWICE & 2
          {
            auto p2 = path;
            asm volatile("" : "+v"(p2.n), "+v"(p2.frame));
            f3 r2 = rand_unit_vec3(p2);
            asm volatile("" ::"v"(r2.x), "v"(r2.y), "v"(r2.z));
          }
#endif
          if (Has<F, kFeatSpecular>() && type == kMatMetal) {
            dir = normalize(reflect(rd, hn)) + (m1.x * ru);
            att = mk(m0.y, m0.z, m0.w);
          } else if (dielectric) {
            att = mk(1.0f, 1.0f, 1.0f);
            float ri = front ? m1.w : m1.y;
            f3 ud = normalize(rd);
            float cos_t = gmin(dot(-ud, hn), 1.0f);
            float sin_t = sqrtf(1.0f - cos_t * cos_t);
            bool refl = ri * sin_t > 1.0f;
            if (!refl) {
              float r0 = (1.0f - ri) / (1.0f + ri);
              r0 = r0 * r0;
              double xx = (double)(1.0f - cos_t);
              double x2 = xx * xx;
              double x5 = (x2 * x2) * xx;
              double schlick = (double)r0 + (double)(1.0f - r0) * x5;
              refl = schlick > (double)path.uniform();
            }
            dir = refl ? reflect(ud, hn) : refract(ud, hn, ri);
          } else if (Has<F, kFeatMedium>() && type == kMatIsotropic) {
            dir = ru;
            att = tex_value<F>(S, bits(m1.z), hp);
          } else {  // Lambertian / Texture
            dir = hn + ru;
            if (near_zero(dir)) dir = hn;
            att = (type == kMatLambertian) ? mk(m0.y, m0.z, m0.w) : tex_value<F>(S, bits(m1.z), hp);
          }
          thr = thr * att;
          ro = hp;
          rd = dir;
          dl--;  // depth_left > 0 here: no borrow into the frame count
        }
    };
    if ((dl & 0xFFFFu) == 0u) {
      done = true;  // RayColor(depth <= 0) returns 0 without casting a ray
    } else {
      if constexpr (kStats) item_rays++;
      if constexpr (kPark) {
        pk_st3(pk, kPkThr, thr);
        pk_st(pk, kPkDl, dl);
        pk_st(pk, kPkSij, path.sij);
        pk_st(pk, kPkFrame, path.frame);
        pk_st(pk, kPkPix, path.pix);
        pk_st(pk, kPkN, path.n);
        pk_st3(pk, kPkO, ro);
        pk_st3(pk, kPkD, rd);
        ParkedPath pp{path.rb, pk};
        hit = trace_linear<F, kStats>(P, ParkRay{pk}, rtime, pp, h, lp + 64u * kCandP, nullptr, cnt);
        thr = pk_ld3(pk, kPkThr);
        dl = pk_ld(pk, kPkDl);
        path.sij = pk_ld(pk, kPkSij);
        path.frame = pk_ld(pk, kPkFrame);
        path.pix = pk_ld(pk, kPkPix);
        path.n = pk_ld(pk, kPkN);
        ro = pk_ld3(pk, kPkO);
        rd = pk_ld3(pk, kPkD);
      } else if constexpr (kMode == kModeLinear) {
        hit = trace_linear<F, kStats>(P, RegRay{ro, rd}, rtime, path, h, lp + 64u * kCandP,
                                      kXray ? lp + 64u * kXrayP : nullptr, cnt);
#if RT2_EXP_TRACE_TWICE
        {
          f3 ro2 = ro;
          asm volatile("" : "+v"(ro2.x), "+v"(ro2.y), "+v"(ro2.z));
          HitRef h2;
          auto p2 = path;
          bool hit2 = trace_linear<F, kStats>(P, RegRay{ro2, rd}, rtime, p2, h2, lp + 64u * kCandP, nullptr, cnt);
          asm volatile("" ::"v"(h2.t), "v"(h2.prim), "v"(h2.xf), "v"((int)hit2));
        }
#endif
      } else {
        hit = trace_stack<F, kMode, kStats>(P, N, ro, rd, rtime, path, h, stk, cnt, overflow);
      }
      RT2_STAMP(st_trace);
      if constexpr (!kRing) {
        if (!hit) {
          color = thr * bg;
          done = true;
        } else {
          const ShadeArgs S = shade_args();
          shade(resolve(S), S);
        }
      }
    }
    if constexpr (kRing) {
      // the hit lanes' records and materials first, so the bounce's one Philox site (PathT kRing)
      // knows which lanes scatter and which start their next frame
      HitShade hs{mk(0, 0, 0), mk(0, 0, 0), false, make_float4(0, 0, 0, 0), make_float4(0, 0, 0, 0),
                  kMatDiffuseLight};
      const ShadeArgs S = shade_args();
      if (hit) hs = resolve(S);
      const bool scatter = hit && hs.type != kMatDiffuseLight;
      path.prefetch(scatter, !scatter && ((dl >> 16) & kChunkLeftMask) != 0u);
      if (!done) {
        if (!hit) {
          color = thr * bg;
          done = true;
        } else {
          shade(hs, S);
        }
      }
    }
    RT2_STAMP(st_shade);
    if (done) {
      // this frame's sample, summed in frame order by accumulate_kernel (RayTracer.cpp:64)
      const LoopArgs A = loop_args();
      uint32_t px = 0, py = 0;
      pix_xy(A, path.pix, px, py);
      const uint32_t lidx = A.world() > 1 ? local_index(A, px, py) : path.pix;
      const uint32_t fr = path.frame - (uint32_t)A.frame_begin();  // launch-relative frame
      const uint32_t slot = fr & (kOctet - 1u);
      float* blk = A.samples() + 3ull * kOctet * ((unsigned long long)(fr / kOctet) * A.local_pixels() + lidx);
      const bool more = ((dl >> 16) & kChunkLeftMask) != 0u;  // frames of the chunk after this one
#if RT2_EXP_TWICE & 512
      for (int rep2 = 0; rep2 < 2; rep2++) {
        asm volatile("" : "+v"(color.x), "+v"(color.y), "+v"(color.z));
#endif
#if RT2_EXP_NOSTORE  // diagnostic (tools/c5_traffic.sh): no sample store, to attribute HBM writes
      if (false)
#endif
      if constexpr (kGroup != 0u) {
        lds_f32* oct = (lds_f32*)(lp + 64u * kOctP);
        const uint32_t gs = slot & (kGroup - 1u);  // slot within the group = LDS slot
        if (gs == kGroup - 1u || !more) {
          const uint32_t g0 = slot - gs;  // the group's first octet slot
          const uint32_t first = max(dl >> 27, g0) - g0;  // this lane's first LDS slot of the group
          if (first == 0u && gs == kGroup - 1u) {  // the whole group: 16-B stores
            float4* b4 = reinterpret_cast<float4*>(blk + 3u * g0);
#pragma unroll
            for (uint32_t j = 0; j + 1u < 3u * kGroup / 4u; j++)  // planes 4j..4j+3, few live registers
              b4[j] = make_float4(oct[64u * (4u * j)], oct[64u * (4u * j + 1u)], oct[64u * (4u * j + 2u)],
                                  oct[64u * (4u * j + 3u)]);
            b4[3u * kGroup / 4u - 1u] = make_float4(oct[64u * (kPlanes - 1u)], color.x, color.y, color.z);
          } else {  // a chunk edge inside the group: this lane's slots first..gs
            for (uint32_t k = first; k < gs; k++) {
              blk[3u * (g0 + k)] = oct[64u * (3u * k)];
              blk[3u * (g0 + k) + 1u] = oct[64u * (3u * k + 1u)];
              blk[3u * (g0 + k) + 2u] = oct[64u * (3u * k + 2u)];
            }
            blk[3u * slot] = color.x;
            blk[3u * slot + 1u] = color.y;
            blk[3u * slot + 2u] = color.z;
          }
        } else {
          oct[64u * (3u * gs)] = color.x;
          oct[64u * (3u * gs + 1u)] = color.y;
          oct[64u * (3u * gs + 2u)] = color.z;
        }
      } else {
        blk[3u * slot] = color.x;
        blk[3u * slot + 1u] = color.y;
        blk[3u * slot + 2u] = color.z;
      }
#if RT2_EXP_TWICE & 512
      }
#endif
      int f = (int)path.frame + 1;
      if (more) {
        if constexpr (kRing) {
          path.start_loaded((uint32_t)f);  // its block 0 came with the bounce's prefetch
        } else {
          path.start((uint32_t)f);
        }
        {  // next stratum: (f % sq, f / sq % sq) from the previous frame's
          const uint32_t sq = (uint32_t)P.cam.sqrt_spp;
          uint32_t si = (path.sij & 0xFFFFu) + 1u, sj = path.sij >> 16;
          if (si == sq) {
            si = 0u;
            sj = sj + 1u == sq ? 0u : sj + 1u;
          }
          path.sij = si | (sj << 16);
        }
#if RT2_EXP_TWICE & 4
        {
          auto p2 = path;
          f3 o2, d2;
          float t2;
          asm volatile("" : "+v"(p2.frame), "+v"(p2.sij));
          camera_ray<F>(P, p2, px, py, o2, d2, t2);
          asm volatile("" ::"v"(o2.x), "v"(d2.x), "v"(d2.y), "v"(d2.z), "v"(t2));
        }
#endif
        camera_ray<F>(P, path, px, py, ro, rd, rtime);
        thr = mk(1, 1, 1);
        // one frame fewer left; after the octet's last slot the next octet starts at slot 0
        dl = (((dl & 0x07FF0000u) - 0x10000u) | (uint32_t)A.max_depth()) | (slot == kOctet - 1u ? 0u : (dl & 0xF8000000u));
      } else {
        if (kStats && P.ray_counts) atomicAdd(P.ray_counts + lidx, item_rays);
        need = true;
      }
    }
    RT2_STAMP(st_finish);
  }

#if RT2_EXP_STAMPS
  if (lane == __builtin_amdgcn_readfirstlane(lane)) {
    atomicAdd(P.stats + StatsCounters::kStamps, st_fetch);
    atomicAdd(P.stats + StatsCounters::kStamps + 1, st_trace);
    atomicAdd(P.stats + StatsCounters::kStamps + 2, st_shade);
    atomicAdd(P.stats + StatsCounters::kStamps + 3, st_finish);
  }
#endif
  if (lane == 0) atomicAdd(P.stats + StatsCounters::kRays, rays);
  if (kStats) {
    atomicAdd(P.stats + StatsCounters::kBvhTests, (unsigned long long)cnt.bvh);
    atomicAdd(P.stats + StatsCounters::kQuadTests, (unsigned long long)cnt.quad);
    atomicAdd(P.stats + StatsCounters::kSphereTests, (unsigned long long)cnt.sphere);
    atomicAdd(P.stats + StatsCounters::kXformVisits, (unsigned long long)cnt.xform);
    atomicAdd(P.stats + StatsCounters::kMediumTests, (unsigned long long)cnt.medium);
    atomicAdd(P.stats + StatsCounters::kListVisits, (unsigned long long)cnt.list);
    if (BoxOn<F>()) {
      atomicAdd(P.stats + StatsCounters::kBoxTests, (unsigned long long)cnt.box);
      atomicAdd(P.stats + StatsCounters::kBoxCertified, (unsigned long long)cnt.box_cert);
      atomicAdd(P.stats + StatsCounters::kBoxWaveVisits, (unsigned long long)cnt.box_wave);
      atomicAdd(P.stats + StatsCounters::kBoxWaveRuns, (unsigned long long)cnt.box_wave_run);
    }
  }
  if (overflow) atomicAdd(P.stats + StatsCounters::kCount, 1ull);  // overflow flag slot
  // the launch's last-wave end
  if (lane == 0 && P.launch_clock != nullptr) atomicMax(P.launch_clock + 1, __builtin_amdgcn_s_memrealtime());
#if RT2_EXP_WAVESTEPS
  for (int k = 0; k < 8; k++) atomicAdd(P.stats + StatsCounters::kDiag + k, (unsigned long long)cnt.wd[k]);
#endif
#if RT2_EXP_ENDTIME
  if (lane == 0) {  // minima as maxima of complements (the slots start at 0); 100 MHz ticks
    const unsigned long long et_end = __builtin_amdgcn_s_memrealtime();
    unsigned long long* d = P.stats + StatsCounters::kDiag;
    atomicMax(d + 0, ~et_start);
    atomicMax(d + 1, et_start);
    atomicMax(d + 2, ~et_idle);
    atomicMax(d + 3, et_end);
    atomicAdd(d + 4, et_end - et_idle);
    atomicAdd(d + 5, et_end - et_start);
    atomicAdd(d + 6, 1ull);
    atomicMax(d + 7, et_idle);
  }
#endif
}

// ------------------------------------------------------------------------------------------
// RayTracer.cpp:64-66 for a launch's frames: accum[i] += sample(f) in frame order (the float sum
// of the reference's per-Update accumulation, bit for bit), then the live display value
// pixels[i] = ToColor(clamp(accum[i] / frame_idx, 0, 1)). One thread per local pixel reading its
// octets (96 contiguous bytes, six 16-B loads; neighbouring threads' octets are adjacent), so the
// kernel streams the sample buffer once at HBM rate.
__global__ __launch_bounds__(256) void accumulate_kernel(const float* __restrict__ samples, float* __restrict__ accum,
                                                         uint32_t* __restrict__ pixels, uint32_t npix, int n_frames,
                                                         int frame_idx) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= npix) return;
  float a0 = accum[3 * i], a1 = accum[3 * i + 1], a2 = accum[3 * i + 2];
  const float4* s = reinterpret_cast<const float4*>(samples) + 6ull * i;
  const unsigned long long stride = 6ull * npix;  // float4s per octet plane
  for (int f = 0; f < n_frames; f += (int)kOctet, s += stride) {
    float x[3 * kOctet];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const float4 q = s[j];
      x[4 * j] = q.x, x[4 * j + 1] = q.y, x[4 * j + 2] = q.z, x[4 * j + 3] = q.w;
    }
    const int m = n_frames - f < (int)kOctet ? n_frames - f : (int)kOctet;  // frames of this octet
#pragma unroll
    for (int k = 0; k < (int)kOctet; k++) {
      if (k < m) {
        a0 += x[3 * k];
        a1 += x[3 * k + 1];
        a2 += x[3 * k + 2];
      }
    }
  }
  accum[3 * i] = a0;
  accum[3 * i + 1] = a1;
  accum[3 * i + 2] = a2;
  if (pixels) {
    const float fi = (float)frame_idx;
    const float cc[3] = {a0 / fi, a1 / fi, a2 / fi};
    uint32_t rgba = 0xFF000000u;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float v = gmin(gmax(cc[k], 0.0f), 1.0f);
      rgba |= ((uint32_t)(uint8_t)floor((double)v * 255.999)) << (8 * k);
    }
    pixels[i] = rgba;
  }
}

// ------------------------------------------------------------------------------------------
// Instantiated feature sets (a launch picks the smallest superset of the scene's features).
constexpr uint32_t kVariants[] = {
    kFeatXform,                                   // Cornell box
    kFeatXform | kFeatMedium,                     // Cornell volume
    kFeatSphere | kFeatSpecular | kFeatDefocus,   // RTIOW book 1
    kFeatSphere | kFeatMedium | kFeatXform | kFeatNoise | kFeatSpecular | kFeatAccList | kFeatMotion,  // RTNW book 2
    kFeatAll,                                     // everything (scene graphs, checker textures)
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

using KernelFn = void (*)(RenderParams);

template <int V, int kMode>
KernelFn Pick(bool stats) {
  return stats ? reinterpret_cast<KernelFn>(&render_kernel<kVariants[V], kMode, true>)
               : reinterpret_cast<KernelFn>(&render_kernel<kVariants[V], kMode, false>);
}

template <int V>
KernelFn PickMode(int mode, bool stats) {
  switch (mode) {
    case kModeStackLds: return Pick<V, kModeStackLds>(stats);
    case kModeLinear: return Pick<V, kModeLinear>(stats);
    case kModeStackHybrid: return Pick<V, kModeStackHybrid>(stats);
    default: return Pick<V, kModeStackGlobal>(stats);
  }
}

KernelFn Kernel(int v, int mode, bool stats) {
#ifdef RT2_ONLY_VARIANT  // register-allocation experiments: one threaded product kernel only (not a usable build)
  (void)v, (void)mode, (void)stats;
  return reinterpret_cast<KernelFn>(&render_kernel<kVariants[RT2_ONLY_VARIANT], kModeLinear, false>);
#else
  switch (v) {
    case 0: return PickMode<0>(mode, stats);
    case 1: return PickMode<1>(mode, stats);
    case 2: return PickMode<2>(mode, stats);
    case 3: return PickMode<3>(mode, stats);
    case 4: return PickMode<4>(mode, stats);
  }
  return nullptr;
#endif
}

// ------------------------------------------------------------------------------------------
// Self-tests of the kernel's exact shortcuts on random inputs (rt2_selftest):
//   which 0: div_by_inv(a, b, fl(1/b)) == a / b for |b| > 1e-8, |a / b| >= 1e-3 (accepted quad t)
//   which 3: the same for any quotient with 2^-100 <= |a| < 2^21 (medium box boundaries, any t)
//   which 1: aabb_hit_fin == aabb_hit for rays with finite inv
//   which 2: rcp_nr == 1/x and sqrt_nr == sqrt(x) in their ranges
//   which 4: acc_slab (accelerated-list padded slab) never culls a box the exact padded slab accepts
//   which 5: rcp_nr == 1/x for every float in its range (exhaustive over the 2^32 bit patterns)
//   which 6: div_by_inv's single correction == a / b for every pair of significands (n = 2^46)
//   which 7: the same for every numerator significand against n / 2^23 divisor significands each
//   which 8: sphere_t_rec's fast roots (sphere_fast_ok) == IEEE division, cancelled numerators included
//   which 9: sqrt_nr == sqrt at the samplers' inputs for every 24-bit uniform (n = 2^24)
__device__ __forceinline__ float rand_float(uint32_t bits, int emin, int emax, uint32_t sel) {
  const int e = emin + (int)(sel % (uint32_t)(emax - emin + 1));
  return __uint_as_float((bits & 0x807FFFFFu) | ((uint32_t)(e + 127) << 23));
}
__global__ void selftest_kernel(int which, unsigned long long n, uint32_t seed, unsigned long long* out) {
  unsigned long long bad = 0, checked = 0;
  for (unsigned long long idx = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
       idx += (unsigned long long)gridDim.x * blockDim.x) {
    if (which == 6) {
      // every pair of significands (n = 2^46): a, b in [1, 2); div_by_inv against IEEE a / b (the
      // algorithm and the quotient scale exactly with the exponents)
      const float a = __uint_as_float(0x3F800000u | (uint32_t)(idx >> 23));
      const float b = __uint_as_float(0x3F800000u | ((uint32_t)idx & 0x7FFFFFu));
      checked++;
      if (__float_as_uint(div_by_inv(a, b, rcp_nr(b))) != __float_as_uint(a / b)) bad++;
      continue;
    }
    if (which == 9) {
      // every 24-bit uniform u (n = 2^24): sqrt_nr against IEEE sqrt at the samplers' two inputs,
      // 1 - z^2 with z = 1 - 2u (rand_unit_vec3) and u itself (the defocus disk's radius)
      if (idx >= (1ull << 24)) continue;
      const float u = to_unit((uint32_t)idx << 8);
      const float z = 1.0f - 2.0f * u, x = 1.0f - z * z;
      checked++;
      if (__float_as_uint(sqrt_nr(x)) != __float_as_uint(sqrtf(x)) ||
          __float_as_uint(sqrt_nr(u)) != __float_as_uint(sqrtf(u)))
        bad++;
      continue;
    }
    if (which == 7) {
      // every numerator significand (2^23 values of a in [1, 2)), each against n / 2^23 divisor
      // significands: b = 1, b = 2 - 2^-23 and a scrambled stride over the rest (neighbouring a values
      // see different divisors)
      const uint32_t sa = (uint32_t)idx & 0x7FFFFFu, j = (uint32_t)(idx >> 23);
      uint32_t sb = (sa * 0x9E3779B1u + j * 0x85EBCA77u) ^ (j * 0x2545F491u) ^ (sa >> 7);
      sb = j == 0u ? 0u : (j == 1u ? 0x7FFFFFu : sb & 0x7FFFFFu);
      const float a = __uint_as_float(0x3F800000u | sa), b = __uint_as_float(0x3F800000u | sb);
      checked++;
      if (__float_as_uint(div_by_inv(a, b, rcp_nr(b))) != __float_as_uint(a / b)) bad++;
      continue;
    }
    uint32_t r0, r1, r2, r3;
    philox(seed, 0x7E57u, (uint32_t)idx, (uint32_t)(idx >> 32), 0u, r0, r1, r2, r3);
    if (which == 3) {
      const float a = rand_float(r0, -100, 20, r2 & 0xFFFFu);
      const float b = rand_float(r1, -27, 1, r2 >> 16);
      const float q = a / b;
      if (!(fabsf(b) > 1e-8f) || !__builtin_isfinite(q)) continue;
      checked++;
      if (__float_as_uint(div_by_inv(a, b, 1.0f / b)) != __float_as_uint(q)) bad++;
    } else if (which == 0) {
      const float a = rand_float(r0, -30, 17, r2 & 0xFFFFu);
      const float b = rand_float(r1, -27, 1, r2 >> 16);
      const float q = a / b;
      if (!(fabsf(b) > 1e-8f) || !(fabsf(q) >= 1e-3f) || !__builtin_isfinite(q)) continue;
      checked++;
      const float inv = 1.0f / b;
      if (__float_as_uint(div_by_inv(a, b, inv)) != __float_as_uint(q)) bad++;
    } else if (which == 4) {
      // acc_slab never culls a box the exact padded slab test accepts; direction components are +-0
      // with probability 1/4 each (an infinite 1/d), origins often inside the padding band
      uint32_t s0, s1, s2, s3;
      philox(seed, 0xACC5u, (uint32_t)idx, (uint32_t)(idx >> 32), 1u, s0, s1, s2, s3);
      const float lo_x = rand_float(r0, -4, 9, r1), hi_x = lo_x + fabsf(rand_float(r1, -6, 8, r0 >> 7));
      const float lo_y = rand_float(r2, -4, 9, r3), hi_y = lo_y + fabsf(rand_float(r3, -6, 8, r2 >> 7));
      const float lo_z = rand_float(s0, -4, 9, s1), hi_z = lo_z + fabsf(rand_float(s1, -6, 8, s0 >> 7));
      const float pad = fabsf(rand_float(s2, -14, -6, s3));  // (the same test with 1/d = inf unclamped:
                                                             // 8 % of these inputs wrongly culled)
      // origin: inside the padding band of a face on about half the axes
      auto coord = [&](float lo, float hi, uint32_t r) {
        const uint32_t m = r & 3u;
        const float u = to_unit(r);
        if (m == 0u) return hi + pad * u;          // between hi and hi + pad
        if (m == 1u) return lo - pad * u;          // between lo - pad and lo
        return lo + (hi - lo) * 3.0f * (u - 0.33f);  // anywhere around the box
      };
      const f3 o = mk(coord(lo_x, hi_x, s3), coord(lo_y, hi_y, s2 ^ r3), coord(lo_z, hi_z, s1 ^ r2));
      f3 d = mk(rand_float(r0 ^ s0, -20, 1, r3), rand_float(r1 ^ s1, -20, 1, s3 >> 3), rand_float(r2 ^ s2, -20, 1, r0));
      const uint32_t zz = s0 >> 24;
      if ((zz & 3u) == 0u) d.x = (zz & 64u) ? -0.0f : 0.0f;
      if (((zz >> 2) & 3u) == 0u) d.y = (zz & 128u) ? -0.0f : 0.0f;
      if (((zz >> 4) & 3u) == 0u) d.z = (zz & 32u) ? -0.0f : 0.0f;
      const f3 inv0 = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
      const f3 inv = mk(acc_slab_inv(inv0.x), acc_slab_inv(inv0.y), acc_slab_inv(inv0.z));
      const f3 pinv = pad * inv;
      const float tmax = (s3 & 1u) ? FLT_MAX : rand_float(s0 ^ r3, -3, 12, s2);
      const bool got = acc_slab(mk(lo_x, lo_y, lo_z), mk(hi_x, hi_y, hi_z), o, inv, pinv, 0.001f, tmax);
      // exact padded slab in double, shrunk by a relative 1e-6 so that rounding at a face is not a miss
      double t0 = 0.001, t1 = (double)tmax;
      bool ref = true;
      const double los[3] = {lo_x, lo_y, lo_z}, his[3] = {hi_x, hi_y, hi_z}, os[3] = {o.x, o.y, o.z},
                   ds[3] = {d.x, d.y, d.z};
      for (int k = 0; k < 3; k++) {
        const double a = los[k] - pad, b = his[k] + pad, w = 1e-6 * (fabs(a) + fabs(b) + 1.0);
        if (ds[k] == 0.0) {
          ref = ref && (a + w < os[k] && os[k] < b - w);
        } else {
          double u0 = (a + w - os[k]) / ds[k], u1 = (b - w - os[k]) / ds[k];
          if (u0 > u1) { const double t = u0; u0 = u1; u1 = t; }
          t0 = t0 > u0 ? t0 : u0;
          t1 = t1 < u1 ? t1 : u1;
        }
      }
      ref = ref && t0 * (1.0 + 1e-6) < t1 * (1.0 - 1e-6);
      checked++;
      if (ref && !got) bad++;
    } else if (which == 8) {
      // sphere roots: sphere_t_rec with the fast roots wherever this lane is in sphere_fast_ok's range
      // against IEEE division, on rays from on / near a sphere's surface (c about 0: one root's
      // numerator hh -+ sq cancels, down to the subnormal range) and generic rays, spheres at scales
      // 2^-50 .. 2^20, every interval kind of the kernel (Surrounds on [0.001, t], the medium's boundary
      // queries on [-FLT_MAX, FLT_MAX] and [fl(t1 + 1e-4), FLT_MAX], tiny bounds around 0). Every lane
      // is compared; `checked` counts the admitted lanes whose smaller numerator cancelled (|num| <
      // 2^-20 |hh|, or 0).
      uint32_t s0, s1, s2, s3;
      philox(seed, 0x5F3Eu, (uint32_t)idx, (uint32_t)(idx >> 32), 1u, s0, s1, s2, s3);
      const float S = __uint_as_float((uint32_t)(127 - 50 + (int)(r0 % 71u)) << 23);  // 2^-50 .. 2^20
      const float rad = S * (0.25f + to_unit(r1));
      const f3 cen = mk(S * (4.0f * to_unit(r2) - 2.0f), S * (4.0f * to_unit(r3) - 2.0f), S * (4.0f * to_unit(s0) - 2.0f));
      const f3 u = normalize(mk(2.0f * to_unit(s1) - 1.0f, 2.0f * to_unit(s2) - 1.0f, 2.0f * to_unit(s3) + 0.01f - 1.0f));
      const uint32_t kind = r0 >> 29;
      f3 o;
      if (kind <= 2u) {  // on the surface (rounded), a few ulps off it, or about a sphere at the origin
        const f3 c2 = kind == 2u ? mk(0.0f, 0.0f, 0.0f) : cen;
        o = c2 + u * rad;
        if (kind == 1u) o = o * (1.0f + (float)((int)(s0 & 7u) - 4) * 0x1p-23f);
      } else {
        o = cen + mk(S * (8.0f * to_unit(r3 ^ s1) - 4.0f), S * (8.0f * to_unit(r2 ^ s2) - 4.0f), S * (8.0f * to_unit(r1 ^ s3) - 4.0f));
      }
      const f3 cen_s = kind == 2u ? mk(0.0f, 0.0f, 0.0f) : cen;
      // direction: random, or nearly tangent to the sphere at o (hh about 0), scaled 2^-20 .. 2^20
      f3 v = mk(2.0f * to_unit(s2 ^ r1) - 1.0f, 2.0f * to_unit(s3 ^ r2) - 1.0f, 2.0f * to_unit(s1 ^ r3) - 1.0f);
      if ((s1 & 3u) == 0u) v = v - u * dot(v, u);
      const float ds = __uint_as_float((uint32_t)(127 - 20 + (int)(s0 % 41u)) << 23);
      const f3 d = v * ds;
      const uint32_t ik = s2 & 3u;
      const float tmin = ik == 0u ? -FLT_MAX
                       : ik == 1u ? 0.001f
                       : ik == 2u ? ((s3 & 1u) ? -1.0f : 1.0f) * __uint_as_float((uint32_t)(127 - (int)(s3 % 126u)) << 23)
                                  : (float)((double)(S * (2.0f * to_unit(s0 ^ s3) - 1.0f)) + 0.0001);
      const float tmax = (s3 & 8u) ? FLT_MAX : fabsf(S) * 4.0f * (to_unit(r2 ^ s0) + 0.01f);
      const float4 q0 = make_float4(cen_s.x, cen_s.y, cen_s.z, rad), q1 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      float tf = 0.0f, ti = 0.0f;
      const bool hf = sphere_t_rec<1>(q0, q1, o, d, 0.0f, tmin, tmax, tf);
      const bool hi = sphere_t_rec<2>(q0, q1, o, d, 0.0f, tmin, tmax, ti);
      if (hf != hi || (hf && __float_as_uint(tf) != __float_as_uint(ti))) bad++;
      // the regular queries' guard (sphere_fast_ok_pos) on [0.001, tmax]
      float tp = 0.0f, tq = 0.0f;
      const bool hp = sphere_t_rec<3>(q0, q1, o, d, 0.0f, 0.001f, tmax, tp);
      const bool hq = sphere_t_rec<2>(q0, q1, o, d, 0.0f, 0.001f, tmax, tq);
      if (hp != hq || (hp && __float_as_uint(tp) != __float_as_uint(tq))) bad++;
      // (the operations of sphere_t_rec up to its guard)
      const f3 oc = cen_s - o;
      const float a = dot(d, d), hh = dot(d, oc), c = dot(oc, oc) - rad * rad, disc = hh * hh - a * c;
      if (disc >= 0.0f) {
        const float sq = sqrtf(disc), nmin = fminf(fabsf(hh - sq), fabsf(hh + sq));
        if (sphere_fast_ok(a, hh, sq) && (nmin < 0x1p-20f * fabsf(hh) || nmin == 0.0f)) checked++;
      }
    } else if (which == 5) {
      // every float bit pattern (n = 2^32): rcp_nr against IEEE 1/x over its whole range
      const float x = __uint_as_float((uint32_t)idx);
      if (!rcp_in_range(x)) continue;
      checked++;
      if (__float_as_uint(rcp_nr(x)) != __float_as_uint(1.0f / x)) bad++;
    } else if (which == 2) {
      // rcp_nr / sqrt_nr against IEEE 1/x and sqrt(x) over their whole ranges
      const float x = rand_float(r0, -95, 125, r1);
      const float y = fabsf(rand_float(r2, -96, 125, r3));
      checked++;
      if (__float_as_uint(rcp_nr(x)) != __float_as_uint(1.0f / x)) bad++;
      if (__float_as_uint(sqrt_nr(y)) != __float_as_uint(sqrtf(y))) bad++;
    } else {
      uint32_t s0, s1, s2, s3;
      philox(seed, 0xAABBu, (uint32_t)idx, (uint32_t)(idx >> 32), 1u, s0, s1, s2, s3);
      const float lo_x = rand_float(r0, -4, 9, r1), hi_x = lo_x + rand_float(r1, -6, 8, r0 >> 7);
      const float lo_y = rand_float(r2, -4, 9, r3), hi_y = lo_y + rand_float(r3, -6, 8, r2 >> 7);
      const float lo_z = rand_float(s0, -4, 9, s1), hi_z = lo_z + rand_float(s1, -6, 8, s0 >> 7);
      const f3 o = mk(rand_float(s2, -3, 10, s3), rand_float(s3, -3, 10, s2 >> 5), rand_float(s2 ^ s3, -3, 10, s1));
      const f3 d = mk(rand_float(r0 ^ s0, -40, 1, r3), rand_float(r1 ^ s1, -40, 1, s3 >> 3), rand_float(r2 ^ s2, -40, 1, r0));
      const f3 inv = recip3(d);
      if (!finite3(inv)) continue;
      const float tmax = (s3 & 1u) ? FLT_MAX : rand_float(s0 ^ r3, -3, 12, s2);
      const float4 lo = make_float4(lo_x, lo_y, lo_z, 0.0f), hi = make_float4(hi_x, hi_y, hi_z, 0.0f);
      checked++;
      if (aabb_hit_fin(lo, hi, o, inv, 0.001f, tmax) != aabb_hit(lo, hi, o, inv, 0.001f, tmax)) bad++;
    }
  }
  atomicAdd(out, bad);
  atomicAdd(out + 1, checked);
}

}  // namespace dev

int RenderVariant(uint32_t features) {
  int best = dev::kNumVariants - 1;
  for (int v = 0; v < dev::kNumVariants; v++) {
    if ((dev::kVariants[v] & features) == features &&
        __builtin_popcount(dev::kVariants[v]) < __builtin_popcount(dev::kVariants[best]))
      best = v;
  }
  return best;
}

uint32_t RenderVariantFeatures(int v) { return dev::kVariants[v]; }

int RenderMode(const RenderParams& p) {
  if (p.lin_len) return kModeLinear;
  if (!p.lds_nodes) return kModeStackGlobal;
  return p.lds_partial ? kModeStackHybrid : kModeStackLds;
}

size_t RenderLdsBytes(const RenderParams& p) {
  if (p.lin_len) return 0;
  return (size_t)p.lds_nodes * 16 + (size_t)p.stack_depth * dev::kBlock * 4;
}

// Launch entry used by capi.cpp. grid = resident workgroups (persistent lanes).
hipError_t LaunchRender(const RenderParams& p, int variant, bool stats, int grid, hipStream_t stream) {
  dev::KernelFn fn = dev::Kernel(variant, RenderMode(p), stats);
  if (!fn) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(dev::kBlock), RenderLdsBytes(p), stream, p);
  return hipGetLastError();
}

hipError_t LaunchAccumulate(const float* samples, float* accum, uint8_t* pixels, uint32_t npix, int n_frames,
                            int frame_idx, hipStream_t stream) {
  if (npix == 0) return hipSuccess;
  hipLaunchKernelGGL(dev::accumulate_kernel, dim3((npix + 255u) / 256u), dim3(256), 0, stream, samples, accum,
                     reinterpret_cast<uint32_t*>(pixels), npix, n_frames, frame_idx);
  return hipGetLastError();
}

hipError_t LaunchSelftest(int which, unsigned long long n, uint32_t seed, unsigned long long* d_out, hipStream_t stream) {
  hipLaunchKernelGGL(dev::selftest_kernel, dim3(4096), dim3(256), 0, stream, which, n, seed, d_out);
  return hipGetLastError();
}

int RenderBlocksPerCU(int variant, int mode, bool stats, size_t lds_bytes) {
  int n = 0;
  dev::KernelFn fn = dev::Kernel(variant, mode, stats);
  if (!fn) return 1;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(fn), dev::kBlock,
                                                             lds_bytes);
  return e == hipSuccess && n > 0 ? n : 1;
}

int RenderBlockSize() { return dev::kBlock; }

}  // namespace rt2
