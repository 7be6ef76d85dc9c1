// render.hip — the hot path: RayTracer::Update (RayTracer.cpp:55-70) → Camera::GetRay
// (Camera.hpp:50-67) → RayColor (RayTracer.cpp:20-45) → closest-hit traversal (BVH.cpp:50-55,
// HittableList.cpp:8-22, Quad.cpp:19-43, Sphere.cpp:7-37, Transform.cpp:75-88,
// ConstantMedium.cpp:14-58) → Scatter/Emit (Material.cpp:10-83, Texture.cpp:7-22,
// PerlinNoiseGen.cpp:54-88), as one persistent gfx950 kernel.
//
// Execution model (MI355X):
//  * one lane = one pixel for a whole launch; a lane renders that pixel's frames
//    [frame_begin, frame_begin + n_frames) back to back and accumulates them in registers in
//    frame order, so the float sum is the reference's `accumulation_data_[i] += c` sequence;
//  * one loop iteration = one bounce for every live lane; a lane whose path ends starts its next
//    frame in the same iteration (path regeneration), so lanes never idle inside a wave until
//    their pixel is done;
//  * pixels are handed out in 8x8 tiles by a wave-aggregated atomic: __ballot of the lanes that
//    need work, one atomicAdd per wave, mbcnt-style prefix for each lane's slot;
//  * the traversal stack lives in LDS (kTraversalStack entries per lane, lane-major columns, so a
//    wave's push/pop is one conflict-free ds_write/ds_read);
//  * the flattened scene (rt2_layout.h) is read with 16-byte loads; it is small and shared by
//    every lane, so it is served from L1/L2.
//
// Numerics: compiled with -ffp-contract=off; fp32 division and sqrt are correctly rounded (HIP
// default). Every expression repeats the reference's operation order, so results match the
// CPU restatement bit for bit except the radiance product, which is accumulated front to back
// (thr *= att) instead of the reference's recursion order (att0*(att1*(...*E))).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "rt2_layout.h"

namespace rt2 {
namespace dev {

constexpr int kBlock = 256;

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
__device__ __forceinline__ f3 normalize(f3 v) { return v * (1.0f / sqrtf(dot(v, v))); }
__device__ __forceinline__ f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }
__device__ __forceinline__ uint32_t bits(float f) { return __float_as_uint(f); }
// glm scalar max/min
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }
__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }

// ------------------------------------------------------------------------------------------
// Philox4x32-10 path stream keyed by (seed, pixel, frame).
struct Rng {
  uint32_t k0, k1, a, b, block, idx;
  uint32_t r0, r1, r2, r3;
  __device__ __forceinline__ void init(uint32_t seed_lo, uint32_t seed_hi, uint32_t pixel, uint32_t frame) {
    k0 = seed_lo;
    k1 = seed_hi;
    a = pixel;
    b = frame;
    block = 0;
    idx = 4;
  }
  __device__ __forceinline__ void refill() {
    uint32_t c0 = a, c1 = b, c2 = block++, c3 = kTagPathDev;
    uint32_t key0 = k0, key1 = k1;
#pragma unroll
    for (int r = 0; r < 10; r++) {
      uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
      uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
      uint32_t n0 = hi1 ^ c1 ^ key0, n2 = hi0 ^ c3 ^ key1;
      c0 = n0;
      c1 = lo1;
      c2 = n2;
      c3 = lo0;
      key0 += 0x9E3779B9u;
      key1 += 0xBB67AE85u;
    }
    r0 = c0;
    r1 = c1;
    r2 = c2;
    r3 = c3;
    idx = 0;
  }
  __device__ __forceinline__ float uniform() {
    if (idx == 4) refill();
    uint32_t v = idx == 0 ? r0 : (idx == 1 ? r1 : (idx == 2 ? r2 : r3));
    idx++;
    return (float)(v >> 8) * (1.0f / 16777216.0f);
  }
  // Math.hpp:15 RandReal(min, max)
  __device__ __forceinline__ float uniform(float mn, float mx) { return mn + uniform() * (mx - mn); }
  static constexpr uint32_t kTagPathDev = 0x52543250u;
};

// Math.hpp:26-43
__device__ __forceinline__ f3 rand_unit_vec3(Rng& g) {
  f3 p;
  while (true) {
    float x = g.uniform(-1.0f, 1.0f);
    float y = g.uniform(-1.0f, 1.0f);
    float z = g.uniform(-1.0f, 1.0f);
    p = mk(x, y, z);
    float lsq = dot(p, p);
    if (lsq > 0.0f && lsq <= 1.0f) break;  // 1e-160 < |p|^2 <= 1 for a float |p|^2
  }
  return normalize(p);
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

struct Hit {
  float t;
  f3 p, n;
  uint32_t mat;
  bool front;
};

struct Counters {
  uint32_t bvh, quad, sphere, xform, medium, list;
};

// ------------------------------------------------------------------------------------------
// Primitive tests. Each returns true and fills (t, p, n, front, mat) in the ray's space.

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

// Quad::Hit (Quad.cpp:19-43): inclusive interval (Contains)
__device__ __forceinline__ bool quad_hit(const float4* N, uint32_t off, f3 o, f3 d, float tmin, float tmax, Hit& h) {
  float4 r0 = N[off];
  f3 n = xyz(r0);
  float n_dot = dot(n, d);
  if (fabsf(n_dot) <= 1e-8f) return false;
  float t = (r0.w - dot(n, o)) / n_dot;
  if (!(tmin <= t && t <= tmax)) return false;
  float4 r1 = N[off + 1], r2 = N[off + 2], r3 = N[off + 3], r4 = N[off + 4];
  f3 p = o + d * t;
  f3 pv = p - xyz(r1);
  float alpha = dot(xyz(r4), cross(pv, xyz(r3)));
  float beta = dot(xyz(r4), cross(xyz(r2), pv));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return false;
  h.t = t;
  h.p = p;
  h.mat = bits(r1.w);
  h.front = dot(d, n) < 0.0f;
  h.n = h.front ? n : -n;
  return true;
}

// Sphere::Hit (Sphere.cpp:7-37): exclusive interval (Surrounds); uv is dead output
__device__ __forceinline__ bool sphere_hit(const float4* N, uint32_t off, f3 o, f3 d, float time, float tmin,
                                           float tmax, Hit& h) {
  float4 r0 = N[off], r1 = N[off + 1];
  f3 center = xyz(r0) + xyz(r1) * time;
  f3 oc = center - o;
  float a = dot(d, d);
  float hh = dot(d, oc);
  float c = dot(oc, oc) - r0.w * r0.w;
  float disc = hh * hh - a * c;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  float root = (hh - sq) / a;
  if (!(tmin < root && root < tmax)) {
    root = (hh + sq) / a;
    if (!(tmin < root && root < tmax)) return false;
  }
  h.t = root;
  h.p = o + d * root;
  h.mat = bits(r1.w);
  f3 outward = (h.p - center) / r0.w;
  h.front = dot(d, outward) < 0.0f;
  h.n = h.front ? outward : -outward;
  return true;
}

// Closest t of a ConstantMedium boundary (quad, sphere or a list of them) on [lo, hi]
__device__ __forceinline__ bool boundary_hit(const float4* N, uint32_t ref, f3 o, f3 d, float time, float lo,
                                             float hi, float& t_out, Counters& cnt) {
  uint32_t kind = ref >> 28, off = ref & kOffsetMask;
  Hit tmp;
  if (kind == kQuad) {
    cnt.quad++;
    if (!quad_hit(N, off, o, d, lo, hi, tmp)) return false;
    t_out = tmp.t;
    return true;
  }
  if (kind == kSphere) {
    cnt.sphere++;
    if (!sphere_hit(N, off, o, d, time, lo, hi, tmp)) return false;
    t_out = tmp.t;
    return true;
  }
  // leaf-only list (box): sequential, shrinking max
  uint32_t n = bits(N[off].x);
  bool any = false;
  for (uint32_t k = 0; k < n; k++) {
    uint32_t c = bits(reinterpret_cast<const float*>(N + off + 1)[k]);
    uint32_t ck = c >> 28, co = c & kOffsetMask;
    bool hit;
    if (ck == kQuad) {
      cnt.quad++;
      hit = quad_hit(N, co, o, d, lo, hi, tmp);
    } else {
      cnt.sphere++;
      hit = sphere_hit(N, co, o, d, time, lo, hi, tmp);
    }
    if (hit) {
      any = true;
      hi = tmp.t;
    }
  }
  if (any) t_out = hi;
  return any;
}

// World -> model space of one XFORM (Transform.cpp:13-20)
__device__ __forceinline__ void to_model(const float4* N, uint32_t off, f3& o, f3& d) {
  float4 c0 = N[off], c1 = N[off + 1], c2 = N[off + 2], c3 = N[off + 3];
  f3 no = mk((c0.x * o.x + c1.x * o.y) + (c2.x * o.z + c3.x), (c0.y * o.x + c1.y * o.y) + (c2.y * o.z + c3.y),
             (c0.z * o.x + c1.z * o.y) + (c2.z * o.z + c3.z));
  f3 nd = mk(c0.x * d.x + c1.x * d.y + c2.x * d.z, c0.y * d.x + c1.y * d.y + c2.y * d.z,
             c0.z * d.x + c1.z * d.y + c2.z * d.z);
  o = no;
  d = normalize(nd);
}

// Ray in the space of XFORM `xref` (kRefNone = world), rebuilt from the world ray through the
// chain of enclosing transforms (only needed for nested transforms; depth <= 8).
__device__ void ray_in_space(const float4* N, uint32_t xref, f3 wo, f3 wd, f3& o, f3& d) {
  o = wo;
  d = wd;
  if (xref == kRefNone) return;
  uint32_t chain[8];
  int n = 0;
  for (uint32_t x = xref; x != kRefNone && n < 8; x = bits(N[(x & kOffsetMask) + 1].w)) chain[n++] = x;
  for (int k = n - 1; k >= 0; k--) to_model(N, chain[k] & kOffsetMask, o, d);
}

// ------------------------------------------------------------------------------------------
// Closest hit over the scene program (HittableList{BVHNode} at the root, App.cpp:126).
// Reference semantics preserved: left-then-right, right subtree pruned by the current closest t,
// model-space t of transformed children compared as-is (Transform.cpp:82), span-1 media tested
// twice with fresh random numbers, media boundaries queried on (-FLT_MAX, FLT_MAX).
template <bool kStats>
__device__ bool trace(const RenderParams& P, f3 wo, f3 wd, float time, Rng& rng, Hit& h, uint32_t* stk,
                      Counters& cnt, bool& overflow) {
  const float4* N = reinterpret_cast<const float4*>(P.nodes);
  f3 o = wo, d = wd;
  f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const float tmin = 0.001f;  // Interval{0.001, kInfinity}
  float tmax = FLT_MAX;
  bool any = false;
  int depth = 0;           // transform nesting depth
  uint32_t hitmask = 0;    // bit k: a hit was recorded inside the transform at depth k
  int sp = 0;
  stk[0] = P.root;
  sp = 1;
  while (sp > 0) {
    sp--;
    uint32_t ref = stk[sp * kBlock];
    uint32_t kind = ref >> 28, off = ref & kOffsetMask;
    if (kind == kBvh) {
      if (kStats) cnt.bvh++;
      float4 lo = N[off], hi = N[off + 1];
      if (aabb_hit(lo, hi, o, inv, tmin, tmax)) {
        uint32_t right = bits(hi.w);
        if (sp + 2 > kTraversalStack) {
          overflow = true;
          continue;
        }
        if (right != kRefNone) stk[(sp++) * kBlock] = right;
        stk[(sp++) * kBlock] = bits(lo.w);
      }
    } else if (kind == kQuad) {
      if (kStats) cnt.quad++;
      if (quad_hit(N, off, o, d, tmin, tmax, h)) {
        tmax = h.t;
        any = true;
        hitmask |= 1u << depth;
      }
    } else if (kind == kSphere) {
      if (kStats) cnt.sphere++;
      if (sphere_hit(N, off, o, d, time, tmin, tmax, h)) {
        tmax = h.t;
        any = true;
        hitmask |= 1u << depth;
      }
    } else if (kind == kList) {
      if (kStats) cnt.list++;
      float4 hdr = N[off];
      uint32_t n = bits(hdr.x);
      const float* refs = reinterpret_cast<const float*>(N + off + 1);
      if (bits(hdr.y) & kListLeafOnly) {
        for (uint32_t k = 0; k < n; k++) {
          uint32_t c = bits(refs[k]);
          uint32_t co = c & kOffsetMask;
          bool hit;
          if ((c >> 28) == kQuad) {
            if (kStats) cnt.quad++;
            hit = quad_hit(N, co, o, d, tmin, tmax, h);
          } else {
            if (kStats) cnt.sphere++;
            hit = sphere_hit(N, co, o, d, time, tmin, tmax, h);
          }
          if (hit) {
            tmax = h.t;
            any = true;
            hitmask |= 1u << depth;
          }
        }
      } else {
        if (sp + (int)n > kTraversalStack) {
          overflow = true;
          continue;
        }
        for (int k = (int)n - 1; k >= 0; k--) stk[(sp++) * kBlock] = bits(refs[k]);
      }
    } else if (kind == kXform) {
      if (kStats) cnt.xform++;
      if (sp + 2 > kTraversalStack || depth >= 31) {
        overflow = true;
        continue;
      }
      depth++;
      hitmask &= ~(1u << depth);
      to_model(N, off, o, d);
      inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
      stk[(sp++) * kBlock] = make_ref(kXformExit, off);
      stk[(sp++) * kBlock] = bits(N[off].w);
    } else if (kind == kXformExit) {
      if ((hitmask >> depth) & 1u) {
        // back to the parent space: point via M, normal via transpose(inverse(M)) (Transform.cpp:85-86)
        float4 m0 = N[off + 4], m1 = N[off + 5], m2 = N[off + 6], m3 = N[off + 7];
        f3 p = h.p;
        h.p = mk((m0.x * p.x + m1.x * p.y) + (m2.x * p.z + m3.x), (m0.y * p.x + m1.y * p.y) + (m2.y * p.z + m3.y),
                 (m0.z * p.x + m1.z * p.y) + (m2.z * p.z + m3.z));
        float4 c0 = N[off], c1 = N[off + 1], c2 = N[off + 2];
        f3 n = h.n;
        h.n = normalize(mk(c0.x * n.x + c0.y * n.y + c0.z * n.z, c1.x * n.x + c1.y * n.y + c1.z * n.z,
                           c2.x * n.x + c2.y * n.y + c2.z * n.z));
        hitmask |= 1u << (depth - 1);
      }
      depth--;
      ray_in_space(N, bits(N[off + 1].w), wo, wd, o, d);
      inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    } else {  // kMedium
      if (kStats) cnt.medium++;
      float4 r0 = N[off];
      uint32_t bref = bits(r0.z);
      float t1, t2;
      if (!boundary_hit(N, bref, o, d, time, -FLT_MAX, FLT_MAX, t1, cnt)) continue;
      if (!boundary_hit(N, bref, o, d, time, (float)((double)t1 + 0.0001), FLT_MAX, t2, cnt)) continue;
      t1 = fmaxf(t1, tmin);
      t2 = fminf(t2, tmax);
      if (t1 >= t2) continue;
      t1 = fmaxf(t1, 0.0f);
      float len = sqrtf(dot(d, d));
      float inside = (t2 - t1) * len;
      float hit_dist = r0.x * (float)log((double)rng.uniform());
      if (hit_dist > inside) continue;
      h.t = t1 + hit_dist / len;
      h.p = o + d * h.t;
      h.n = mk(1.0f, 0.0f, 0.0f);
      h.front = true;
      h.mat = bits(r0.y);
      tmax = h.t;
      any = true;
      hitmask |= 1u << depth;
    }
  }
  return any;
}

// ------------------------------------------------------------------------------------------
// Textures (Texture.cpp:7-22, PerlinNoiseGen.cpp:10-88)
__device__ float perlin_noise(const RenderParams& P, uint32_t voff, uint32_t poff, uint32_t pc, f3 p) {
  const float4* V = reinterpret_cast<const float4*>(P.perlin_vec) + voff;
  const int* Px = P.perlin_perm + poff;
  const int* Py = Px + pc;
  const int* Pz = Py + pc;
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int i = (int)fx, j = (int)fy, k = (int)fz;
  float uu = u * u * (3.0f - 2.0f * u);
  float vv = v * v * (3.0f - 2.0f * v);
  float ww = w * w * (3.0f - 2.0f * w);
  float accum = 0.0f;
#pragma unroll
  for (int di = 0; di < 2; di++)
#pragma unroll
    for (int dj = 0; dj < 2; dj++)
#pragma unroll
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

__device__ f3 tex_value(const RenderParams& P, uint32_t idx, f3 p) {
  const float4* T = reinterpret_cast<const float4*>(P.textures);
  for (int guard = 0; guard < 32; guard++) {
    float4 t0 = T[3 * idx], t1 = T[3 * idx + 1];
    uint32_t type = bits(t0.x);
    if (type == kTexSolid) return mk(t0.y, t0.z, t0.w);
    if (type == kTexChecker) {
      f3 sp = t1.x * p;
      int ix = (int)floorf(sp.x), iy = (int)floorf(sp.y), iz = (int)floorf(sp.z);
      idx = ((ix + iy + iz) % 2 == 0) ? bits(t1.y) : bits(t1.z);
      continue;
    }
    float4 t2 = T[3 * idx + 2];
    uint32_t voff = bits(t2.x), poff = bits(t2.y), pc = bits(t2.z);
    f3 alb = mk(t0.y, t0.z, t0.w) * 0.5f;
    if (bits(t1.w) == 1u) {  // NoiseType::kMarble
      float acc = 0.0f, weight = 1.0f;
      f3 tp = p;
      for (int k = 0; k < 7; k++) {
        acc += weight * perlin_noise(P, voff, poff, pc, tp);
        weight *= 0.5f;
        tp = tp * 2.0f;
      }
      float arg = t1.x * p.z + 10.0f * fabsf(acc);
      return alb * (1.0f + (float)sin((double)arg));
    }
    return alb * (1.0f + perlin_noise(P, voff, poff, pc, t1.x * p));
  }
  return mk(0.0f, 0.0f, 0.0f);  // checker cycle (the reference recurses forever)
}

// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void camera_ray(const RenderParams& P, int x, int y, int s_i, int s_j, Rng& g, f3& o,
                                           f3& d, float& time) {
  const CameraParams& C = P.cam;
  float px = ((float)s_i + g.uniform()) * C.recip_sqrt_spp - 0.5f;
  float py = ((float)s_j + g.uniform()) * C.recip_sqrt_spp - 0.5f;
  f3 p00 = mk(C.pixel00[0], C.pixel00[1], C.pixel00[2]);
  f3 du = mk(C.du[0], C.du[1], C.du[2]);
  f3 dv = mk(C.dv[0], C.dv[1], C.dv[2]);
  f3 pc = (p00 + (((float)x + px) * du)) + (((float)y + py) * dv);
  f3 c = mk(C.center[0], C.center[1], C.center[2]);
  if (!(C.defocus_angle <= 0.0f)) {
    float dx, dy;
    while (true) {  // RandInUnitDisk (x drawn before y)
      dx = g.uniform(-1.0f, 1.0f);
      dy = g.uniform(-1.0f, 1.0f);
      if ((dx * dx + dy * dy) + 0.0f * 0.0f < 1.0f) break;
    }
    c = (c + (dx * mk(C.defocus_u[0], C.defocus_u[1], C.defocus_u[2]))) +
        (dy * mk(C.defocus_v[0], C.defocus_v[1], C.defocus_v[2]));
  }
  time = g.uniform();
  o = c;
  d = normalize(pc - c);
}

template <bool kStats>
__global__ __launch_bounds__(kBlock) void render_kernel(const RenderParams P) {
  __shared__ uint32_t s_stack[kTraversalStack * kBlock];
  uint32_t* stk = s_stack + threadIdx.x;
  const int lane = (int)__lane_id();
  const float4* M = reinterpret_cast<const float4*>(P.materials);
  const f3 bg = mk(P.background[0], P.background[1], P.background[2]);
  const int sq = P.cam.sqrt_spp;
  const int frame_end = P.frame_begin + P.n_frames;

  bool need = true;  // lane wants a pixel
  int x = 0, y = 0;
  uint32_t lidx = 0, pix = 0;
  int f = 0;
  f3 acc = mk(0, 0, 0);
  uint32_t item_rays = 0;
  // path state
  f3 ro = mk(0, 0, 0), rd = mk(0, 0, 1), thr = mk(1, 1, 1);
  float rtime = 0.0f;
  int depth_left = 0;
  Rng rng;
  rng.init(0, 0, 0, 0);
  Counters cnt = {0, 0, 0, 0, 0, 0};
  unsigned long long rays = 0, paths = 0;
  bool overflow = false;

  while (true) {
    // ---- hand out pixels: one atomic per wave
    unsigned long long mask = __ballot(need);
    if (mask != 0ull) {
      uint32_t count = (uint32_t)__popcll(mask);
      int leader = __ffsll((long long)mask) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(P.work_counter, count);
      base = (uint32_t)__shfl((int)base, leader);
      if (need) {
        uint32_t item = base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        if (item >= P.n_items) break;  // no work left for this lane
        uint32_t tile = item >> 6, within = item & 63u;
        x = (int)((tile % (uint32_t)P.tiles_x) * 8u + (within & 7u));
        int r = (int)((tile / (uint32_t)P.tiles_x) * 8u + (within >> 3));
        if (x >= P.width || r >= P.local_rows) continue;  // partial edge tile
        y = ((r / P.band_h) * P.world + P.rank) * P.band_h + (r % P.band_h);
        lidx = (uint32_t)r * (uint32_t)P.width + (uint32_t)x;
        pix = (uint32_t)y * (uint32_t)P.width + (uint32_t)x;
        acc = mk(P.accum[3 * lidx], P.accum[3 * lidx + 1], P.accum[3 * lidx + 2]);
        item_rays = 0;
        f = P.frame_begin;
        need = false;
        if (f >= frame_end) {
          need = true;  // zero frames requested
          continue;
        }
        rng.init(P.seed_lo, P.seed_hi, pix, (uint32_t)f);
        camera_ray(P, x, y, f % sq, f / sq % sq, rng, ro, rd, rtime);
        thr = mk(1, 1, 1);
        depth_left = P.max_depth;
      }
    }
    if (need) continue;

    // ---- one bounce (RayColor, RayTracer.cpp:20-45)
    bool done = false;
    f3 color = mk(0, 0, 0);
    if (depth_left <= 0) {
      done = true;  // RayColor(depth <= 0) returns 0 without casting a ray
    } else {
      item_rays++;
      rays++;
      Hit h;
      if (!trace<kStats>(P, ro, rd, rtime, rng, h, stk, cnt, overflow)) {
        color = thr * bg;
        done = true;
      } else {
        float4 m0 = M[2 * h.mat], m1 = M[2 * h.mat + 1];
        uint32_t type = bits(m0.x);
        if (type == kMatDiffuseLight) {
          color = thr * tex_value(P, bits(m1.z), h.p);
          done = true;
        } else {
          f3 att, dir;
          if (type == kMatMetal) {
            dir = normalize(reflect(rd, h.n)) + (m1.x * rand_unit_vec3(rng));
            att = mk(m0.y, m0.z, m0.w);
          } else if (type == kMatDielectric) {
            att = mk(1.0f, 1.0f, 1.0f);
            float ri = h.front ? m1.w : m1.y;
            f3 ud = normalize(rd);
            float cos_t = gmin(dot(-ud, h.n), 1.0f);
            float sin_t = sqrtf(1.0f - cos_t * cos_t);
            bool refl = ri * sin_t > 1.0f;
            if (!refl) {
              float r0 = (1.0f - ri) / (1.0f + ri);
              r0 = r0 * r0;
              double xx = (double)(1.0f - cos_t);
              double x2 = xx * xx;
              double x5 = (x2 * x2) * xx;
              double schlick = (double)r0 + (double)(1.0f - r0) * x5;
              refl = schlick > (double)rng.uniform();
            }
            dir = refl ? reflect(ud, h.n) : refract(ud, h.n, ri);
          } else if (type == kMatIsotropic) {
            dir = rand_unit_vec3(rng);
            att = tex_value(P, bits(m1.z), h.p);
          } else {  // Lambertian / Texture
            dir = h.n + rand_unit_vec3(rng);
            if (near_zero(dir)) dir = h.n;
            att = (type == kMatLambertian) ? mk(m0.y, m0.z, m0.w) : tex_value(P, bits(m1.z), h.p);
          }
          thr = thr * att;
          ro = h.p;
          rd = dir;
          depth_left--;
        }
      }
    }
    if (done) {
      acc = acc + color;
      paths++;
      f++;
      if (f < frame_end) {
        rng.init(P.seed_lo, P.seed_hi, pix, (uint32_t)f);
        camera_ray(P, x, y, f % sq, f / sq % sq, rng, ro, rd, rtime);
        thr = mk(1, 1, 1);
        depth_left = P.max_depth;
      } else {
        // RayTracer.cpp:64-66: accumulate; live display value = ToColor(clamp(accum / frame_idx, 0, 1))
        P.accum[3 * lidx] = acc.x;
        P.accum[3 * lidx + 1] = acc.y;
        P.accum[3 * lidx + 2] = acc.z;
        if (P.pixels) {
          float fi = (float)frame_end;
          f3 c = acc / fi;
          float cc[3] = {c.x, c.y, c.z};
          uint32_t rgba = 0xFF000000u;
#pragma unroll
          for (int k = 0; k < 3; k++) {
            float v = gmin(gmax(cc[k], 0.0f), 1.0f);
            rgba |= ((uint32_t)(uint8_t)floor((double)v * 255.999)) << (8 * k);
          }
          reinterpret_cast<uint32_t*>(P.pixels)[lidx] = rgba;
        }
        if (P.ray_counts) P.ray_counts[lidx] += item_rays;
        need = true;
      }
    }
  }

  atomicAdd(P.stats + StatsCounters::kRays, rays);
  atomicAdd(P.stats + StatsCounters::kPaths, paths);
  if (kStats) {
    atomicAdd(P.stats + StatsCounters::kBvhTests, (unsigned long long)cnt.bvh);
    atomicAdd(P.stats + StatsCounters::kQuadTests, (unsigned long long)cnt.quad);
    atomicAdd(P.stats + StatsCounters::kSphereTests, (unsigned long long)cnt.sphere);
    atomicAdd(P.stats + StatsCounters::kXformVisits, (unsigned long long)cnt.xform);
    atomicAdd(P.stats + StatsCounters::kMediumTests, (unsigned long long)cnt.medium);
    atomicAdd(P.stats + StatsCounters::kListVisits, (unsigned long long)cnt.list);
  }
  if (overflow) atomicAdd(P.stats + StatsCounters::kCount, 1ull);  // overflow flag slot
}

}  // namespace dev

// Launch entry used by capi.cpp. grid = resident workgroups (persistent lanes).
hipError_t LaunchRender(const RenderParams& p, bool stats, int grid, hipStream_t stream) {
  if (stats) {
    hipLaunchKernelGGL(dev::render_kernel<true>, dim3(grid), dim3(dev::kBlock), 0, stream, p);
  } else {
    hipLaunchKernelGGL(dev::render_kernel<false>, dim3(grid), dim3(dev::kBlock), 0, stream, p);
  }
  return hipGetLastError();
}

int RenderBlocksPerCU(bool stats) {
  int n = 0;
  hipError_t e;
  if (stats) {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::render_kernel<true>, dev::kBlock, 0);
  } else {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::render_kernel<false>, dev::kBlock, 0);
  }
  return e == hipSuccess && n > 0 ? n : 1;
}

int RenderBlockSize() { return dev::kBlock; }

}  // namespace rt2
