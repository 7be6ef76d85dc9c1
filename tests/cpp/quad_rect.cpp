// Host check of the rectangle shortcut of the threaded kernel's quad test (rt2_layout.h RectAA,
// render.hip quad_aa / quad_inside), compiled with -ffp-contract=off like the kernel:
//   quad_rect <scene.json> <rays per quad>
// For every unit-normal axis-aligned quad of the scene that RectAA accepts, random rays and rays
// aimed at its edges and corners are tested two ways: Quad::Hit as the reference writes it
// (Quad.cpp:19-43, glm dot / cross operation order) and the kernel's form from the QUADAA words
// (t = (sD - o_K) / d_K, alpha = w_K (pva v_B), beta = w_K (u_A pvb)). The hit decision and t
// must be equal on every ray. Prints "rect=<n> rays=<n> hits=<n>"; exits non-zero on a mismatch.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "scene.h"

using namespace rt2;

namespace {
struct V3 {
  float x, y, z;
};
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
V3 cross(V3 x, V3 y) { return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
float comp(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// Quad.cpp:19-43 (no interval test: both forms are compared on the candidate itself)
bool ref_hit(V3 q, V3 u, V3 v, V3 w, V3 n, float d, V3 o, V3 dir, float& t) {
  const float n_dot = dot(n, dir);
  if (std::fabs(n_dot) < 1e-8) return false;
  t = (d - dot(n, o)) / n_dot;
  const V3 pv = sub(add(o, mul(dir, t)), q);
  const float alpha = dot(w, cross(pv, v)), beta = dot(w, cross(u, pv));
  return 0.0f <= alpha && alpha <= 1.0f && 0.0f <= beta && beta <= 1.0f;
}
// render.hip quad_aa with IEEE division (div_by_inv equals it, GPU self-test) and quad_inside
bool rect_hit(const float* r, int K, V3 o, V3 dir, float& t) {
  const int A = (K + 1) % 3, B = (K + 2) % 3;
  const float dk = comp(dir, K);
  t = (r[0] - comp(o, K)) / dk;
  const float pva = (comp(o, A) + comp(dir, A) * t) - r[2];
  const float pvb = (comp(o, B) + comp(dir, B) * t) - r[3];
  const float alpha = r[1] * (pva * r[7]), beta = r[1] * (r[4] * pvb);
  return !(std::fabs(dk) <= 1e-8f) && 0.0f <= alpha && alpha <= 1.0f && 0.0f <= beta && beta <= 1.0f;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  Scene s;
  std::string err;
  if (!LoadScene(argv[1], 0x5EED2024ull, s, err)) {
    std::fprintf(stderr, "load: %s\n", err.c_str());
    return 2;
  }
  const long per = std::atol(argv[2]);
  std::mt19937 rng(12345);
  std::uniform_real_distribution<float> U(-1.0f, 1.0f), U01(0.0f, 1.0f);
  long rects = 0, rays = 0, hits = 0;
  for (const Obj& ob : s.objs) {
    if (ob.kind != kQuad) continue;
    int K = -1;
    for (int k = 0; k < 3; k++) {
      const int a = (k + 1) % 3, b = (k + 2) % 3;
      if (comp({ob.n.x, ob.n.y, ob.n.z}, a) == 0.0f && comp({ob.n.x, ob.n.y, ob.n.z}, b) == 0.0f &&
          comp({ob.w.x, ob.w.y, ob.w.z}, a) == 0.0f && comp({ob.w.x, ob.w.y, ob.w.z}, b) == 0.0f &&
          std::fabs(comp({ob.n.x, ob.n.y, ob.n.z}, k)) == 1.0f)
        K = k;
    }
    if (K < 0) continue;
    const V3 q{ob.q.x, ob.q.y, ob.q.z}, u{ob.u.x, ob.u.y, ob.u.z}, v{ob.v.x, ob.v.y, ob.v.z};
    const V3 w{ob.w.x, ob.w.y, ob.w.z}, n{ob.n.x, ob.n.y, ob.n.z};
    // the QUAD record (rt2_layout.h) as the compiler writes it
    float rec[20] = {n.x, n.y, n.z, ob.d, q.x, q.y, q.z, 0, u.x, u.y, u.z, 0, v.x, v.y, v.z, 0,
                     w.x, w.y, w.z, comp(n, K) * ob.d};
    float aa[8];
    if (!RectAA(rec, K, aa)) continue;
    rects++;
    const float span = std::sqrt(dot(u, u)) + std::sqrt(dot(v, v)) + 1.0f;
    const float edge[7] = {0.0f, 1.0f, 0.5f, std::nextafter(0.0f, 1.0f), std::nextafter(0.0f, -1.0f),
                           std::nextafter(1.0f, 2.0f), std::nextafter(1.0f, 0.0f)};
    for (long i = 0; i < per; i++) {
      const V3 o = add(q, V3{U(rng) * 2 * span, U(rng) * 2 * span, U(rng) * 2 * span});
      V3 dir;
      if (i % 3 == 0) {
        dir = V3{U(rng), U(rng), U(rng)};
      } else {  // aimed at an edge / corner / the interior
        const float a = i % 3 == 1 ? edge[rng() % 7] : U01(rng), b = edge[rng() % 7];
        const V3 target = (rng() & 1) ? add(add(q, mul(u, a)), mul(v, b)) : add(add(q, mul(u, b)), mul(v, a));
        dir = sub(target, o);
      }
      float t0 = 0, t1 = 0;
      const bool h0 = ref_hit(q, u, v, w, n, ob.d, o, dir, t0), h1 = rect_hit(aa, K, o, dir, t1);
      rays++;
      if (h0 != h1 || (h0 && std::memcmp(&t0, &t1, 4) != 0)) {
        std::fprintf(stderr, "mismatch: quad q=(%g %g %g) ray o=(%a %a %a) d=(%a %a %a): ref %d t=%a, rect %d t=%a\n",
                     q.x, q.y, q.z, o.x, o.y, o.z, dir.x, dir.y, dir.z, h0, t0, h1, t1);
        return 1;
      }
      hits += h0;
    }
  }
  std::printf("rect=%ld rays=%ld hits=%ld\n", rects, rays, hits);
  return rects > 0 ? 0 : 3;
}
