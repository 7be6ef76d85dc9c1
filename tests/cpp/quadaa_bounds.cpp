// Host check of the QUADAA interior bounds (compile.cpp RectAAWords / CoordRange):
//   quadaa_bounds <n_quads> <seed>
// For random axis-aligned rectangles of every orientation (u along A or along B, both normal signs,
// corners and edges from tiny to huge, exact zeros), built as Quad's constructor builds them
// (Quad.cpp:6-17: n = cross(u, v), D = dot(normal, q), w = n / dot(n, n)), the kernel's decision
// lo[A] <= p[A] <= hi[A] && lo[B] <= p[B] <= hi[B], and its sign-word form (render.hip quad_aa),
// must equal Quad::Hit's interior test
// (Quad.cpp:27-36: alpha = dot(w, cross(pv, v)), beta = dot(w, cross(u, pv)), pv = p - q, both in
// [0, 1]) for hit points p around and on the bounds, at +-0, +-inf, NaN and far away, off the plane by
// rounding (compile.cpp RectAAWords: corners and edges within +-2^40, ray origins within +-2^100, so a hit
// point lies off the plane by up to about 2^-20 (|q| + |o|) = 2^80). Prints the
// number of decisions compared; exits non-zero at the first disagreement.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "scene.h"

namespace {
struct V3 {
  float x, y, z;
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
V3 cross(V3 x, V3 y) { return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }

uint32_t Bits(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return b;
}
bool reference_inside(V3 p, V3 q, V3 u, V3 v, V3 w) {
  const V3 pv = sub(p, q);
  const float alpha = dot(w, cross(pv, v)), beta = dot(w, cross(u, pv));
  return 0.0f <= alpha && alpha <= 1.0f && 0.0f <= beta && beta <= 1.0f;
}
}  // namespace

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
  std::uniform_real_distribution<float> unit(-1.0f, 1.0f);
  auto magnitude = [&]() {  // 0, tiny, ordinary, at the QUADAA limit (2^40) or huge, either sign
    const int c = (int)(rng() % 9);
    if (c == 0) return 0.0f;
    const float e = c == 1 ? -120.0f : (c == 2 ? 100.0f : (c == 3 ? 40.0f : (float)(rng() % 8) - 2.0f));
    return std::ldexp(unit(rng), (int)e);
  };
  long compared = 0;
  int rects = 0;
  for (int i = 0; i < n; i++) {
    const int k = (int)(rng() % 3), a = (k + 1) % 3, b = (k + 2) % 3;
    V3 q{magnitude(), magnitude(), magnitude()}, u{0, 0, 0}, v{0, 0, 0};
    float eu = magnitude(), ev = magnitude();
    if (eu == 0.0f) eu = 1.0f;
    if (ev == 0.0f) ev = -3.0f;
    const bool along_b = (rng() & 1) != 0;  // the mirrored orientation
    u[along_b ? b : a] = eu;
    v[along_b ? a : b] = ev;
    const V3 nn = cross(u, v);
    const float len = std::sqrt(dot(nn, nn));
    const float inv = 1.0f / len;
    const V3 normal{nn.x * inv, nn.y * inv, nn.z * inv};
    const float nd = dot(nn, nn);
    const V3 w{nn.x / nd, nn.y / nd, nn.z / nd};
    if (!(std::fabs(normal[k]) == 1.0f)) continue;  // (axis code K + 4 needs n[K] = +-1 exactly)
    float r[20] = {normal.x, normal.y, normal.z, dot(normal, q), q.x, q.y, q.z, 0, u.x, u.y, u.z, 0,
                   v.x,      v.y,      v.z,      0,              w.x, w.y, w.z, 0};
    r[19] = normal[k] * r[3];
    float t[8];
    if (!rt2::QuadAATestWords(r, k, t)) continue;  // general path (a word not finite)
    rects++;
    const float lo[2] = {t[1], t[3]}, hi[2] = {t[2], t[4]};
    // candidate coordinates per axis: the bounds and their neighbours, +-0, +-inf, NaN, far values,
    // random points over the rectangle and around it
    auto candidates = [&](int j, float* c) {
      int m = 0;
      const float l = lo[j], h = hi[j], qq = j == 0 ? q[a] : q[b];
      const float e = j == 0 ? (along_b ? ev : eu) : (along_b ? eu : ev);
      for (float x : {l, h}) {
        c[m++] = x;
        c[m++] = std::nextafter(x, INFINITY);
        c[m++] = std::nextafter(x, -INFINITY);
        c[m++] = std::nextafter(std::nextafter(x, INFINITY), INFINITY);
        c[m++] = std::nextafter(std::nextafter(x, -INFINITY), -INFINITY);
      }
      for (float x : {0.0f, -0.0f, INFINITY, -INFINITY, NAN, FLT_MAX, -FLT_MAX, 1e30f, -1e30f, qq, qq + e}) c[m++] = x;
      while (m < 40) c[m++] = qq + e * (1.5f * unit(rng) + 0.5f);
      return m;
    };
    float ca[40], cb[40];
    const int na = candidates(0, ca), nb = candidates(1, cb);
    for (int x = 0; x < na; x++)
      for (int y = 0; y < nb; y++) {
        V3 p = q;
        p[a] = ca[x];
        p[b] = cb[y];
        // the hit point's coordinate along the normal: on the plane up to the rounding of o + t d
        // (a few ulps of the origin's and the corner's coordinates; origins within +-2^100, so offsets
        // up to 2^80: exponents -44 .. 80)
        const float off = std::ldexp(unit(rng), (int)(rng() % 125) - 44);
        p[k] = (rng() & 3) == 0 ? q[k] : q[k] + off;
        const bool ref = reference_inside(p, q, u, v, w);
        const bool got = lo[0] <= p[a] && p[a] <= hi[0] && lo[1] <= p[b] && p[b] <= hi[1];
        // the kernel's form (render.hip quad_aa): the sign bits of the four rounded differences, for
        // every non-NaN p (a NaN p needs a non-finite ray, which the kernel never traces)
        const uint32_t rej = Bits(p[a] - lo[0]) | Bits(hi[0] - p[a]) | Bits(p[b] - lo[1]) | Bits(hi[1] - p[b]);
        const bool got_word = (rej >> 31) == 0u;
        compared++;
        if (ref != got || (!std::isnan(p[a]) && !std::isnan(p[b]) && ref != got_word)) {
          std::fprintf(stderr,
                       "mismatch: k=%d along_b=%d q=(%a %a %a) eu=%a ev=%a p=(%a %a %a) ref=%d got=%d bounds A [%a %a] B "
                       "[%a %a]\n",
                       k, (int)along_b, q.x, q.y, q.z, eu, ev, p.x, p.y, p.z, ref, got, lo[0], hi[0], lo[1], hi[1]);
          return 1;
        }
      }
  }
  std::printf("rects=%d decisions=%ld\n", rects, compared);
  return rects > n / 4 ? 0 : 1;
}
