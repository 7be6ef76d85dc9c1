// Host proof check of the box-level MakeBox test (boxaa.h BoxAATest, run by the kernel before a flagged
// MakeBox quad run, render.hip):
//   box_cert <n_boxes> <rays_per_box> <seed> <scratch_dir>
// Random boxes (MakeBox, Quad.hpp:34-50: corners from 2^-6 to 2^12, thin and flat boxes, boxes far from
// the origin) are written as a scene, loaded and compiled by the product (scene.cpp, compile.cpp), and
// for every box-flagged run of the compiled program the box test is compared with the six-face run it
// stands for, executed as the kernel executes it (render.hip quad_aa: each face's t, hit point and
// QUADAA rejection word; accepted iff key | rejection <= kmax, later faces winning ties), on rays that
// stress the certificate: entering through face interiors, edges and corners (on them and a few ulps
// beside), grazing faces, starting on a face as a hit point rounded off the plane (leaving, re-entering,
// along the face), starting inside, passing near the box, with zero direction components, intervals
// ending exactly at a face's t and every tmax. Whenever the box test certifies a lane, its answer (face,
// and the run's final kmax) must equal the run's, and whenever the medium form (BoxAAPair) certifies one,
// its two boundary answers must equal the two ConstantMedium queries' over the six faces (render.hip
// boundary_aa_pair): exits non-zero at the first disagreement. Prints the counts and the certified
// fractions per ray class.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "scene.h"
#define RT2_BOXAA_FN inline
#include "boxaa.h"

using namespace rt2;

namespace {
uint32_t B(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return b;
}
float F(uint32_t b) {
  float f;
  memcpy(&f, &b, 4);
  return f;
}
struct HostMath {
  static float div(float a, float b, float inv) {
    const float q = a * inv;
    return std::fma(std::fma(-b, q, a), inv, q);
  }
  static float min(float a, float b) { return std::fmin(a, b); }
  static float max(float a, float b) { return std::fmax(a, b); }
  static float min3(float a, float b, float c) { return std::fmin(std::fmin(a, b), c); }
  static float max3(float a, float b, float c) { return std::fmax(std::fmax(a, b), c); }
  static float amin3(float a, float b, float c) { return min3(std::fabs(a), std::fabs(b), std::fabs(c)); }
  static float amax3(float a, float b, float c) { return max3(std::fabs(a), std::fabs(b), std::fabs(c)); }
  static float med3(float a, float b, float c) { return std::fmax(std::fmin(a, b), std::fmin(std::fmax(a, b), c)); }
  static float fma(float a, float b, float c) { return std::fma(a, b, c); }
  static float abs(float a) { return std::fabs(a); }
  static uint32_t bits(float a) { return B(a); }
};
constexpr float kAbove1e8 = 0x1.5798f0p-27f;

struct Box {
  float w[kBoxAAWords];
  float mB;
  float tw[6][8];  // the run's QUADAA test words
  int axis[6];
};

// the six-face run as render.hip's quad-run loop executes it
void Run(const Box& bx, const float o[3], const float d[3], const float inv[3], float tmin, uint32_t& kmax, int& prim) {
  for (int j = 0; j < 6; j++) {
    const int k = bx.axis[j], a = (k + 1) % 3, b = (k + 2) % 3;
    const float* r = bx.tw[j];
    const float t = HostMath::div(r[0] - o[k], d[k], inv[k]);
    const float pa = o[a] + d[a] * t, pb = o[b] + d[b] * t;
    const uint32_t rej = (B(pa - r[1]) | B(r[2] - pa) | B(pb - r[3])) | (B(r[4] - pb) | B(std::fabs(d[k]) - kAbove1e8));
    const uint32_t x = (B(t) - B(tmin)) | (rej & 0x80000000u);
    if (x <= kmax) prim = j;
    kmax = std::min(kmax, x);
  }
}

// both boundary queries of ConstantMedium::Hit on the box as render.hip boundary_aa_pair runs them: each
// face's t by IEEE division and its QUADAA interior test (quad_aa_div), candidates in [-FLT_MAX,
// FLT_MAX]; t1 = the smallest, t2 = the smallest >= fl(t1 + 0.0001)
bool Pair(const Box& bx, const float o[3], const float d[3], float& t1, float& t2) {
  float c[6], m = INFINITY;
  for (int j = 0; j < 6; j++) {
    const int k = bx.axis[j], a = (k + 1) % 3, b = (k + 2) % 3;
    const float* r = bx.tw[j];
    const float t = (r[0] - o[k]) / d[k];
    const float pa = o[a] + d[a] * t, pb = o[b] + d[b] * t;
    const uint32_t rej = (B(pa - r[1]) | B(r[2] - pa) | B(pb - r[3])) | (B(r[4] - pb) | B(std::fabs(d[k]) - kAbove1e8));
    c[j] = ((int32_t)rej >= 0 && -FLT_MAX <= t && t <= FLT_MAX) ? t : INFINITY;
    m = std::fmin(m, c[j]);
  }
  if (!(m <= FLT_MAX)) return false;
  t1 = m;
  const float lb = (float)((double)m + 0.0001);
  float m2 = INFINITY;
  for (int j = 0; j < 6; j++) m2 = (lb <= c[j] && c[j] < m2) ? c[j] : m2;
  if (!(m2 <= FLT_MAX)) return false;
  t2 = m2;
  return true;
}

std::mt19937_64 rng;
float U(float lo, float hi) { return std::uniform_real_distribution<float>(lo, hi)(rng); }
float Ulps(float x, int n) {  // x moved by n ulps
  uint32_t b = B(x);
  if (x == 0.0f) return n == 0 ? x : std::ldexp((float)n, -149);
  if ((x > 0) == (n > 0)) b += (uint32_t)std::abs(n); else b -= (uint32_t)std::abs(n);
  return F(b);
}
void Dir(float d[3], bool unit) {
  float l;
  do {
    d[0] = U(-1, 1), d[1] = U(-1, 1), d[2] = U(-1, 1);
    l = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
  } while (l > 1.0f || l < 1e-6f);
  const float s = unit ? 1.0f / std::sqrt(l) : U(0.3f, 3.0f);
  for (int i = 0; i < 3; i++) d[i] *= s;
}
}  // namespace

int main(int argc, char** argv) {
  const int nbox = argc > 1 ? atoi(argv[1]) : 200;
  const int nray = argc > 2 ? atoi(argv[2]) : 20000;
  rng.seed(argc > 3 ? strtoull(argv[3], nullptr, 10) : 1);
  const std::string dir = argc > 4 ? argv[4] : "/tmp";
  // a scene of random boxes (v2 schema), loaded and compiled by the product
  std::string js = "{\"camera\": {\"center\": [0, 0, -10], \"look_at\": [0, 0, 0]}, \"materials\": [{\"type\": "
                   "\"lambertian\", \"albedo\": [0.5, 0.5, 0.5]}], \"primitives\": [";
  for (int i = 0; i < nbox; i++) {
    const int cls = i % 5;
    const float sc = std::ldexp(1.0f, (int)(rng() % 19) - 6);  // 2^-6 .. 2^12
    float a[3], e[3];
    for (int k = 0; k < 3; k++) {
      a[k] = U(-4, 4) * sc * (cls == 3 ? 64.0f : 1.0f);
      e[k] = U(0.05f, 2.0f) * sc;
    }
    if (cls == 1) e[(int)(rng() % 3)] *= 1e-3f;  // flat
    if (cls == 2) a[0] = std::round(a[0]), a[1] = std::round(a[1]), e[0] = std::round(e[0] + 1);  // integer corners
    char buf[256];
    snprintf(buf, sizeof buf, "%s{\"type\": \"box\", \"a\": [%.9g, %.9g, %.9g], \"b\": [%.9g, %.9g, %.9g], \"material\": 0}",
             i ? ", " : "", a[0], a[1], a[2], a[0] + e[0], a[1] + e[1], a[2] + e[2]);
    js += buf;
  }
  js += "], \"scene\": [";
  for (int i = 0; i < nbox; i++) js += (i ? ", " : "") + std::string("{\"primitive\": ") + std::to_string(i) + "}";
  js += "]}";
  const std::string path = dir + "/box_cert_scene.json";
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return 2;
  fputs(js.c_str(), f);
  fclose(f);
  Scene s;
  std::string err;
  CompiledScene c;
  unsetenv("RT2_BOX_AA");  // the default: box steps (compile.cpp SetBoxAA)
  if (!LoadScene(path, 1, s, err) || !CompileScene(s, c, err)) {
    fprintf(stderr, "scene: %s\n", err.c_str());
    return 2;
  }
  std::vector<Box> boxes;
  const size_t n = c.lin.size() / 4;
  for (size_t i = 0; i < n; i++) {
    if (c.lin[4 * i] != kQuad || !(c.lin[4 * i + 3] & kRunBoxFlag)) continue;
    Box bx;
    if ((c.lin[4 * i + 3] & kRunLenMask) != 6 || c.lin[4 * i + 1] != kBoxAARunCodes) {
      fprintf(stderr, "box run at step %zu is not a MakeBox run\n", i);
      return 1;
    }
    const size_t rec = c.lin[4 * i + 2];  // the run's first face record; the box record is the 2 before it
    memcpy(bx.w, &c.lind[4 * (rec - kBoxAARecords)], 4 * kBoxAAWords);
    bx.mB = c.lind[4 * (rec - kBoxAARecords) + 6];
    for (int j = 0; j < 6; j++) {
      if (c.lin[4 * (i + j) + 2] != rec + 5u * (uint32_t)j) {
        fprintf(stderr, "box run at step %zu: face records are not contiguous\n", i);
        return 1;
      }
      memcpy(bx.tw[j], &c.lind[4 * (size_t)c.lin[4 * (i + j) + 2]], 32);
      bx.axis[j] = (int)((kBoxAARunCodes >> (3 * j)) & 7u) - 4;
    }
    boxes.push_back(bx);
  }
  if ((int)boxes.size() < nbox * 2 / 5) {  // (faces whose normalized normal is not exactly +-1 take the general run)
    fprintf(stderr, "only %zu of %d boxes got a box step\n", boxes.size(), nbox);
    return 1;
  }
  const char* names[] = {"enter face", "enter edge/corner", "graze", "leave surface", "inside", "near miss", "zero comp"};
  long tot[7] = {}, cert[7] = {}, hits[7] = {}, pcert[7] = {};
  const float tmin = 0.001f;
  for (const Box& bx : boxes) {
    const float lo[3] = {bx.w[0], bx.w[2], bx.w[4]}, hi[3] = {bx.w[1], bx.w[3], bx.w[5]};
    float size = 0;
    for (int k = 0; k < 3; k++) size = std::max(size, hi[k] - lo[k]);
    for (int r = 0; r < nray; r++) {
      const int cls = r % 7;
      float o[3], d[3], p[3];
      const bool unit = (r / 7) % 2 == 0;
      // a point on the box surface: a face interior, or an edge / corner (moved by a few ulps)
      const int K = (int)(rng() % 3), side = (int)(rng() % 2);
      for (int k = 0; k < 3; k++) p[k] = U(lo[k], hi[k]);
      p[K] = side ? hi[K] : lo[K];
      if (cls == 1) {
        const int K2 = (K + 1 + (int)(rng() % 2)) % 3;
        p[K2] = Ulps((rng() % 2) ? hi[K2] : lo[K2], (int)(rng() % 9) - 4);
        if (rng() % 3 == 0) {
          const int K3 = 3 - K - K2;
          p[K3] = Ulps((rng() % 2) ? hi[K3] : lo[K3], (int)(rng() % 9) - 4);
        }
        p[K] = Ulps(p[K], (int)(rng() % 5) - 2);
      }
      float n[3] = {0, 0, 0};
      n[K] = side ? 1.0f : -1.0f;
      if (cls == 0 || cls == 1 || cls == 2) {  // from outside towards p
        float v[3];
        do Dir(v, true); while (v[0] * n[0] + v[1] * n[1] + v[2] * n[2] <= (cls == 2 ? 0.0f : 0.05f));
        if (cls == 2) {  // grazing: almost parallel to the face
          v[K] = n[K] * std::ldexp(U(0.5f, 1.0f), -(int)(rng() % 24));
        }
        const float L = size * std::ldexp(U(0.5f, 1.0f), (int)(rng() % 24) - 10);
        for (int k = 0; k < 3; k++) o[k] = p[k] + L * v[k];
        for (int k = 0; k < 3; k++) d[k] = p[k] - o[k];
        if (unit) {
          const float l = 1.0f / std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
          for (int k = 0; k < 3; k++) d[k] *= l;
        }
      } else if (cls == 3) {  // a hit point (o0 + d0 t, rounded as the kernel rounds it) leaving in any direction
        float o0[3], d0[3];
        Dir(d0, true);
        if (d0[0] * n[0] + d0[1] * n[1] + d0[2] * n[2] > 0) for (int k = 0; k < 3; k++) d0[k] = -d0[k];
        const float L = size * U(0.1f, 10.0f);
        for (int k = 0; k < 3; k++) o0[k] = p[k] - L * d0[k];
        const float t = (p[K] - o0[K]) / d0[K];
        for (int k = 0; k < 3; k++) o[k] = o0[k] + d0[k] * t;
        Dir(d, unit);
        if (rng() % 4 == 0) d[K] = n[K] * std::ldexp(U(0.5f, 1.0f), -(int)(rng() % 30));  // along the face
      } else if (cls == 4) {  // inside
        for (int k = 0; k < 3; k++) o[k] = U(lo[k], hi[k]);
        Dir(d, unit);
      } else if (cls == 5) {  // anywhere near
        for (int k = 0; k < 3; k++) o[k] = U(lo[k] - size, hi[k] + size);
        Dir(d, unit);
      } else {  // a zero (or tiny) direction component
        for (int k = 0; k < 3; k++) o[k] = U(lo[k] - size, hi[k] + size);
        Dir(d, unit);
        d[rng() % 3] = (rng() % 2) ? 0.0f : std::ldexp(1.0f, -(int)(rng() % 40) - 20);
      }
      float inv[3];
      for (int k = 0; k < 3; k++) inv[k] = 1.0f / d[k];
      bool finite = true;
      for (int k = 0; k < 3; k++) finite = finite && std::isfinite(inv[k]) && std::isfinite(o[k]) && std::isfinite(d[k]);
      if (!finite) continue;  // (the kernel's rays are finite; a +-0 component gives an infinite inv: below)
      // the interval: everything, a random end, or ending exactly at (or next to) one face's t
      float tmax = FLT_MAX;
      const int tk = (int)(rng() % 4);
      if (tk == 1) tmax = size * U(0.01f, 20.0f);
      if (tk >= 2) {
        const int j = (int)(rng() % 6), k = bx.axis[j];
        const float t = HostMath::div(bx.tw[j][0] - o[k], d[k], inv[k]);
        if (t > tmin && std::isfinite(t)) tmax = tk == 2 ? t : Ulps(t, (int)(rng() % 3) - 1);
        if (!(tmax >= tmin)) tmax = FLT_MAX;
      }
      if (!(tmax >= tmin)) tmax = tmin;  // (the kernel's interval is never empty: tmax >= tmin)
      const uint32_t kmax0 = B(tmax) - B(tmin);
      uint32_t kmax = kmax0;
      int prim = -1;
      Run(bx, o, d, inv, tmin, kmax, prim);
      const BoxAAResult res =
          BoxAATest<HostMath>(bx.w, bx.mB, o[0], o[1], o[2], d[0], d[1], d[2], inv[0], inv[1], inv[2], tmin);
      // the medium form: both boundary queries (boxaa.h BoxAAPair)
      {
        float q1 = 0, q2 = 0;
        const bool qok = Pair(bx, o, d, q1, q2);
        const BoxAAPairResult pr =
            BoxAAPair<HostMath>(bx.w, bx.mB, o[0], o[1], o[2], d[0], d[1], d[2], inv[0], inv[1], inv[2]);
        if (pr.cert) {
          pcert[cls]++;
          // the second query starts at fl(t1 + 0.0001), which is t1 itself for a t1 above 2^10 or so
          const float lb = (float)((double)pr.tin + 0.0001);
          const float bt2 = lb <= pr.tin ? pr.tin : pr.tout;
          const bool bok = pr.through && bt2 >= lb;
          // (t values compared as values: a +-0 t1 is clamped to tmin by the medium step either way)
          if (bok != qok || (qok && (q1 != pr.tin || q2 != bt2 || (q1 != 0.0f && B(q1) != B(pr.tin))))) {
            fprintf(stderr, "PAIR MISMATCH class %s: queries %d t1 %a t2 %a, box %d t1 %a t2 %a\n o = (%a %a %a) d = (%a %a %a)\n",
                    names[cls], (int)qok, q1, q2, (int)bok, pr.tin, bt2, o[0], o[1], o[2], d[0], d[1], d[2]);
            return 1;
          }
        }
      }
      tot[cls]++;
      if (prim >= 0) hits[cls]++;
      if (!res.cert) continue;
      cert[cls]++;
      const int bprim = res.x <= kmax0 ? (int)res.face : -1;
      const uint32_t bk = std::min(kmax0, res.x);
      if (bprim != prim || bk != kmax) {
        fprintf(stderr,
                "MISMATCH class %s: run face %d kmax %08x, box face %d kmax %08x (t %a)\n o = (%a %a %a) d = (%a %a %a) "
                "tmax %a\n box %a %a %a %a %a %a mB %a\n",
                names[cls], prim, kmax, bprim, bk, res.t, o[0], o[1], o[2], d[0], d[1], d[2], tmax, bx.w[0], bx.w[1],
                bx.w[2], bx.w[3], bx.w[4], bx.w[5], bx.mB);
        return 1;
      }
    }
  }
  long all = 0, allc = 0;
  for (int k = 0; k < 7; k++) {
    printf("%-18s rays %9ld  hits %9ld  pair certified %.5f  certified %.5f\n", names[k], tot[k], hits[k],
           tot[k] ? (double)pcert[k] / tot[k] : 0.0, tot[k] ? (double)cert[k] / tot[k] : 0.0);
    all += tot[k];
    allc += cert[k];
  }
  printf("boxes=%zu rays=%ld certified=%.5f\n", boxes.size(), all, (double)allc / all);
  return 0;
}
