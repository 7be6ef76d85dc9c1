// compile.cpp — flattens the host object graph (scene.h) into the node array the gfx950 kernel
// walks (rt2_layout.h), and proves the kernel's traversal-stack bound for the scene.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <unordered_map>
#include <unordered_set>

#include "scene.h"
#ifndef RT2_BOXAA_FN
#define RT2_BOXAA_FN inline
#endif
#include "boxaa.h"

namespace rt2 {

namespace {

// Quad::Hit's interior decision on one coordinate of a rectangle, 0 <= c1 ((p - q) c2) <= 1 with the
// float operations in that order (the rectangle forms below), as a function of the hit point's
// coordinate p alone.
bool CoordIn(float p, float q, float c1, float c2) {
  const float a = c1 * ((p - q) * c2);
  return 0.0f <= a && a <= 1.0f;
}
// Floats in the order of the reals as integers (-0 and +0 both 0) and back (0 -> +0).
int64_t OrderKey(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return (b & 0x80000000u) ? -(int64_t)(b & 0x7FFFFFFFu) : (int64_t)b;
}
float FromOrderKey(int64_t k) {
  const uint32_t b = k >= 0 ? (uint32_t)k : ((uint32_t)(-k) | 0x80000000u);
  float f;
  memcpy(&f, &b, 4);
  return f;
}
// The floats p with CoordIn(p, q, c1, c2) are one interval [lo, hi] of the reals' order, which holds
// q: p -> p - q, y -> y c2 and y -> c1 y are each monotone under round-to-nearest (non-decreasing,
// or non-increasing for a negative factor), so their composition g is monotone and {0 <= g <= 1} is
// an interval; a p whose p - q overflows gives +-inf or NaN, rejected, and lies beyond both ends; a
// zero's sign changes no decision (+-0 - q = -q; q = +-0 gives a +-0 product, accepted); g(q) = +-0.
// Found by bisection over the order keys with the host's float arithmetic, which rounds as the device
// does (SSE single precision, -ffp-contract=off). False when a word is not finite.
bool CoordRange(float q, float c1, float c2, float& lo, float& hi) {
  if (!std::isfinite(q) || !std::isfinite(c1) || !std::isfinite(c2) || !CoordIn(q, q, c1, c2)) return false;
  const int64_t k0 = OrderKey(q), kinf = 0x7F800000;  // CoordIn(+-inf) is false
  int64_t in = k0, out = kinf;
  while (out - in > 1) {
    const int64_t mid = in + (out - in) / 2;
    (CoordIn(FromOrderKey(mid), q, c1, c2) ? in : out) = mid;
  }
  hi = FromOrderKey(in);
  in = k0;
  out = -kinf;
  while (in - out > 1) {
    const int64_t mid = in - (in - out) / 2;
    (CoordIn(FromOrderKey(mid), q, c1, c2) ? in : out) = mid;
  }
  lo = FromOrderKey(in);
  if (lo == 0.0f) lo = -0.0f;  // (the same bound; p - lo is then +0 for p = +-0, render.hip quad_aa)
  return true;
}

// The 8 test words (sD, lo[A], hi[A], lo[B], hi[B], 0, 0, 0) of a unit-normal axis-aligned quad
// (QUAD record r, axis code K + 4, rt2_layout.h QUADAA) when it is a rectangle in the A-B plane (one
// edge along A, the other along B, the off-axis components exactly zero). Its Quad::Hit interior
// coordinates are alpha = w[K] ((p[A] - q[A]) v[B]) and beta = w[K] ((p[B] - q[B]) u[A]) (the cross
// products' other terms are signed zeros, which decide nothing); a quad whose u runs along B is taken
// as its mirror (u and v swapped, w negated), whose coordinates are (beta, alpha) of the original, bit
// for bit (a - b = -(b - a), negation commutes with rounding). Each coordinate's [0, 1] test is then
// lo <= p <= hi on the hit point's own coordinate (CoordRange): the kernel compares p[A] and p[B]
// with the four bounds instead of computing alpha and beta. False for other quads, or when a word is
// not finite (kept on the general path).
bool RectAAWords(const float* r, int k, float out[8]) {
  const int a = (k + 1) % 3, b = (k + 2) % 3;
  const float* u = r + 8;
  const float* v = r + 12;
  const float wk = r[16 + k];
  float c1, ca, cb;  // alpha = c1 ((p[A] - q[A]) ca), beta = c1 ((p[B] - q[B]) cb)
  if (u[b] == 0.0f && v[a] == 0.0f) {
    c1 = wk;
    ca = v[b];
    cb = u[a];
  } else if (u[a] == 0.0f && v[b] == 0.0f) {
    c1 = -wk;
    ca = u[b];
    cb = v[a];
  } else {
    return false;
  }
  // The reduction to one product per coordinate leaves out the cross products' off-axis terms, e.g.
  // w[A] (p[K] - q[K]) v[B]: +-0 while (p[K] - q[K]) v[B] is finite. p[K] is the hit point's coordinate
  // along the normal, off the plane by rounding only (|p[K] - q[K]| <= 2^-20 (|q[K]| + |o[K]|)), so
  // corners and edges within +-2^40 keep that product finite for every ray origin o within +-2^100
  // (the callers check it: Flattener::QuadAASpace, and the camera at every launch, capi.cpp).
  // Larger quads take the general path.
  for (int i = 0; i < 3; i++)
    if (!(std::fabs(r[4 + i]) <= 0x1p40f) || !(std::fabs(u[i]) <= 0x1p40f) || !(std::fabs(v[i]) <= 0x1p40f)) return false;
  float rec[8] = {r[19], 0, 0, 0, 0, 0, 0, 0};
  if (!CoordRange(r[4 + a], c1, ca, rec[1], rec[2]) || !CoordRange(r[4 + b], c1, cb, rec[3], rec[4])) return false;
  std::copy(rec, rec + 8, out);
  return true;
}

// The box step's record (boxaa.h) of a MakeBox run: six QUAD records (node layout, 20 floats each) in the
// order z+ x+ z- x- y+ y- (Quad.hpp:43-48), each a unit-normal rectangle with QUADAA test words. Words:
// the six planes per axis (lo, hi: the faces' sD); mB = 2^-21 B + s (B = max |plane|, s = the largest
// distance of a face's interior bound from the plane of the box it approximates, rounded up). False
// unless the faces are a box (lo < hi per axis, the lo faces at the face map's indices) with s <= 2^-20 B,
// the bound the kernel's margin assumes (DESIGN.md §4 "Box-level test").
bool BoxAAWordsOf(const float* const face[6], float out[6], float& mB) {
  static const int kAxis[6] = {2, 0, 2, 0, 1, 1};
  float tw[6][8];
  for (int j = 0; j < 6; j++) {
    uint32_t code;
    memcpy(&code, &face[j][11], 4);
    if (code != 4u + (uint32_t)kAxis[j] || !RectAAWords(face[j], kAxis[j], tw[j])) return false;
  }
  // planes: lo / hi face index per axis (boxaa.h kBoxAAFaceMap: x- 3, x+ 1, y- 5, y+ 4, z- 2, z+ 0)
  const int lo_face[3] = {(int)(kBoxAAFaceMap & 7u), (int)((kBoxAAFaceMap >> 6) & 7u), (int)((kBoxAAFaceMap >> 12) & 7u)};
  const int hi_face[3] = {(int)((kBoxAAFaceMap >> 3) & 7u), (int)((kBoxAAFaceMap >> 9) & 7u),
                          (int)((kBoxAAFaceMap >> 15) & 7u)};
  float plane[6];
  double B = 0;
  for (int k = 0; k < 3; k++) {
    plane[2 * k] = tw[lo_face[k]][0];
    plane[2 * k + 1] = tw[hi_face[k]][0];
    if (!(plane[2 * k] < plane[2 * k + 1])) return false;
    B = std::max(B, std::max(std::fabs((double)plane[2 * k]), std::fabs((double)plane[2 * k + 1])));
  }
  double slack = 0;
  for (int j = 0; j < 3; j++) {
    for (int f = 0; f < 6; f++) {
      const int k = kAxis[f];
      if (k == j) continue;
      const int slot = (j == (k + 1) % 3) ? 1 : 3;  // test words: sD, lo[A], hi[A], lo[B], hi[B]
      const float lo = tw[f][slot], hi = tw[f][slot + 1];
      slack = std::max(slack, std::fabs((double)lo - (double)plane[2 * j]));
      slack = std::max(slack, std::fabs((double)hi - (double)plane[2 * j + 1]));
    }
  }
  if (!(B > 0) || !(B <= 0x1p100) || !(slack <= 0x1p-20 * B)) return false;
  std::copy(plane, plane + 6, out);
  mB = std::nextafter((float)(0x1p-21 * B + slack), INFINITY);
  return true;
}

// The world-space normal of a quad under transforms, n_world = normalize(invM^T n) through the chain
// of enclosing transforms innermost first (Transform.cpp:85-86), with the float operations of
// render.hip resolve_hit in its order: each row product ((c.x n.x + c.y n.y) + c.z n.z) over the
// XFORM record's invM columns c0..c2 (threaded-program copies, parent link in c1.w), then glm's
// normalize v * (1 / sqrt(dot(v, v))). Every hit on the quad transforms the same normal, so the
// kernel reads it from the record (QUADAA words 12-14) instead of computing it per hit; the sign
// follows front_face (normalize(-v) = -normalize(v) and M(-n) = -(M n) exactly). The host build
// rounds every operation as the device does (-ffp-contract=off, SSE single precision, correctly
// rounded sqrt and division).
void WorldNormal(const std::vector<float>& lind, uint32_t xf, const float n_model[3], float out[3]) {
  float n[3] = {n_model[0], n_model[1], n_model[2]};
  for (uint32_t x = xf; x != kRefNone;) {
    const size_t xo = 4 * (size_t)(x & kOffsetMask);
    const float* c0 = &lind[xo];
    const float* c1 = &lind[xo + 4];
    const float* c2 = &lind[xo + 8];
    const float v[3] = {c0[0] * n[0] + c0[1] * n[1] + c0[2] * n[2], c1[0] * n[0] + c1[1] * n[1] + c1[2] * n[2],
                        c2[0] * n[0] + c2[1] * n[1] + c2[2] * n[2]};
    const float l2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const float s = 1.0f / std::sqrt(l2);
    n[0] = v[0] * s;
    n[1] = v[1] * s;
    n[2] = v[2] * s;
    uint32_t parent;
    memcpy(&parent, &c1[3], 4);
    x = parent;
  }
  out[0] = n[0];
  out[1] = n[1];
  out[2] = n[2];
}

struct Flattener {
  // the threaded program holds a test whose exactness needs ray origins within +-2^64 in world space
  // (QUADAA rectangles, box boundaries as QUADAA words, transforms about y: CompiledScene::origins_bounded)
  bool origins_bounded = false;
  const Scene& s;
  CompiledScene& out;
  std::unordered_map<int, uint32_t> ref_of;  // obj index -> node ref (DAG sharing)
  std::unordered_map<int, int> acc_depth;    // accelerated list obj -> tree depth
  std::unordered_map<uint32_t, uint32_t> lind_axis;  // program quad record -> axis code
  bool accelerate_lists = true;
  // depth of an accelerated list's tree beyond the balanced ceil(log2 n) that SAH splits may use
  // (CompileScene retries with 0 when the scene's traversal stack would not fit)
  int acc_depth_slack = kAccDepthSlack;
  std::unordered_map<int, bool> medium_memo;

  Flattener(const Scene& sc, CompiledScene& o) : s(sc), out(o) {}

  // BVH node records go to the prefix [0, out.hot_records), in breadth-first order, when it is
  // reserved (bvh_rank: BVH object -> breadth-first rank)
  const std::unordered_map<int, uint32_t>* bvh_rank = nullptr;
  uint32_t hot_next = 0;
  uint32_t Alloc(int records) {
    uint32_t off = (uint32_t)(out.nodes.size() / 4);
    out.nodes.resize(out.nodes.size() + 4 * (size_t)records, 0.0f);
    return off;
  }
  float* Rec(uint32_t off) { return out.nodes.data() + 4 * (size_t)off; }
  static float Bits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
  }
  void Put(uint32_t off, float a, float b, float c, float d) {
    float* r = Rec(off);
    r[0] = a;
    r[1] = b;
    r[2] = c;
    r[3] = d;
  }

  bool HasMedium(int i) {
    auto it = medium_memo.find(i);
    if (it != medium_memo.end()) return it->second;
    const Obj& o = s.objs[(size_t)i];
    bool r = false;
    switch (o.kind) {
      case kMedium: r = true; break;
      case kXform: r = HasMedium(o.child); break;
      case kBvh: r = HasMedium(o.left) || HasMedium(o.right); break;
      case kList:
        for (int c : o.children) r = r || HasMedium(c);
        break;
      default: break;
    }
    medium_memo[i] = r;
    return r;
  }

  // A leaf-only list of spheres, long enough, whose children's records are distinct and in list
  // order (so record-offset order is child order; the kernel breaks equal roots by it).
  bool AccelEligible(const Obj& o, const std::vector<uint32_t>& refs) const {
    if ((int)refs.size() < kListAccelMin) return false;
    for (size_t k = 0; k < refs.size(); k++) {
      if ((refs[k] >> 28) != kSphere) return false;
      if (k && (refs[k] & kOffsetMask) <= (refs[k - 1] & kOffsetMask)) return false;
    }
    for (int c : o.children)
      if (s.objs[(size_t)c].radius <= 0.0f) return false;
    return true;
  }
  // Binary tree over the children's boxes (SAH split, or the median on the longest centroid axis);
  // returns the subtree ref and its depth, at most `budget`: a split leaves each side at most
  // 2^(budget - 1) children, which the median split always does when hi - lo <= 2^budget, so
  // the SAH cannot build the lopsided (up to n - 1 levels deep) trees that clustered or graded
  // sphere sizes invite.
  uint32_t BuildAcc(std::vector<std::pair<int, uint32_t>>& items, size_t lo, size_t hi, int budget, int& depth) {
    if (hi - lo == 1) {
      depth = 0;
      return make_ref(kAccSphere, items[lo].second & kOffsetMask);
    }
    AABB box = s.objs[(size_t)items[lo].first].aabb;
    vec3 cmin(FLT_MAX, FLT_MAX, FLT_MAX), cmax(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (size_t k = lo; k < hi; k++) {
      const AABB& b = s.objs[(size_t)items[k].first].aabb;
      box = AABB(box, b);
      vec3 c((b.x.min + b.x.max) * 0.5f, (b.y.min + b.y.max) * 0.5f, (b.z.min + b.z.max) * 0.5f);
      cmin = vec3(std::min(cmin.x, c.x), std::min(cmin.y, c.y), std::min(cmin.z, c.z));
      cmax = vec3(std::max(cmax.x, c.x), std::max(cmax.y, c.y), std::max(cmax.z, c.z));
    }
    vec3 ext = cmax - cmin;
    int axis = ext.x >= ext.y && ext.x >= ext.z ? 0 : (ext.y >= ext.z ? 1 : 2);
    auto key_on = [&](int ax, const std::pair<int, uint32_t>& it) {
      const AABB& b = s.objs[(size_t)it.first].aabb;
      const Interval& iv = ax == 0 ? b.x : (ax == 1 ? b.y : b.z);
      return iv.min + iv.max;
    };
    auto less_on = [&](int ax) {
      return [&, ax](const auto& a, const auto& b) {
        const float ka = key_on(ax, a), kb = key_on(ax, b);
        return ka < kb || (ka == kb && a.second < b.second);
      };
    };
    size_t mid = lo + (hi - lo) / 2;
    // surface-area heuristic over centroid-sorted sweeps on each axis (book 2 +0.6 % over the
    // median split on the longest axis, which RT2_ACC_SAH=0 keeps)
    const char* se = getenv("RT2_ACC_SAH");
    if (!(se && atoi(se) == 0) && hi - lo > 2) {
      auto area = [](const AABB& b) {
        const float dx = b.x.max - b.x.min, dy = b.y.max - b.y.min, dz = b.z.max - b.z.min;
        return dx * dy + dy * dz + dz * dx;
      };
      double best = 1e300;
      const size_t n = hi - lo;
      const size_t side_max = budget - 1 >= 62 ? n : std::min(n, (size_t)1 << (budget - 1));
      std::vector<float> right(n);
      for (int ax = 0; ax < 3; ax++) {
        std::sort(items.begin() + (long)lo, items.begin() + (long)hi, less_on(ax));
        AABB acc = s.objs[(size_t)items[hi - 1].first].aabb;
        for (size_t k = n; k-- > 0;) {
          acc = AABB(acc, s.objs[(size_t)items[lo + k].first].aabb);
          right[k] = area(acc);
        }
        acc = s.objs[(size_t)items[lo].first].aabb;
        for (size_t k = 1; k < n; k++) {  // left = [lo, lo + k)
          acc = AABB(acc, s.objs[(size_t)items[lo + k - 1].first].aabb);
          if (k > side_max || n - k > side_max) continue;  // a side deeper than the budget allows
          const double c = (double)area(acc) * (double)k + (double)right[k] * (double)(n - k);
          if (c < best) best = c, axis = ax, mid = lo + k;
        }
      }
    }
    std::sort(items.begin() + (long)lo, items.begin() + (long)hi, less_on(axis));
    int dl = 0, dr = 0;
    uint32_t l = BuildAcc(items, lo, mid, budget - 1, dl);
    uint32_t r = BuildAcc(items, mid, hi, budget - 1, dr);
    depth = 1 + std::max(dl, dr);
    uint32_t off = Alloc(kBvhRecords);
    Put(off, box.x.min, box.y.min, box.z.min, Bits(l));
    Put(off + 1, box.x.max, box.y.max, box.z.max, Bits(r));
    out.acc_nodes++;
    return make_ref(kAccBvh + (uint32_t)axis, off);
  }
  uint32_t EmitListAcc(int i, const Obj& o, const std::vector<uint32_t>& refs) {
    std::vector<std::pair<int, uint32_t>> items;
    float rmin = FLT_MAX;
    AABB box = s.objs[(size_t)o.children[0]].aabb;
    for (size_t k = 0; k < refs.size(); k++) {
      const Obj& c = s.objs[(size_t)o.children[k]];
      items.emplace_back(o.children[k], refs[k]);
      rmin = std::min(rmin, c.radius);
      box = AABB(box, c.aabb);
    }
    int depth = 0, balanced = 0;
    while (((size_t)1 << balanced) < items.size()) balanced++;  // ceil(log2 n): the median tree's depth
    uint32_t root = BuildAcc(items, 0, items.size(), balanced + acc_depth_slack, depth);
    acc_depth[i] = depth;
    vec3 c((box.x.min + box.x.max) * 0.5f, (box.y.min + box.y.max) * 0.5f, (box.z.min + box.z.max) * 0.5f);
    float hx = box.x.max - c.x, hy = box.y.max - c.y, hz = box.z.max - c.z;
    float R = std::sqrt(hx * hx + hy * hy + hz * hz) * 1.001f + 1e-3f;
    uint32_t off = Alloc(2);
    // pad(L) = (k2 L + k1) L + k0: k2 = 4e-6 / r_min bounds the discriminant's float error
    // (~1e-6 a|oc|^2) turned into distance beyond the radius, with a 4x margin; k1, k0 cover the
    // rounding of roots and of the slab test
    Put(off, c.x, c.y, c.z, R);
    Put(off + 1, 4e-6f / rmin, 1e-5f, 1e-4f, Bits(root));
    out.acc_lists++;
    return make_ref(kListAcc, off);
  }

  bool IsLeafPrim(int i) const {
    NodeKind k = s.objs[(size_t)i].kind;
    return k == kQuad || k == kSphere;
  }

  // Emits object i (children first) and returns its ref. parent_xf = enclosing XFORM ref.
  uint32_t Emit(int i, uint32_t parent_xf, std::string& err) {
    auto it = ref_of.find(i);
    if (it != ref_of.end()) return it->second;
    const Obj& o = s.objs[(size_t)i];
    uint32_t ref = kRefNone;
    switch (o.kind) {
      case kQuad: {
        uint32_t off = Alloc(kQuadRecords);
        Put(off, o.n.x, o.n.y, o.n.z, o.d);
        Put(off + 1, o.q.x, o.q.y, o.q.z, Bits(o.material));
        // axis code (the kernel's exact axis-aligned tests): k+1 when n and w have exact zeros off
        // axis k; k+4 when in addition n[k] is exactly +-1 (then sign(n[k]) * D rides in w.w)
        uint32_t axis = 0;
        float signed_d = 0.0f;
        for (int k = 0; k < 3 && !axis; k++) {
          int a = (k + 1) % 3, b = (k + 2) % 3;
          if (o.n[a] == 0.0f && o.n[b] == 0.0f && o.w[a] == 0.0f && o.w[b] == 0.0f && o.n[k] != 0.0f) {
            axis = (uint32_t)k + 1;
            if (o.n[k] == 1.0f || o.n[k] == -1.0f) {
              axis = (uint32_t)k + 4;
              signed_d = o.n[k] * o.d;  // exact
            }
          }
        }
        Put(off + 2, o.u.x, o.u.y, o.u.z, Bits(axis));
        Put(off + 3, o.v.x, o.v.y, o.v.z, 0);
        Put(off + 4, o.w.x, o.w.y, o.w.z, signed_d);
        ref = make_ref(kQuad, off);
        out.quads++;
        break;
      }
      case kSphere: {
        uint32_t off = Alloc(kSphereRecords);
        Put(off, o.c0.x, o.c0.y, o.c0.z, o.radius);
        Put(off + 1, o.disp.x, o.disp.y, o.disp.z, Bits(o.material));
        ref = make_ref(kSphere, off);
        out.spheres++;
        break;
      }
      case kList: {
        std::vector<uint32_t> refs;
        bool leaf_only = true;
        for (int c : o.children) {
          uint32_t r = Emit(c, parent_xf, err);
          if (r == kRefNone) return kRefNone;
          refs.push_back(r);
          leaf_only = leaf_only && IsLeafPrim(c);
        }
        if (accelerate_lists && AccelEligible(o, refs)) {
          ref = EmitListAcc(i, o, refs);
          out.lists++;
          break;
        }
        int recs = 1 + (int)((refs.size() + 3) / 4);
        uint32_t off = Alloc(recs);
        Put(off, Bits((uint32_t)refs.size()), Bits(leaf_only ? kListLeafOnly : 0u), 0, 0);
        for (size_t k = 0; k < refs.size(); k++) Rec(off + 1 + (uint32_t)(k / 4))[k % 4] = Bits(refs[k]);
        ref = make_ref(kList, off);
        out.lists++;
        if (!leaf_only) out.features |= kFeatGenList;
        break;
      }
      case kXform: {
        // The XFORM's own record is allocated first so its ref can be the children's parent.
        uint32_t off = Alloc(kXformRecords);
        uint32_t self = make_ref(kXform, off);
        // children of an XFORM are emitted with this XFORM as their parent; a shared child that
        // was already emitted under another parent would get the wrong parent link
        if (ref_of.count(o.child) && s.objs[(size_t)o.child].kind == kXform) {
          err = "a transformed node is shared between two transforms";
          return kRefNone;
        }
        uint32_t child = Emit(o.child, self, err);
        if (child == kRefNone) return kRefNone;
        const mat4& iv = o.inv_model;
        const mat4& m = o.model;
        Put(off + 0, iv[0][0], iv[0][1], iv[0][2], Bits(child));
        Put(off + 1, iv[1][0], iv[1][1], iv[1][2], Bits(parent_xf));
        Put(off + 2, iv[2][0], iv[2][1], iv[2][2], 0);
        Put(off + 3, iv[3][0], iv[3][1], iv[3][2], 0);
        Put(off + 4, m[0][0], m[0][1], m[0][2], 0);
        Put(off + 5, m[1][0], m[1][1], m[1][2], 0);
        Put(off + 6, m[2][0], m[2][1], m[2][2], 0);
        Put(off + 7, m[3][0], m[3][1], m[3][2], 0);
        ref = self;
        out.xforms++;
        break;
      }
      case kMedium: {
        const Obj& b = s.objs[(size_t)o.child];
        bool ok = b.kind == kQuad || b.kind == kSphere;
        if (b.kind == kList) {
          ok = true;
          for (int c : b.children) ok = ok && IsLeafPrim(c);
        }
        if (!ok) {
          err = "constant_medium boundary must be a quad, a sphere or a box";
          return kRefNone;
        }
        uint32_t bref = Emit(o.child, parent_xf, err);
        if (bref == kRefNone) return kRefNone;
        uint32_t off = Alloc(kMediumRecords);
        Put(off, o.neg_inv_density, Bits(o.material), Bits(bref), 0);
        ref = make_ref(kMedium, off);
        out.media++;
        break;
      }
      case kBvh: {
        uint32_t l = Emit(o.left, parent_xf, err);
        if (l == kRefNone) return kRefNone;
        uint32_t r;
        if (o.left == o.right && !HasMedium(o.left)) {
          // Span-1 leaf (BVH.cpp:18-20) tests its object twice. The second test runs on
          // [min, rec.t] and provably leaves the hit record unchanged unless a ConstantMedium
          // (which draws a fresh random number per call) lies below, so it is skipped.
          r = kRefNone;
        } else {
          r = Emit(o.right, parent_xf, err);
          if (r == kRefNone) return kRefNone;
        }
        uint32_t off;
        if (bvh_rank) {
          off = bvh_rank->at(i) * (uint32_t)kBvhRecords;
          hot_next += (uint32_t)kBvhRecords;
        } else {
          off = Alloc(kBvhRecords);
        }
        const AABB& bb = o.aabb;
        Put(off, bb.x.min, bb.y.min, bb.z.min, Bits(l));
        Put(off + 1, bb.x.max, bb.y.max, bb.z.max, Bits(r));
        ref = make_ref(kBvh, off);
        out.bvh_nodes++;
        break;
      }
      default:
        err = "unknown object kind";
        return kRefNone;
    }
    ref_of[i] = ref;
    return ref;
  }

  // Threaded program (rt2_layout.h): pre-order of the tree the reference traverses, plus a copy of
  // every visited record in program order (`lind`), so consecutive steps read consecutive bytes.
  // References inside copied records (XFORM parent, medium boundary) point into `lind`.
  // Returns false when the program would exceed kLinearMaxSteps.
  // kLinearMaxSteps, or RT2_LINEAR_MAX_STEPS from the environment (ablation of the mode switch)
  static size_t LinearMaxSteps() {
    static const size_t v = [] {
      const char* e = getenv("RT2_LINEAR_MAX_STEPS");
      return e ? (size_t)strtoul(e, nullptr, 10) : (size_t)kLinearMaxSteps;
    }();
    return v;
  }
  uint32_t CopyRecords(uint32_t src_off, int n, std::vector<float>& lind) {
    uint32_t off = (uint32_t)(lind.size() / 4);
    const float* r = out.nodes.data() + 4 * (size_t)src_off;
    lind.insert(lind.end(), r, r + 4 * n);
    return off;
  }
  // copies a medium boundary (quad, sphere, or a leaf-only list) and returns its lind ref
  uint32_t CopyBoundary(int i, std::vector<float>& lind) {
    const Obj& o = s.objs[(size_t)i];
    uint32_t src = ref_of.at(i) & kOffsetMask;
    if (o.kind == kQuad) return make_ref(kQuad, CopyRecords(src, kQuadRecords, lind));
    if (o.kind == kSphere) return make_ref(kSphere, CopyRecords(src, kSphereRecords, lind));
    std::vector<uint32_t> kids;
    for (int c : o.children) kids.push_back(CopyBoundary(c, lind));
    uint32_t off = CopyRecords(src, 1 + (int)((kids.size() + 3) / 4), lind);
    for (size_t k = 0; k < kids.size(); k++) lind[4 * (off + 1 + k / 4) + k % 4] = Bits(kids[k]);
    return make_ref(kList, off);
  }
  // A medium boundary that is a list of at most kBoundaryAAMax unit-normal axis-aligned quads (a box
  // in its own space, MakeBox) also gets its children as consecutive QUADAA test words (8 words
  // each, rt2_layout.h), right after the medium's record, so that a kernel loads the whole boundary
  // at once with no child-ref indirection (two dependent scalar loads per quad and boundary query
  // otherwise). A MakeBox boundary (six faces, boxaa.h BoxAAWordsOf) also gets its box record after the
  // quads' words and kBoundaryBoxFlag (the medium step's box-level test of both boundary queries,
  // render.hip medium_t_lin). Returns the medium record's word 3 (kBoundaryAAFlag | kBoundaryBoxFlag |
  // n << 24 | axis codes, 3 bits per child), or 0 (general path only). The general copy of the boundary
  // is kept for kernels without the box path.
  uint32_t BoundaryAA(int i, uint32_t parent_xf, std::vector<float>& lind) {
    const Obj& o = s.objs[(size_t)i];
    if (o.kind != kList || o.children.empty() || o.children.size() > kBoundaryAAMax) return 0;
    if (!QuadAASpace(parent_xf, lind)) return 0;
    uint32_t codes = 0;
    std::vector<float> words;
    for (size_t k = 0; k < o.children.size(); k++) {
      const int c = o.children[k];
      if (s.objs[(size_t)c].kind != kQuad) return 0;
      const float* r = out.nodes.data() + 4 * (size_t)(ref_of.at(c) & kOffsetMask);
      uint32_t axis;
      memcpy(&axis, &r[11], 4);
      if (axis < 4 || axis > 6) return 0;
      float rec[8];
      if (!RectAAWords(r, (int)axis - 4, rec)) return 0;
      words.insert(words.end(), rec, rec + 8);
      codes |= (axis - 4) << (3 * k);
    }
    lind.insert(lind.end(), words.begin(), words.end());
    origins_bounded = true;
    uint32_t box = 0;
    if (box_aa && o.children.size() == 6) {  // a MakeBox: its box record (boxaa.h BoxAAPair) follows
      const float* faces[6];
      for (int j = 0; j < 6; j++) faces[j] = out.nodes.data() + 4 * (size_t)(ref_of.at(o.children[(size_t)j]) & kOffsetMask);
      float bw[6], mB;
      if (BoxAAWordsOf(faces, bw, mB)) {
        float rec[4 * kBoxAARecords] = {};
        std::copy(bw, bw + 6, rec);
        rec[6] = mB;
        lind.insert(lind.end(), rec, rec + 4 * kBoxAARecords);
        box = kBoundaryBoxFlag;
        out.box_steps++;
      }
    }
    return kBoundaryAAFlag | box | ((uint32_t)o.children.size() << 24) | codes;
  }
  // An accelerated list's tree in the threaded program: ACCBVH steps (padded box, skip = index
  // after the subtree) near child first, ACCSPHERE steps with aux = the sphere's record offset in
  // the node array, which is the list's child order (the kernel breaks equal roots by it).
  // `octant` (bit k: the ray direction is negative along axis k) orders each node's children for
  // such rays: the child with the larger centroids first along a split axis the ray runs down.
  bool LinearizeAcc(uint32_t ref, std::vector<uint32_t>& lin, std::vector<float>& lind, uint32_t octant = 0) {
    if (lin.size() / 4 >= LinearMaxSteps()) return false;
    const uint32_t kind = ref >> 28, off = ref & kOffsetMask;
    if (kind == kAccSphere) {
      lin.insert(lin.end(), {kAccSphere, 0u, CopyRecords(off, kSphereRecords, lind), off});
      return true;
    }
    const size_t me = lin.size() / 4;
    lin.insert(lin.end(), {kAccBvh, 0u, CopyRecords(off, kBvhRecords, lind), 0u});
    uint32_t near_ref, far_ref;
    memcpy(&near_ref, &out.nodes[4 * (size_t)off + 3], 4);
    memcpy(&far_ref, &out.nodes[4 * (size_t)off + 7], 4);
    if ((octant >> (kind - kAccBvh)) & 1u) std::swap(near_ref, far_ref);
    if (!LinearizeAcc(near_ref, lin, lind, octant) || !LinearizeAcc(far_ref, lin, lind, octant)) return false;
    lin[4 * me + 1] = (uint32_t)(lin.size() / 4);
    return true;
  }
  // Whether rays in the space of transform chain xf (innermost first) start within +-2^100, the bound
  // RectAAWords' reduction needs: world-space origins (the camera, checked at every launch, and hit
  // points on the geometry) lie within +-2^64 when the scene does, and each transform from the outermost
  // in maps a bound B to |invM| B + |translation| (row sums of the inverse's 3x3 part, in double).
  bool QuadAASpace(uint32_t xf, const std::vector<float>& lind) const {
    const AABB& w = s.objs[(size_t)s.root].aabb;
    const double lim = 0x1p64;
    for (float v : {w.x.min, w.x.max, w.y.min, w.y.max, w.z.min, w.z.max})
      if (!(std::fabs((double)v) <= lim)) return false;
    std::vector<uint32_t> chain;
    for (uint32_t x = xf; x != kRefNone;) {
      chain.push_back(x & kOffsetMask);
      uint32_t parent;
      memcpy(&parent, &lind[4 * (size_t)(x & kOffsetMask) + 7], 4);
      x = parent;
    }
    double b = lim;
    for (size_t k = chain.size(); k-- > 0;) {
      const float* m = &lind[4 * (size_t)chain[k]];  // invM columns c0..c3 (records 0-3, xyz)
      double nb = 0;
      for (int row = 0; row < 3; row++) {
        const double r = std::fabs((double)m[row]) + std::fabs((double)m[4 + row]) + std::fabs((double)m[8 + row]);
        nb = std::max(nb, r * b + std::fabs((double)m[12 + row]));
      }
      if (!(nb <= 0x1p100)) return false;
      b = nb;
    }
    return true;
  }
  // A transform about the y axis (every scene transform of the reference's files: ParseTransform's
  // rotation is angleAxis about a y axis, Serialize.cpp:106-132): the off-pattern entries of M^-1 and
  // of M (col0.y, col1.x, col1.z, col2.y) are exactly +-0, so each of their products with a finite
  // coordinate is a +-0 summand, and the kernel leaves them out (rt2_layout.h kXformYAxis). A +-0
  // summand changes a sum only when every other summand is zero too, and then only the sign of the
  // zero; a zero's sign reaches no decision and no nonzero value of the path (DESIGN.md §4
  // "Transforms about y"). The coordinates must be finite (0 * inf is NaN): the scene and the
  // transformed object lie within +-2^100, so every ray origin (the camera, a hit point) is finite.
  bool YAxisPattern(int i, const std::vector<float>& lind, uint32_t off) const {
    const float* r = &lind[4 * (size_t)off];
    for (int c : {0, 4}) {  // M^-1 (records 0-3), M (records 4-7)
      const float* m = r + 4 * c;
      if (!(m[1] == 0.0f && m[4] == 0.0f && m[6] == 0.0f && m[9] == 0.0f)) return false;
      for (int k = 0; k < 12; k += 4)  // (the 3x3 part: its products stay finite)
        for (int j = 0; j < 3; j++)
          if (!(std::fabs(m[k + j]) <= 0x1p10f)) return false;
    }
    auto inside = [](const AABB& b) {
      const float lim = 0x1p100f;
      return std::fabs(b.x.min) <= lim && std::fabs(b.x.max) <= lim && std::fabs(b.y.min) <= lim &&
             std::fabs(b.y.max) <= lim && std::fabs(b.z.min) <= lim && std::fabs(b.z.max) <= lim;
    };
    const Obj& o = s.objs[(size_t)i];
    return inside(o.aabb) && inside(s.objs[(size_t)o.child].aabb) && inside(s.objs[(size_t)s.root].aabb);
  }
  // Box-level steps (boxaa.h) for every MakeBox run whose faces take the QUADAA test (DESIGN.md §4
  // "Box-level test"). RT2_BOX_AA=0 keeps every MakeBox a plain six-face run (the A/B baseline).
  bool box_aa = true;
  std::vector<uint32_t> box_runs;  // first quad step of each MakeBox run with a box record
  void SetBoxAA() {
    const char* e = getenv("RT2_BOX_AA");
    box_aa = !(e && atoi(e) == 0);
  }
  // A list that is a MakeBox whose faces all take the QUADAA rectangle test in this space: its box words
  bool BoxList(const Obj& o, uint32_t parent_xf, const std::vector<float>& lind, float bw[6], float& mB) const {
    if (o.kind != kList || o.children.size() != 6 || !QuadAASpace(parent_xf, lind)) return false;
    const float* faces[6];
    for (int j = 0; j < 6; j++) {
      const int c = o.children[(size_t)j];
      if (s.objs[(size_t)c].kind != kQuad) return false;
      faces[j] = out.nodes.data() + 4 * (size_t)(ref_of.at(c) & kOffsetMask);
    }
    return BoxAAWordsOf(faces, bw, mB);
  }
  bool ContainsAccList(int i) const {
    const Obj& o = s.objs[(size_t)i];
    if (o.kind == kList && acc_depth.count(i)) return true;
    if (o.kind == kList)
      for (int c : o.children)
        if (ContainsAccList(c)) return true;
    return false;
  }
  bool Linearize(int i, uint32_t parent_xf, std::vector<uint32_t>& lin, std::vector<float>& lind, int xf_depth = 0) {
    if (lin.size() / 4 >= LinearMaxSteps()) return false;
    const Obj& o = s.objs[(size_t)i];
    uint32_t src = ref_of.at(i) & kOffsetMask;
    auto emit = [&](uint32_t kind, uint32_t rec, uint32_t aux) {
      lin.insert(lin.end(), {kind, 0u, rec, aux});
      return lin.size() / 4 - 1;
    };
    switch (o.kind) {
      case kBvh: {
        size_t me = emit(kBvh, CopyRecords(src, kBvhRecords, lind), 0);
        if (!Linearize(o.left, parent_xf, lin, lind, xf_depth)) return false;
        if (!(o.left == o.right && !HasMedium(o.left))) {
          if (!Linearize(o.right, parent_xf, lin, lind, xf_depth)) return false;
        }
        lin[4 * me + 1] = (uint32_t)(lin.size() / 4);
        return true;
      }
      case kList:
        if (acc_depth.count(i)) {  // LISTACC step (the ray's padding), then its tree in pre-order
          // LISTACC step (aux = steps per copy of the tree, skip = the index after the copies), then
          // the tree in pre-order, and, when they fit, seven more copies, one per ray-direction
          // octant, each visiting a node's children nearer-first for rays of that octant (the list's
          // answer does not depend on the order: rt2_layout.h LISTACC). RT2_ACC_OCTANTS=0: one copy.
          const size_t me = emit(kListAcc, CopyRecords(src, 2, lind), 0);
          uint32_t root;
          memcpy(&root, &out.nodes[4 * (size_t)src + 7], 4);
          const size_t first = lin.size() / 4;
          if (!LinearizeAcc(root, lin, lind)) return false;
          const uint32_t copy = (uint32_t)(lin.size() / 4 - first);
          lin[4 * me + 3] = copy;
          const char* oe = getenv("RT2_ACC_OCTANTS");
          if (!(oe && atoi(oe) == 0) && lin.size() / 4 + 7 * (size_t)copy <= LinearMaxSteps())
            for (uint32_t oct = 1; oct < 8; oct++)
              if (!LinearizeAcc(root, lin, lind, oct)) return false;
          lin[4 * me + 1] = (uint32_t)(lin.size() / 4);
          return true;
        }
        {
          // a MakeBox list (Quad.hpp:34-50) whose six faces take the QUADAA test: its box record (boxaa.h:
          // the six planes, then mB, padded to 2 records) right before the faces' records, and its first quad
          // step noted; after the run pass its run (exactly these six quads) gets the box flag (aux bit
          // 31), and the kernel runs the box-level test before the six-face run
          if (box_aa) {
            float bw[6], mB;
            if (BoxList(o, parent_xf, lind, bw, mB)) {
              float rec[4 * kBoxAARecords] = {};
              std::copy(bw, bw + 6, rec);
              rec[6] = mB;
              lind.insert(lind.end(), rec, rec + 4 * kBoxAARecords);
              box_runs.push_back((uint32_t)(lin.size() / 4));
            }
          }
          for (int c : o.children)
            if (!Linearize(c, parent_xf, lin, lind, xf_depth)) return false;
          return true;
        }
      case kXform: {
        uint32_t off = CopyRecords(src, kXformRecords, lind);
        lind[4 * (off + 1) + 3] = Bits(parent_xf);
        const bool yaxis = YAxisPattern(i, lind, off);
        origins_bounded = origins_bounded || yaxis;
        lind[4 * (off + 2) + 3] = Bits(yaxis ? kXformYAxis : 0u);
        uint32_t self = make_ref(kXform, off);
        if (xf_depth >= kLinearMaxXformDepth) return false;  // the kernel nests one loop per level
        size_t me = emit(kXform, off, 0);
        out.lin_xform_depth = std::max(out.lin_xform_depth, xf_depth + 1);
        if (!Linearize(o.child, self, lin, lind, xf_depth + 1)) return false;
        lin[4 * me + 1] = (uint32_t)(lin.size() / 4);  // index of the matching exit step
        // exit step: skip = the end of the transform's record range [off + kXformRecords, end) (the
        // records of every primitive under it follow its own record)
        const size_t ex = emit(kXformExit, off, parent_xf);
        lin[4 * ex + 1] = (uint32_t)(lind.size() / 4);
        return true;
      }
      case kMedium: {
        if (ContainsAccList(o.child)) return false;  // boundary copies hold plain lists only
        uint32_t off = CopyRecords(src, kMediumRecords, lind);
        lind[4 * off + 3] = Bits(BoundaryAA(o.child, parent_xf, lind));  // the box words follow the record
        uint32_t b = CopyBoundary(o.child, lind);
        lind[4 * off + 2] = Bits(b);
        emit(kMedium, off, 0);
        return lin.size() / 4 <= LinearMaxSteps();
      }
      case kQuad: {
        uint32_t off = CopyRecords(src, kQuadRecords, lind);
        uint32_t axis;
        memcpy(&axis, &lind[4 * (off + 2) + 3], 4);
        const float* r = out.nodes.data() + 4 * (size_t)src;
        float test[8];
        // a unit-normal quad that is not a rectangle in its plane takes the axis-aligned test
        // with division (code K + 1: the same decision and t)
        if (axis >= 4 && axis <= 6 && !(QuadAASpace(parent_xf, lind) && RectAAWords(r, (int)axis - 4, test))) axis -= 3;
        lind_axis[off] = axis;
        if (axis >= 4 && axis <= 6) {  // QUADAA layout (rt2_layout.h)
          origins_bounded = true;
          const float n[3] = {r[0], r[1], r[2]}, d = r[3], q[3] = {r[4], r[5], r[6]}, mat = r[7];
          float w[3] = {q[0], q[1], q[2]};
          if (parent_xf != kRefNone) WorldNormal(lind, parent_xf, n, w);  // replaces q (unused here)
          const float rec[12] = {n[0], n[1], n[2], d, w[0], w[1], w[2], mat, Bits(axis), Bits(parent_xf), 0, 0};
          std::copy(test, test + 8, lind.begin() + 4 * (long)off);
          std::copy(rec, rec + 12, lind.begin() + 4 * (long)off + 8);
        } else {
          lind[4 * (off + 3) + 3] = Bits(parent_xf);  // enclosing transform of this occurrence
        }
        emit(kQuad, off, 0);
        return lin.size() / 4 <= LinearMaxSteps();
      }
      default:  // sphere
        emit(kSphere, CopyRecords(src, kSphereRecords, lind), 0);
        return lin.size() / 4 <= LinearMaxSteps();
    }
  }

  // Stack entries the kernel holds for this subtree once its ref has been popped.
  int StackNeed(int i, int& depth_out) {
    const Obj& o = s.objs[(size_t)i];
    depth_out = 0;
    switch (o.kind) {
      case kBvh: {
        int dl = 0, dr = 0;
        int nl = StackNeed(o.left, dl);
        int nr = StackNeed(o.right, dr);
        depth_out = 1 + std::max(dl, dr);
        return std::max(2, std::max(1 + nl, nr));
      }
      case kList: {
        auto acc = acc_depth.find(i);
        if (acc != acc_depth.end()) return acc->second;  // one pushed sibling per tree level
        bool leaf_only = true;
        for (int c : o.children) leaf_only = leaf_only && IsLeafPrim(c);
        if (leaf_only) return 0;
        int n = (int)o.children.size(), need = n;
        for (int k = 0; k < n; k++) {
          int d = 0;
          need = std::max(need, (n - 1 - k) + StackNeed(o.children[(size_t)k], d));
        }
        return need;
      }
      case kXform: {
        int d = 0;
        return std::max(2, 1 + StackNeed(o.child, d));
      }
      default:
        return 0;  // quad / sphere / medium (boundary evaluated inline)
    }
  }
};

void PackMaterials(const Scene& s, CompiledScene& out) {
  for (const MaterialDesc& m : s.materials) {
    uint32_t type = m.type, tex = m.tex_idx;
    float ri_inv = (float)(1.0 / (double)m.refraction_index);
    float rec[8];
    memcpy(&rec[0], &type, 4);
    rec[1] = m.albedo.x;
    rec[2] = m.albedo.y;
    rec[3] = m.albedo.z;
    rec[4] = m.fuzz;
    rec[5] = m.refraction_index;
    memcpy(&rec[6], &tex, 4);
    rec[7] = ri_inv;
    out.materials.insert(out.materials.end(), rec, rec + 8);
  }
}

void PackTextures(const Scene& s, CompiledScene& out) {
  for (const TextureDesc& t : s.textures) {
    uint32_t u[12] = {0};
    float* f = reinterpret_cast<float*>(u);
    u[0] = t.type;
    f[1] = t.albedo.x;
    f[2] = t.albedo.y;
    f[3] = t.albedo.z;
    f[4] = t.type == kTexChecker ? t.inv_scale : t.scale;
    u[5] = t.even;
    u[6] = t.odd;
    u[7] = (uint32_t)t.noise_type;
    if (t.type == kTexNoise) {
      u[8] = (uint32_t)(out.perlin_vec.size() / 4);
      u[9] = (uint32_t)out.perlin_perm.size();
      u[10] = (uint32_t)t.point_count;
      for (const vec3& g : t.perlin_vec) {
        out.perlin_vec.push_back(g.x);
        out.perlin_vec.push_back(g.y);
        out.perlin_vec.push_back(g.z);
        out.perlin_vec.push_back(0.0f);
      }
      out.perlin_perm.insert(out.perlin_perm.end(), t.perm_x.begin(), t.perm_x.end());
      out.perlin_perm.insert(out.perlin_perm.end(), t.perm_y.begin(), t.perm_y.end());
      out.perlin_perm.insert(out.perlin_perm.end(), t.perm_z.begin(), t.perm_z.end());
    }
    out.textures.insert(out.textures.end(), f, f + 12);
  }
}

}  // namespace

bool QuadAATestWords(const float* r, int k, float out[8]) { return RectAAWords(r, k, out); }
bool BoxAAWords(const float* const faces[6], float out[6], float& mB) { return BoxAAWordsOf(faces, out, mB); }

bool CompileScene(const Scene& s, CompiledScene& out, std::string& err, bool accelerate_lists) {
  return CompileSceneWith(s, out, err, accelerate_lists, kAccDepthSlack);
}

bool CompileSceneWith(const Scene& s, CompiledScene& out, std::string& err, bool accelerate_lists,
                      int acc_depth_slack) {
  out = CompiledScene();
  if (s.root < 0) {
    err = "scene has no BVH root";
    return false;
  }
  // BVH node records come first, in breadth-first order from the root, so any prefix of the record
  // array holds the top levels of the tree (the stack traversal stages such a prefix in LDS when
  // the whole scene does not fit, kModeStackHybrid); everything else follows. Record contents are
  // the same in any order.
  std::unordered_map<int, uint32_t> rank;
  {
    std::vector<int> q{s.root};
    std::unordered_set<int> seen{s.root};
    auto push = [&](int c) {
      if (c >= 0 && seen.insert(c).second) q.push_back(c);
    };
    for (size_t h = 0; h < q.size(); h++) {
      const Obj& o = s.objs[(size_t)q[h]];
      if (o.kind == kBvh) {
        rank.emplace(q[h], (uint32_t)rank.size());
        push(o.left);
        push(o.right);
      } else if (o.kind == kList) {
        for (int c : o.children) push(c);
      } else if (o.kind == kXform || o.kind == kMedium) {
        push(o.child);
      }
    }
  }
  const uint32_t hot = (uint32_t)rank.size() * (uint32_t)kBvhRecords;
  out.hot_records = hot;
  out.nodes.assign(4 * (size_t)hot, 0.0f);
  Flattener fl(s, out);
  fl.accelerate_lists = accelerate_lists;
  fl.acc_depth_slack = acc_depth_slack;
  fl.bvh_rank = &rank;
  out.root = fl.Emit(s.root, kRefNone, err);
  if (out.root == kRefNone) return false;
  if (fl.hot_next != hot) {
    err = "internal: BVH record count changed between passes";
    return false;
  }
  int depth = 0;
  out.max_stack = std::max(1, fl.StackNeed(s.root, depth));
  out.bvh_depth = depth;
  if (out.max_stack > kTraversalStack && out.acc_lists > 0 && acc_depth_slack > 0) {
    // the SAH's extra tree depth pushed the stack past the kernel's: balanced trees instead (a
    // performance heuristic never makes a scene fail to load)
    return CompileSceneWith(s, out, err, accelerate_lists, 0);
  }
  if (out.nodes.size() / 4 > kOffsetMask) {
    err = "scene too large for 28-bit node offsets";
    return false;
  }
  fl.SetBoxAA();
  if (!fl.Linearize(s.root, kRefNone, out.lin, out.lind)) {
    out.lin.clear();
    out.lind.clear();
  }
  out.origins_bounded = fl.origins_bounded && !out.lin.empty();
  // The stack traversal needs max_stack entries per lane; the threaded program needs none, so a
  // deeper scene still loads when it has one (and then always runs threaded).
  out.stack_ok = out.max_stack <= kTraversalStack;
  if (!out.stack_ok && out.lin.empty()) {
    err = "scene needs a traversal stack of " + std::to_string(out.max_stack) + " entries (kernel has " +
          std::to_string(kTraversalStack) + ") and has no threaded program";
    return false;
  }
  // Quad runs: for a quad step, aux = number of consecutive quad steps starting there with no
  // skip target inside the run (so every lane that reaches the run's first step walks all of it).
  {
    size_t n = out.lin.size() / 4;
    std::vector<char> entry(n + 1, 0);
    for (size_t i = 0; i < n; i++)
      if (out.lin[4 * i] == kBvh || out.lin[4 * i] == kAccBvh) entry[out.lin[4 * i + 1]] = 1;
    for (uint32_t b : fl.box_runs) entry[b] = entry[b + 6] = 1;  // a box's run is its six quads exactly
    for (size_t i = n; i-- > 0;) {
      if (out.lin[4 * i] != kQuad) continue;
      uint32_t run = 1;
      if (i + 1 < n && out.lin[4 * (i + 1)] == kQuad && !entry[i + 1])
        run = std::min(out.lin[4 * (i + 1) + 3] + 1, kLinearMaxRun);
      out.lin[4 * i + 3] = run;
    }
    // axis codes of each run's quads, 3 bits each, then a 1 bit (the kernel's loop ends when the
    // codes shifted past the last quad equal 1), in the skip word
    for (size_t i = 0; i < n; i++) {
      if (out.lin[4 * i] != kQuad) continue;
      uint32_t codes = 0;
      const uint32_t run = out.lin[4 * i + 3];
      for (uint32_t k = 0; k < run; k++) codes |= fl.lind_axis.at(out.lin[4 * (i + k) + 2]) << (3 * k);
      out.lin[4 * i + 1] = codes | (1u << (3 * run));
    }
    for (uint32_t b : fl.box_runs) {
      if (out.lin[4 * b] != kQuad || out.lin[4 * b + 3] != 6u || out.lin[4 * b + 1] != kBoxAARunCodes) {
        err = "internal: a box's quads did not form its run";
        return false;
      }
      out.lin[4 * b + 3] |= kRunBoxFlag;
      out.box_steps++;
    }
  }
  // Wide program: each 16-byte step entry followed by the first 48 bytes of its record (a whole BVH
  // node or QUADAA quad), so one 64-byte scalar load fetches both
  // plus one entry past the last step, kind kProgramEnd: the wave's next step index reaches n when
  // every lane is done, and the kernel reads that entry's kind instead of comparing the index with n
  {
    size_t n = out.lin.size() / 4;
    out.lin_wide.assign(16 * (n + 1), 0u);
    out.lin_wide[16 * n] = kProgramEnd;
    for (size_t i = 0; i < n; i++) {
      for (int k = 0; k < 4; k++) out.lin_wide[16 * i + k] = out.lin[4 * i + k];
      const size_t rec = 4 * (size_t)out.lin[4 * i + 2];
      for (size_t k = 0; k < 12 && rec + k < out.lind.size(); k++) memcpy(&out.lin_wide[16 * i + 4 + k], &out.lind[rec + k], 4);
    }
    // BVH steps in the wide program: word 2 = the step after a hit, word 3 = the step after a hit
    // whose paired box misses. A BVH step followed by a BVH step (its near child: pre-order puts
    // it next, and no skip index lands on it) also carries that child's box in the words the
    // node's record leaves unused (7, 11-15): one step tests both boxes with the same tmax the
    // child's own step would see, a lane that hits both goes on to the child's first child, and
    // the child's step is never executed. Down a chain of near children every other step drops
    // out. Paired only in scenes with spheres (their kernels carry the second test: book 1 +2.9 %,
    // book 2 +2.5 % against single-box steps; the Cornell kernel without it is 0.7 % faster).
    // RT2_BVH_PAIRS=0 keeps single-box steps.
    const char* pe = getenv("RT2_BVH_PAIRS");
    const bool pairs = out.spheres > 0 && !(pe && atoi(pe) == 0);
    std::vector<char> target(n + 1, 0), second(n + 1, 0);
    for (size_t i = 0; i < n; i++)
      if (out.lin[4 * i] == kBvh || out.lin[4 * i] == kAccBvh || out.lin[4 * i] == kXform) target[out.lin[4 * i + 1]] = 1;
    for (size_t i = 0; i < n; i++) {
      const uint32_t kind = out.lin[4 * i];
      if (kind != kBvh && kind != kAccBvh) continue;  // accelerated-list tree nodes pair alike (padded boxes)
      uint32_t* w = &out.lin_wide[16 * i];
      w[2] = (uint32_t)(i + 1);
      w[3] = out.lin[4 * i + 1];
      if (!pairs || second[i] || i + 1 >= n || out.lin[4 * (i + 1)] != kind || target[i + 1]) continue;
      const size_t c = i + 1;
      second[c] = 1;
      w[2] = (uint32_t)(c + 1);
      w[3] = out.lin[4 * c + 1];
      const float* b = &out.lind[4 * (size_t)out.lin[4 * c + 2]];  // child's box: lo.xyz, _, hi.xyz, _
      memcpy(&w[7], &b[0], 4);
      memcpy(&w[11], &b[1], 4);
      memcpy(&w[12], &b[2], 4);
      memcpy(&w[13], &b[4], 4);
      memcpy(&w[14], &b[5], 4);
      memcpy(&w[15], &b[6], 4);
    }
  }
  PackMaterials(s, out);
  PackTextures(s, out);
  if (out.spheres) out.features |= kFeatSphere;
  for (const Obj& o : s.objs)
    if (o.kind == kSphere && !(o.disp.x == 0.0f && o.disp.y == 0.0f && o.disp.z == 0.0f)) out.features |= kFeatMotion;
  if (out.media) out.features |= kFeatMedium;
  if (out.xforms) out.features |= kFeatXform;
  if (out.acc_lists) out.features |= kFeatAccList;
  for (const MaterialDesc& m : s.materials)
    if (m.type == kMatMetal || m.type == kMatDielectric) out.features |= kFeatSpecular;
  for (const TextureDesc& t : s.textures) {
    if (t.type == kTexNoise) out.features |= kFeatNoise;
    if (t.type == kTexChecker) out.features |= kFeatChecker;
  }
  if (out.perlin_vec.empty()) out.perlin_vec.assign(4, 0.0f);
  if (out.perlin_perm.empty()) out.perlin_perm.assign(1, 0);
  if (out.textures.empty()) out.textures.assign(12, 0.0f);
  return true;
}

}  // namespace rt2
