// boxaa.h — the box-level test of a MakeBox run (Quad.hpp:34-50: a HittableList of six quads, the faces
// z+ x+ z- x- y+ y- of an axis-aligned box in its own space), shared by the kernel (render.hip: the quad-run
// step of a box-flagged run) and its host proof harness (tests/cpp/box_cert.cpp). The includer defines RT2_BOXAA_FN (the
// function qualifiers) and passes a math policy M: min / max / min3 / max3 / med3 of non-NaN floats,
// amin3 / amax3 (of the magnitudes), fma,
// and the division by a correctly rounded reciprocal (render.hip div_by_inv). Every operation is
// correctly rounded IEEE single precision on both sides, so both compute the same bits.
//
// The six-face run (HittableList::Hit over Quad::Hit, HittableList.cpp:8-22, Quad.cpp:19-43) returns the
// accepted face with the smallest t in [tmin, tmax], later faces winning ties. A ray's box test computes
// every face plane's t exactly as that face's own test does, classifies them as slab entry and exit
// times, and takes one candidate face: the entry face when the entry time is >= tmin, else the exit face.
// A per-lane certificate proves that no other face can change the run's answer and that the candidate's
// interior test is decided by the slabs alone; then the run's answer is the candidate's t if the line
// passes through the box and that t lies in the interval, else no hit.
// Where the certificate fails the lane falls back to the six-face run. DESIGN.md §4 "Box-level test"
// has the proof; tests/cpp/box_cert.cpp checks it against the run on adversarial rays.
#pragma once
#include <cstdint>

namespace rt2 {

// The box record (8 words = 2 records right before the run's first face record; compile.cpp BoxAAWordsOf):
//   [0..5]  face planes lo_x, hi_x, lo_y, hi_y, lo_z, hi_z (the faces' sD words: x- x+ y- y+ z- z+)
//   [6]     mB = 2^-21 max|plane| + s, s the largest distance of a face's QUADAA interior bound from the
//           box plane it approximates (the compiler requires s <= 2^-20 max|plane|)
//   [7]     0
constexpr int kBoxAAWords = 6;
constexpr int kBoxAARecords = 2;
// Face indices within the MakeBox run (z+ x+ z- x- y+ y-) of face (axis K, hi side): 3 bits each,
// index 2 K + hi: x- 3, x+ 1, y- 5, y+ 4, z- 2, z+ 0.
constexpr uint32_t kBoxAAFaceMap = 3u | (1u << 3) | (5u << 6) | (4u << 9) | (2u << 12) | (0u << 15);
// The run's axis codes (rt2_layout.h QUADAA, 4 + K) with the end bit: z x z x y y.
constexpr uint32_t kBoxAARunCodes = 6u | (4u << 3) | (6u << 6) | (4u << 9) | (5u << 12) | (5u << 15) | (1u << 18);
// The float above 1e-8f: every face's own parallel-ray rejection (Quad.cpp:22) passes for |d_K| >= it
constexpr float kBoxAADenomMin = 0x1.5798f0p-27f;

struct BoxAAResult {
  bool cert;     // the candidate alone decides the run's answer
  uint32_t x;    // the candidate's key | rejection sign (render.hip quad runs: accepted iff x <= kmax)
  float t;       // the candidate's t
  uint32_t face; // the candidate's index in the run (0..5)
};

template <class M>
RT2_BOXAA_FN BoxAAResult BoxAATest(const float* w, float mB, float ox, float oy, float oz, float dx, float dy, float dz,
                                   float ix, float iy, float iz, float tmin) {
  // the six plane t's, each as its face's QUADAA test computes it (t = (sD - o_K) / d_K, exact)
  const float ax = M::div(w[0] - ox, dx, ix), bx = M::div(w[1] - ox, dx, ix);
  const float ay = M::div(w[2] - oy, dy, iy), by = M::div(w[3] - oy, dy, iy);
  const float az = M::div(w[4] - oz, dz, iz), bz = M::div(w[5] - oz, dz, iz);
  const float tnx = M::min(ax, bx), tfx = M::max(ax, bx);
  const float tny = M::min(ay, by), tfy = M::max(ay, by);
  const float tnz = M::min(az, bz), tfz = M::max(az, bz);
  const float tin = M::max3(tnx, tny, tnz), tout = M::min3(tfx, tfy, tfz);   // slab entry / exit
  const float t2 = M::med3(tnx, tny, tnz), x2 = M::med3(tfx, tfy, tfz);       // second entry / exit
  const bool nearc = tin >= tmin;  // candidate: the entry face (else the exit face)
  const float tc = nearc ? tin : tout;
  // Certificate, in distance along the smallest direction component dmin (DESIGN.md §4 "Box-level test"):
  //  * the candidate's side gap: entry candidate T_in - T2 (the other entry faces' points lie before the
  //    entry plane), exit candidate X2 - T_out (the other exit faces' points lie beyond the exit plane);
  //  * half the slab gap |T_out - T_in|: through the box, the candidate's point lies inside every other
  //    slab by it, so the candidate's interior test accepts; past the box (T_in > T_out), every face's
  //    point lies outside the entry slab (t below the midpoint) or the exit slab (above it): none accepts.
  const float gside = nearc ? tin - t2 : x2 - tout;
  const float gmid = 0.5f * M::abs(tout - tin);
  const float dmin = M::amin3(dx, dy, dz), dmax = M::amax3(dx, dy, dz);
  // rounding margin: 2^-21 (|o| + |d| |t| + max|plane|) + s bounds, with a factor of 2.6 to spare, the
  // rounding of every hit-point coordinate a face computes and of the plane crossings
  const float tabs = M::amax3(M::amax3(tin, t2, tout), x2, x2);
  const float omax = M::amax3(ox, oy, oz);
  const float m = M::fma(0x1p-21f, M::fma(dmax, tabs, omax), mB);
  BoxAAResult r;
  // dmin >= the float above 1e-8: every face's own parallel-ray rejection passes
  r.cert = (dmin >= kBoxAADenomMin) & (dmin * M::min(gside, gmid) >= m);
  const uint32_t key = M::bits(tc) - M::bits(tmin);
  r.x = tin < tout ? key : key | 0x80000000u;  // through the box: the candidate accepts iff in the interval
  r.t = tc;
  // the candidate's face: the plane whose t is tc (unique when certified: the gaps are > 0)
  uint32_t f = 0u;
  f = tc == az ? 2u : f;
  f = tc == by ? 4u : f;
  f = tc == ay ? 5u : f;
  f = tc == bx ? 1u : f;
  f = tc == ax ? 3u : f;
  r.face = f;
  return r;
}

// Both boundary queries of ConstantMedium::Hit on a MakeBox boundary (ConstantMedium.cpp:14-58; render.hip
// boundary_aa_pair: t1 = the smallest accepted face t in [-FLT_MAX, FLT_MAX], t2 = the smallest in
// [fl(t1 + 0.0001), FLT_MAX]). Under the certificate dmin * min(T_in - T2, X2 - T_out, |T_out - T_in| / 2)
// >= m (both side gaps: the entry and the exit face are both candidates), a line through the box has
// exactly two accepting faces, the entry face at T_in and the exit face at T_out (each one's point lies
// inside every other slab, every other face's point outside a slab), and a line past it none. The
// queries' intervals do not enter: every other face is rejected by its interior test.
struct BoxAAPairResult {
  bool cert;  // the two faces below are the boundary's only accepting faces (none when !through)
  bool through;
  float tin, tout;
};
template <class M>
RT2_BOXAA_FN BoxAAPairResult BoxAAPair(const float* w, float mB, float ox, float oy, float oz, float dx, float dy,
                                       float dz, float ix, float iy, float iz) {
  const float ax = M::div(w[0] - ox, dx, ix), bx = M::div(w[1] - ox, dx, ix);
  const float ay = M::div(w[2] - oy, dy, iy), by = M::div(w[3] - oy, dy, iy);
  const float az = M::div(w[4] - oz, dz, iz), bz = M::div(w[5] - oz, dz, iz);
  const float tnx = M::min(ax, bx), tfx = M::max(ax, bx);
  const float tny = M::min(ay, by), tfy = M::max(ay, by);
  const float tnz = M::min(az, bz), tfz = M::max(az, bz);
  const float tin = M::max3(tnx, tny, tnz), tout = M::min3(tfx, tfy, tfz);
  const float t2 = M::med3(tnx, tny, tnz), x2 = M::med3(tfx, tfy, tfz);
  const float dmin = M::amin3(dx, dy, dz), dmax = M::amax3(dx, dy, dz);
  const float tabs = M::amax3(M::amax3(tin, t2, tout), x2, x2);
  const float omax = M::amax3(ox, oy, oz);
  const float m = M::fma(0x1p-21f, M::fma(dmax, tabs, omax), mB);
  const float g = M::min(M::min(tin - t2, x2 - tout), 0.5f * M::abs(tout - tin));
  BoxAAPairResult r;
  r.cert = (dmin >= kBoxAADenomMin) & (dmin * g >= m);
  r.through = tin < tout;
  r.tin = tin;
  r.tout = tout;
  return r;
}

}  // namespace rt2
