// boxaa.h — the box-level test of a MakeBox run (Quad.hpp:34-50: a HittableList of six quads, the faces
// z+ x+ z- x- y+ y- of an axis-aligned box in its own space), shared by the kernel (render.hip: the quad-run
// step of a box-flagged run) and its host proof harness (tests/cpp/box_cert.cpp). The includer defines RT2_BOXAA_FN (the
// function qualifiers) and passes a math policy M: min / max / min3 / max3 / med3 of non-NaN floats, fma,
// and the division by a correctly rounded reciprocal (render.hip div_by_inv). Every operation is
// correctly rounded IEEE single precision on both sides, so both compute the same bits.
//
// The six-face run (HittableList::Hit over Quad::Hit, HittableList.cpp:8-22, Quad.cpp:19-43) returns the
// accepted face with the smallest t in [tmin, tmax], later faces winning ties. A ray's box test computes
// every face plane's t exactly as that face's own test does, classifies them as slab entry and exit
// times, and takes one candidate face: the entry face when the entry time is >= tmin, else the exit face.
// A per-lane certificate proves that no other face can change the run's answer; then the run's answer is
// the candidate's own decision (its t, and its interior test decided against the box's inner bounds).
// Where the certificate fails the lane falls back to the six-face run. DESIGN.md §4 "Box-level test"
// has the proof; tests/cpp/box_cert.cpp checks it against the run on adversarial rays.
#pragma once
#include <cstdint>

namespace rt2 {

// The box record (16 words right before the run's first face record; compile.cpp BoxAAWordsOf):
//   [0..5]  face planes lo_x, hi_x, lo_y, hi_y, lo_z, hi_z (the faces' sD words: x- x+ y- y+ z- z+)
//   [6..11] inner bounds in_lo_x, in_hi_x, in_lo_y, in_hi_y, in_lo_z, in_hi_z: on each coordinate the
//           intersection of the four faces' QUADAA interior ranges on it (compile.cpp BoxAAWords)
//   [12]    mB = 2^-21 max|plane| + s, s the largest distance of a face's interior bound from the
// box plane it approximates (the compiler requires s <= 2^-20 max|plane|).
constexpr int kBoxAAWords = 12;
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
                                   float ix, float iy, float iz, float tmin, uint32_t kmax0) {
  // the six plane t's, each as its face's QUADAA test computes it (t = (sD - o_K) / d_K, exact)
  const float ax = M::div(w[0] - ox, dx, ix), bx = M::div(w[1] - ox, dx, ix);
  const float ay = M::div(w[2] - oy, dy, iy), by = M::div(w[3] - oy, dy, iy);
  const float az = M::div(w[4] - oz, dz, iz), bz = M::div(w[5] - oz, dz, iz);
  const float tnx = M::min(ax, bx), tfx = M::max(ax, bx);
  const float tny = M::min(ay, by), tfy = M::max(ay, by);
  const float tnz = M::min(az, bz), tfz = M::max(az, bz);
  const float tin = M::max3(tnx, tny, tnz), tout = M::min3(tfx, tfy, tfz);   // slab entry / exit
  const float t2 = M::med3(tnx, tny, tnz), x2 = M::med3(tfx, tfy, tfz);       // second entry / exit
  const bool ex = tin == tnx, ey = !ex && tin == tny;                          // entry axis e
  const bool xx = tout == tfx, xy = !xx && tout == tfy;                        // exit axis x
  const bool nearc = tin >= tmin;  // candidate: the entry face (else the exit face)
  const float tc = nearc ? tin : tout;
  const bool kx = nearc ? ex : xx, ky = nearc ? ey : xy;
  // the candidate's hit point as its own test computes it (o + d t, product then sum); its own
  // coordinate is replaced by an inner bound (the face's test does not read it)
  const float px = kx ? w[6] : ox + dx * tc;
  const float py = ky ? w[8] : oy + dy * tc;
  const float pz = (kx || ky) ? oz + dz * tc : w[10];
  // inside the inner bounds: inside every face's interior ranges, the candidate's included (the signs of
  // the rounded differences are the exact signs, render.hip quad_aa)
  const uint32_t win = (M::bits(px - w[6]) | M::bits(w[7] - px) | M::bits(py - w[8])) |
                       (M::bits(w[9] - py) | M::bits(pz - w[10]) | M::bits(w[11] - pz));
  const bool inner = (int32_t)win >= 0;
  const float adx = M::abs(dx), ady = M::abs(dy), adz = M::abs(dz);
  const float ade = ex ? adx : (ey ? ady : adz);
  const float adq = xx ? adx : (xy ? ady : adz);
  // rounding margin: 2^-21 (|o| + |d| |t| + max|plane|) + s bounds, with a factor of 2.7 to spare, the
  // rounding of every hit-point coordinate a face computes and of the plane crossings
  const float tabs = M::max(M::max3(M::abs(tin), M::abs(t2), M::abs(tout)), M::abs(x2));
  const float omax = M::max3(M::abs(ox), M::abs(oy), M::abs(oz));
  const float m = M::fma(0x1p-21f, M::fma(M::max3(adx, ady, adz), tabs, omax), mB);
  const bool hitline = tin < tout;
  // near, line through the box: the other entry faces' points lie before the entry plane (coordinate e)
  // near, line misses the box: every face's point lies outside the entry or the exit slab
  // far: the other exit faces' points lie beyond the exit plane (coordinate x); the entry faces are
  // before tmin
  const bool geo = nearc ? (hitline ? ade * (tin - t2) >= m : M::min(ade, adq) * (tin - tout) >= 2.0f * m)
                         : adq * (x2 - tout) >= m;
  const bool dok = M::min3(adx, ady, adz) >= kBoxAADenomMin;
  const uint32_t key = M::bits(tc) - M::bits(tmin);
  const bool miss = nearc && !hitline;  // the candidate is rejected too (it lies outside a slab)
  // the candidate's decision is needed (in the interval) but undecided by the inner bounds: fall back
  const bool undecided = key <= kmax0 && !miss && !inner;
  BoxAAResult r;
  r.cert = dok && geo && !undecided;
  r.x = key | ((inner && !miss) ? 0u : 0x80000000u);
  r.t = tc;
  const uint32_t axis = kx ? 0u : (ky ? 1u : 2u);
  const float dk = kx ? dx : (ky ? dy : dz);
  // the entry face of axis K is its lo face when d_K > 0; the exit face its hi face
  const uint32_t hi = (nearc == (dk < 0.0f)) ? 1u : 0u;
  r.face = (kBoxAAFaceMap >> (3u * (2u * axis + hi))) & 7u;
  return r;
}

}  // namespace rt2
