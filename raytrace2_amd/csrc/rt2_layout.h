// rt2_layout.h — layout of the flattened scene program in HBM and of the render launch
// parameters. Shared by the host scene compiler (compile.cpp) and the gfx950 kernel
// (render.hip). Plain POD; no HIP or torch types.
//
// The scene is one array of 16-byte records ("nodes", float4 units). A node reference packs the
// node kind in bits 28..31 and the float4 offset in bits 0..27, so a parent knows what it is about
// to fetch. Kinds mirror the reference's Hittable implementations:
//   kBvh    BVHNode            (BVH.cpp:10-55)          2 records
//   kQuad   Quad               (Quad.cpp:19-43)         5 records
//   kSphere Sphere (moving)    (Sphere.cpp:7-37)        2 records
//   kList   HittableList       (HittableList.cpp:8-22)  1 + ceil(n/4) records
//   kXform  TransformedHittable(Transform.cpp:13-88)    8 records
//   kMedium ConstantMedium     (ConstantMedium.cpp:14-58) 1 record
#pragma once
#include <stdint.h>

namespace rt2 {

enum NodeKind : uint32_t {
  kBvh = 0,
  kQuad = 1,
  kSphere = 2,
  kList = 3,
  kXform = 4,
  kMedium = 5,
  kXformExit = 6,  // traversal-stack marker only (never stored in the node array)
  kListAcc = 7,    // a large leaf-only sphere list with its exact acceleration tree
  kAccBvh = 8,     // 8 + split axis (8, 9, 10): node of a list's acceleration tree
  kAccSphere = 11, // a sphere reached through a list's acceleration tree
  kQuadAA = 12,    // threaded program only: a unit-normal axis-aligned quad in the QUADAA layout
  kProgramEnd = 13,  // threaded program only: the wide program's entry at index lin_len (no step)
};
inline constexpr bool is_acc_bvh(uint32_t kind) { return kind - kAccBvh < 3u; }
constexpr int kListAccelMin = 32;  // leaf-only sphere lists at least this long get a tree

constexpr uint32_t kRefNone = 0xFFFFFFFFu;

// Row-band partition of the image over `world` GPUs: rows in bands of band_h; band b lies in
// period p = b / world at phase q = b % world and belongs to rank (q + p) % world. Every rank owns
// one band per period (interleaving spreads costly image regions), and the phase a rank takes
// rotates from period to period, so no rank is tied to one phase of a periodic cost pattern. A rank
// stores its rows compactly in increasing y: local row l = p * band_h + (y % band_h).
inline constexpr int BandRank(int band, int world) { return (band % world + band / world) % world; }
// Rows of the largest rank's band stack: every rank's accumulation is allocated this tall and the
// gather sends this many rows from each rank (padding rows zero), so the root receives rank-major
// stacks [world][BandRowsMax][W]. band_h 0 = one band of the whole height.
inline constexpr int BandRowsMax(int height, int band_h, int world) {
  if (height <= 0) return 0;
  const int bh = band_h > 0 ? band_h : height;
  const int bands = (height + bh - 1) / bh;
  return (bands + world - 1) / world * bh;
}
// Where image row y lives in the gathered stacks: the owning rank and its rank-local row (the
// de-interleave map of gather.hip and of rt2_deinterleave_host; constexpr, so host and device).
struct BandRow {
  int rank, row;
};
inline constexpr BandRow BandSource(int y, int band_h, int world) {
  if (band_h <= 0) return BandRow{0, y};  // one band: rank 0 holds every row
  const int band = y / band_h, period = band / world;
  return BandRow{BandRank(band, world), period * band_h + (y - band * band_h)};
}
constexpr uint32_t kOffsetMask = 0x0FFFFFFFu;
inline constexpr uint32_t make_ref(uint32_t kind, uint32_t off) { return (kind << 28) | off; }

// Record layouts (each line one float4; "(bits)" = uint32 stored with __float_as_uint):
//  BVH   : (min.xyz, left_ref bits) (max.xyz, right_ref bits)  right_ref = kRefNone when a
//          span-1 leaf's duplicate test is provably a no-op (no medium below it).
//  QUAD  : (n.xyz, D) (q.xyz, material bits) (u.xyz, axis bits) (v.xyz, 0) (w.xyz, sD)
//          axis = k + 1 when n and w are exactly zero off axis k (exact axis-aligned test),
//          k + 4 when moreover n[k] = s = +-1 exactly (sD = s * D), else 0
//          In the threaded program's record copy (lind), v.w = the enclosing XFORM's lind ref.
//  QUADAA: (threaded-program record copy of a quad with axis code K + 4 that is a rectangle in
//          its plane; other unit-normal quads get code K + 1 in the program)
//          (sD, lo[A], hi[A], lo[B]) (hi[B], 0, 0, 0) (n.xyz, D) (q.xyz, material bits)
//          (axis bits, xform ref bits, 0, 0), A = (K + 1) % 3, B = (K + 2) % 3: the hit point's
//          in-plane coordinates p[A], p[B] that Quad::Hit's interior test accepts are exactly
//          [lo[A], hi[A]] x [lo[B], hi[B]] (compile.cpp RectAAWords / CoordRange): the test reads
//          the first 5 words only
//  SPHERE: (c0.xyz, radius) (displacement.xyz, material bits)
//  LIST  : (count bits, flags bits, 0, 0) then child refs, 4 per record. flags bit0 = every
//          child is a QUAD or SPHERE (iterated inline, no stack traffic).
//  XFORM : (invM col0.xyz, child_ref bits) (invM col1.xyz, parent_xform_ref bits)
//          (invM col2.xyz, pattern bits) (invM col3.xyz, 0) (M col0.xyz,0) (M col1.xyz,0) (M col2.xyz,0)
//          (M col3.xyz,0); pattern (threaded-program copies only, else 0): kXformYAxis when col0.y,
//          col1.x, col1.z and col2.y of both matrices are +-0 (a transform about y, compile.cpp
//          YAxisPattern): the kernel leaves their +-0 products out
//  MEDIUM: (neg_inv_density, material bits, boundary_ref bits, 0)
//          In the threaded program's record copy, a boundary that is a list of at most
//          kBoundaryAAMax unit-normal axis-aligned quads (a box in the medium's space) also has its
//          children's 8-word QUADAA test records right after the medium record, and word 3 =
//          kBoundaryAAFlag | count << 24 | (axis K of child k) << 3k (boundary_ref keeps the
//          general copy); a MakeBox boundary (six faces, boxaa.h BoxAAWords) also has
//          kBoundaryBoxFlag and its 2-record box record (six planes, margin) after the quads' words.
//  LISTACC: (center.xyz, R) (k2, k1, k0, root_ref bits): a HittableList of n >= kListAccelMin
//          spheres (HittableList.cpp:8-22). The list returns the smallest accepted root and, on
//          equal roots, its first child (Sphere uses the strict Surrounds), so any visiting
//          order gives the same hit when candidates are never wrongly culled and ties go to the
//          lowest child index; the children's records are emitted in list order, so the index
//          order is the record-offset order. The tree's boxes are padded per ray by
//          pad = (k2 * L + k1) * L + k0, L = |o - center| + R (a bound on |center_i - o|), which
//          covers the float error of Sphere::Hit's discriminant for rays that far away
//          ("Exact list acceleration").
//  ACCBVH: (min.xyz, near_ref bits) (max.xyz, far_ref bits); near = the child with the smaller
//          centroids along the node's split axis (kind - kAccBvh); children are ACCBVH or
//          ACCSPHERE refs (an ACCSPHERE ref points at the child's SPHERE record)
constexpr uint32_t kListLeafOnly = 1u;
constexpr uint32_t kXformYAxis = 1u;
// The reciprocal direction component an accelerated list's padded slab test uses (render.hip lane
// walk: ax = fma(lo - o, inv, -pad inv), bx = fma(hi - o, inv, pad inv)): inv itself when finite,
// else +-2^100. With inv = +-inf (d = +-0) the fma form gives NaN or -inf for an origin inside the
// padding band [lo - pad, hi + pad] and culls the box; with +-2^100 (a power of two: the products are
// exact) the two bounds get the signs of (lo - pad - o) and (hi + pad - o), so the axis accepts all
// t >= 0 up to |hi + pad - o| * 2^100 exactly when o lies in the band. That limit only falls below
// a ray's range when o is within 2^-100 * range of the padded face, a quarter pad or more outside
// every sphere's reach (the pad carries a 4x margin), so no hit is lost.
inline constexpr float acc_slab_inv(float inv) {
  return inv > 0x1p100f ? 0x1p100f : (inv < -0x1p100f ? -0x1p100f : inv);
}
constexpr uint32_t kBoundaryAAFlag = 0x80000000u;
constexpr uint32_t kBoundaryBoxFlag = 0x08000000u;  // a MakeBox boundary: a box record (boxaa.h) follows
constexpr uint32_t kBoundaryAAMax = 6;

constexpr int kBvhRecords = 2, kQuadRecords = 5, kSphereRecords = 2, kXformRecords = 8, kMediumRecords = 1;

// Materials: 2 records each: (type bits, albedo.xyz) (fuzz, refraction_index, tex_idx bits, 1/ri)
enum MaterialType : uint32_t {
  kMatMetal = 0,
  kMatLambertian = 1,
  kMatDielectric = 2,
  kMatTexture = 3,
  kMatDiffuseLight = 4,
  kMatIsotropic = 5,
};
// Textures: 3 records each: (type bits, albedo.xyz) (inv_scale|scale, even bits, odd bits,
// noise_type bits) (perlin vec offset bits, perlin perm offset bits, point_count bits, 0)
enum TextureType : uint32_t { kTexSolid = 0, kTexChecker = 1, kTexNoise = 2 };

constexpr int kTraversalStack = 24;  // max entries per lane (LDS); compile.cpp proves the bound

// Scene feature bits. The render kernel is instantiated for a few feature sets; a launch uses the
// smallest instantiated superset of the scene's features, so code (and registers) for absent
// features is not compiled into the kernel that runs.
enum Feature : uint32_t {
  kFeatSphere = 1u << 0,    // Sphere primitives
  kFeatMedium = 1u << 1,    // ConstantMedium + Isotropic
  kFeatXform = 1u << 2,     // TransformedHittable
  kFeatNoise = 1u << 3,     // Noise (Perlin / marble) textures
  kFeatChecker = 1u << 4,   // Checker textures
  kFeatSpecular = 1u << 5,  // Metal / Dielectric materials
  kFeatDefocus = 1u << 6,   // thin-lens camera (defocus_angle > 0)
  kFeatGenList = 1u << 7,   // lists whose children are not all quads/spheres (pushed on the stack)
  kFeatAccList = 1u << 8,   // accelerated sphere lists (LISTACC)
  kFeatMotion = 1u << 9,    // a sphere that moves (displacement not +-0); without it the kernel
                            // takes center(time) = c0 (c0 + (+-0) differs only in a zero's sign)
  kFeatAll = 0x3FFu,
};
constexpr int kLdsSceneBytesMax = 96 * 1024;  // scenes up to this size are staged in LDS

// Threaded ("linear") traversal program: the reference's fixed left-then-right pre-order of the
// scene tree, one 16-byte entry per step: (kind, skip, record offset, aux).
//   kind kBvh: skip = index after the node's subtree (taken when the AABB test misses)
//   kind kQuad / kSphere / kMedium: record of the primitive; the next step is always index + 1;
//     for kQuad, aux = length of the run of consecutive quads starting here (at most
//     kLinearMaxRun) with no skip target inside it, skip = the run's axis codes, 3 bits per quad
//     (codes 4..6 use the QUADAA record layout, the others the QUAD layout), then a 1 bit
//   kind kXform: enter the transform (record = XFORM record, skip = index of its kXformExit);
//     the kernel walks the steps up to the exit in a nested loop with the transformed ray
//   kind kXformExit: leave it (record = XFORM record, aux = parent XFORM ref or kRefNone, skip = the end
//     of the transform's record range: the records under it are [record + 8, skip))
//   kind kListAcc: an accelerated list (record = LISTACC, skip = index after its tree's copies,
//     aux = steps per copy): sets the ray's box padding; its tree follows in pre-order (one copy,
//     or eight: copy k visits a node's children nearer-first for rays whose direction is negative
//     along the axes of k's bits), near child first: kind kAccBvh (record = ACCBVH, skip = index after
//     the subtree, padded box test) and kind kAccSphere (record = SPHERE, aux = the sphere's
//     record offset in the node array, i.e. its list position, for the equal-root rule)
// Lists vanish (their children follow each other); span-1 leaves with a medium appear twice.
// Record offsets refer to a separate record stream (RenderParams::lind) holding each step's
// record in program order, so a run of quads is contiguous.
// All lanes of a wave walk this array in lockstep at the smallest pending index, so the step
// kind is wave-uniform and its record is read with scalar loads.
// Scenes whose program is longer use the stack traversal. Measured (1920x1080, 64 spp): sphere
// fields of 2,000 / 10,000 spheres run 1.72x / 1.37x faster threaded than stacked, 100,000 (about
// 200 k steps) 0.97x; book 2 (accelerated list threaded as well) 1.20x.
constexpr int kLinearMaxSteps = 1 << 16;
#ifndef RT2_LINEAR_MAX_RUN
#define RT2_LINEAR_MAX_RUN 10
#endif
constexpr uint32_t kLinearMaxRun = RT2_LINEAR_MAX_RUN;  // quads per run (3-bit axis codes + 1 bit in one word)
// A quad step's aux word: the run length, and bit 31 for a MakeBox run whose box record (boxaa.h, 2 records:
// the six planes, the margin constant, padding) lies right before the run's first face record
constexpr uint32_t kRunLenMask = 0xFFu, kRunBoxFlag = 0x80000000u;
static_assert(3 * kLinearMaxRun < 32, "a run's codes and their end bit fit one word");
constexpr int kLinearMaxXformDepth = 8;  // deeper transform nesting uses the stack traversal

// kModeStackHybrid: the scene is too large for LDS, but its BVH node records (the prefix
// [0, lds_nodes) of the record array) are staged in LDS; other records are read from global memory.
enum TraversalMode : int { kModeStackGlobal = 0, kModeStackLds = 1, kModeLinear = 2, kModeStackHybrid = 3 };
constexpr int kLdsHotBytesMax = 32 * 1024;  // BVH prefix staged in LDS by kModeStackHybrid

struct CameraParams {
  float pixel00[3], du[3], dv[3], center[3], defocus_u[3], defocus_v[3];
  float defocus_angle;
  float recip_sqrt_spp;
  int sqrt_spp;
};

struct StatsCounters {  // u64 slots written by the kernel
  enum { kRays = 0, kBvhTests, kQuadTests, kSphereTests, kXformVisits, kMediumTests, kListVisits, kPaths, kCount };
  enum { kOverflow = kCount, kStamps = 9, kDiag = 16, kSlots = 32 };  // stamps / diag: diagnostic builds
  // the box-level test of flagged MakeBox runs (boxaa.h): lanes tested, lanes certified; wave visits of
  // a flagged run, and those in which some lane fell back so the wave ran the six faces
  enum { kBoxTests = 24, kBoxCertified, kBoxWaveVisits, kBoxWaveRuns };
};
constexpr int kStatsSlots = StatsCounters::kSlots;

// floor(n / d) = (n * m) >> s for every 0 <= n < 2^31 (Granlund-Montgomery: m = ceil(2^(31+l) / d),
// s = 31 + l, 2^(l-1) < d <= 2^l, so m < 2^32): one 32x32->64 multiply and a shift instead of a
// division by a run-time divisor. Built by the host (MakeMagic, capi.cpp).
struct Magic {
  uint32_t m, s;
};

// Sample buffer: a launch's frames in octets of kOctet consecutive frames (launch-relative frame
// fr: octet fr / kOctet, slot fr % kOctet); a pixel's octet is 3 * kOctet floats (96 bytes)
// contiguous, pixels adjacent within an octet plane: float index
// ((fr / kOctet) * local_pixels + pixel) * 3 * kOctet + 3 * (fr % kOctet) + component.
// A lane writes a whole octet at once (three full 32-B sectors) instead of 12 B at a time.
constexpr uint32_t kOctet = 8;
// Frame chunks hold at most kChunkMaxFrames frames: the kernel keeps a chunk's frames left in
// 11 bits of a register that also holds the ray depth and the lane's sample-staging state.
constexpr int kChunkMaxFrames = 0x800;
constexpr uint32_t kChunkLeftMask = 0x7FFu;

struct RenderParams {
  const void* nodes;      // float4[]
  const void* materials;  // float4[]
  const void* textures;   // float4[]
  const void* perlin_vec; // float4[]
  const int* perlin_perm;
  uint32_t root;
  float background[3];
  CameraParams cam;
  int width, height;       // global image
  int local_rows;          // rows owned by this rank
  int band_h, rank, world; // interleaved row bands: global band b -> rank b % world
  uint32_t tile_shift;     // work tiles of 64 pixels: (1 << tile_shift) wide x (64 >> tile_shift) local rows
  int tiles_x;             // ceil(width / tile width)
  uint32_t tile_items;     // tiles_x * ceil(local_rows / tile rows) * 64: lanes of one frame chunk
  uint32_t n_items;        // tile_items * chunks (work item = one pixel x one chunk of frames)
  uint32_t batch_max;      // most work items a wave reserves at once
  uint32_t batch_div;      // a wave reserves (items left) / batch_div, at least what it needs
  int frame_begin, n_frames, max_depth;
  // Frame chunks of the launch, (first frame, stratum s_i | s_j << 16 of that frame) per chunk
  // (RayTracer.cpp:59-60) and a sentinel (frame_begin + n_frames, 0): chunk c is the frames
  // [chunks[2c], chunks[2c + 2]). Work item = one pixel x one chunk; chunks shrink toward the end
  // of the launch so the last items are short (capi.cpp, ChunkSchedule).
  const uint32_t* chunks;
  uint32_t n_chunks;
  Magic div_tile_items, div_tiles_x;  // item -> (chunk, tile), tile -> tile row
  Magic div_band_h, div_band_w, div_world;  // band_h, band_h * world, world (row-band partition)
  uint32_t seed_lo, seed_hi;
  float* samples;          // float3 per (launch frame, local pixel) in octets (kOctet above)
  uint32_t local_pixels;   // width * local_rows
  uint32_t* ray_counts;    // optional: += rays per local pixel (atomic: chunks of a pixel overlap)
  uint32_t* work_counter;  // zeroed before launch
  unsigned long long* stats;  // StatsCounters::kCount slots
  int stack_depth;         // traversal-stack entries per lane (<= kTraversalStack)
  uint32_t lds_nodes;      // float4 records staged in LDS (0: read the scene from global memory)
  uint32_t lds_partial;    // 1: only the BVH prefix is in LDS (kModeStackHybrid)
  const void* lin;         // uint4[lin_len] threaded traversal program (kModeLinear)
  const void* lind;        // float4 records of the program's steps (kModeLinear)
  const void* lin_wide;    // 64-byte steps: entry + first 48 bytes of its record (kModeLinear)
  uint32_t lin_len;
  // Frame tiles (item mode 1): a wave's 64 items are one pixel x 64 consecutive frames of the launch
  // (chunks of one frame), so its lanes trace paths from the same pixel. item = g * frame_tile +
  // pixel * 64 + k renders chunk 64 g + k of local pixel `pixel`; frame_tile = 64 * local_pixels.
  uint32_t frame_tiles;
  uint32_t frame_tile;
  Magic div_frame_tile, div_width;
  // 1: no transform of the threaded program nests in another (every primitive under a transform lies
  // in that transform's record range; the kernel may keep a hit's model-space ray from the trace)
  uint32_t flat_xforms;
  // Philox4x32-10 round keys of the path streams: (seed_lo + r * 0x9E3779B9, seed_hi + r * 0xBB67AE85)
  // for rounds r = 0..9, interleaved (the kernel loads them with two scalar loads per block instead
  // of computing 18 adds on the scalar unit at every refill)
  uint32_t philox_keys[20];
  // This launch's clock pair (capi.cpp launch-clock ring, zeroed before the launch): word 0 = the
  // largest complement of a wave's start time (so ~word 0 is the first wave's start), word 1 = the
  // last wave's end, in ticks of the GPU's constant 100 MHz clock (s_memrealtime). A launch's GPU
  // time is then measured from its first wave to its last one, whatever it waited for in its queue
  // (with two launch slots the next launch is queued while the previous one still holds the CUs).
  unsigned long long* launch_clock;
};
constexpr int kClockRing = 512;  // launch-clock pairs per tracer (drained at half)

}  // namespace rt2
