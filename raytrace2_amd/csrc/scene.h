// scene.h — host scene model, Camera, SceneLoader and the scene compiler (BVH + flattening).
//
// Mirrors the reference surface that stays on the host:
//   SceneLoader::LoadScene / LoadCamera / WriteCamera / LoadAppSettings   (Serialize.hpp:21-35)
//   Camera (Update / setters, Camera.hpp:10-137)
//   App.cpp:126 (wrap the top-level list in one BVHNode, BVH.cpp:10-31)
// The object graph keeps the reference's construction order so BVH topology (std::sort with the
// same comparator on the same initial order) and material / texture index assignment match.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "hmath.h"
#include "rt2_layout.h"

namespace rt2 {

struct Interval {
  float min = kInfinity, max = -kInfinity;  // default empty (Interval.hpp:15)
  Interval() = default;
  Interval(float a, float b) : min(a), max(b) {}
  Interval(const Interval& a, const Interval& b);
  float Size() const { return max - min; }
};

struct AABB {
  Interval x, y, z;
  AABB() = default;
  AABB(vec3 a, vec3 b);
  AABB(const AABB& a, const AABB& b);
  const Interval& Axis(int n) const { return n == 0 ? x : (n == 1 ? y : z); }
  int LongestAxis() const;
  void PadToMinimums();
};

struct TextureDesc {
  uint32_t type = kTexSolid;
  vec3 albedo{1, 1, 1};
  float inv_scale = 1;  // checker
  uint32_t even = 0, odd = 0;
  float scale = 1;     // noise
  int noise_type = 1;  // NoiseType::kMarble
  int point_count = 256;
  std::vector<vec3> perlin_vec;
  std::vector<int> perm_x, perm_y, perm_z;
};

struct MaterialDesc {
  uint32_t type = kMatLambertian;
  vec3 albedo{1, 1, 1};
  float fuzz = 0;
  float refraction_index = 1;
  uint32_t tex_idx = 0;
};

// One Hittable of the reference object graph.
struct Obj {
  NodeKind kind = kQuad;
  AABB aabb;
  // quad
  vec3 q, u, v, w, n;
  float d = 0;
  // sphere
  vec3 c0, disp;
  float radius = 0;
  uint32_t material = 0;
  // list / bvh / xform / medium
  std::vector<int> children;  // list
  int left = -1, right = -1;  // bvh
  mat4 model, inv_model;      // xform
  int child = -1;             // xform / medium boundary
  float neg_inv_density = 0;  // medium
};

class Camera {
 public:
  void Update();
  void SetCenter(vec3 c) { center_ = c; dirty_ = true; }
  void SetLookAt(vec3 c) { lookat_ = c; dirty_ = true; }
  void SetViewUp(vec3 c) { view_up_ = c; dirty_ = true; }
  void SetFOV(float f) { vfov_ = f; dirty_ = true; }
  void SetDims(int w, int h) { dims_x_ = w; dims_y_ = h; dirty_ = true; }
  void SetDefocusAngle(float a) { defocus_angle_ = a; dirty_ = true; }
  void SetFocusDistance(float d) { focus_dist_ = d; dirty_ = true; }
  void SetSamplesPerPixel(int s) { samples_per_pixel_ = s; dirty_ = true; }
  int SqrtSamplesPerPixel() const { return sqrt_spp_; }
  int SamplesPerPixel() const { return samples_per_pixel_; }
  CameraParams Params();  // Update() + the values GetRay reads

  vec3 center_{0, 0, 0}, lookat_{0, 0, -1}, view_up_{0, 1, 0};
  vec3 viewport_upper_left_, pixel00_loc_, pixel_delta_u_, pixel_delta_v_, defocus_disk_u_, defocus_disk_v_;
  float defocus_angle_ = 0, focus_dist_ = 10, vfov_ = 90.f;
  int dims_x_ = 0, dims_y_ = 0;

 private:
  bool dirty_ = true;
  int sqrt_spp_ = 1;
  float recip_sqrt_spp_ = 1;
  int samples_per_pixel_ = 1;
};

struct AppSettings {  // Settings.hpp:5-11
  bool render_once = false;
  bool save_after_render_once = false;
  int64_t num_samples = 1;
  int64_t max_depth = 50;
  bool render_window = true;
};

struct Scene {
  std::vector<Obj> objs;          // object graph (shared sub-objects referenced by index)
  std::vector<int> primitives;    // loader "list" (Serialize.cpp:287-342)
  std::vector<int> top;           // scene.hittable_list before the BVH wrap
  int root = -1;                  // BVHNode over `top` (App.cpp:126)
  std::vector<MaterialDesc> materials;
  std::vector<TextureDesc> textures;
  Camera cam;
  std::string cam_name;
  vec3 background{1, 1, 1};
  int dims_x = 0, dims_y = 0;
  bool legacy_schema = false;
};

// Loads a scene file (v2 schema, or the legacy {"spheres":[...]} schema through the documented
// adapter) and builds the top-level BVH. `seed` keys the Perlin table streams. Returns false and
// sets `err` on any schema error (the reference prints and continues or crashes).
bool LoadScene(const std::string& path, uint64_t seed, Scene& out, std::string& err);
bool LoadCameraFile(const std::string& path, Camera& out, std::string& err);
bool WriteCameraFile(const Camera& cam, const std::string& path, std::string& err);
std::string CameraToJson(const Camera& cam);
bool LoadAppSettingsFile(const std::string& path, AppSettings& out, std::string& err);

// Flattened scene program (rt2_layout.h) ready for upload.
struct CompiledScene {
  std::vector<float> nodes;  // float4 records; BVH node records first ([0, hot_records))
  uint32_t hot_records = 0;
  uint32_t root = kRefNone;
  std::vector<float> materials;
  std::vector<float> textures;
  std::vector<float> perlin_vec;  // float4 per gradient
  std::vector<int> perlin_perm;
  int max_stack = 0;              // proven traversal-stack bound (entries)
  bool stack_ok = true;           // max_stack <= kTraversalStack: the stack traversal can run it
  int lin_xform_depth = 0;        // deepest transform nesting in the threaded program (0: none)
  int bvh_nodes = 0, quads = 0, spheres = 0, lists = 0, xforms = 0, media = 0;
  int acc_lists = 0, acc_nodes = 0;  // exact list acceleration trees (rt2_layout.h LISTACC)
  int box_steps = 0;                 // MakeBox runs and medium boundaries given a box record (boxaa.h)
  int bvh_depth = 0;
  uint32_t features = 0;          // rt2_layout.h Feature bits (defocus is added per render)
  // The threaded program uses a test that is exact only for ray origins within +-2^64 in world space
  // (QUADAA rectangles and box boundaries: compile.cpp RectAAWords; transforms about y: YAxisPattern):
  // a launch then refuses a camera whose rays would start beyond that (capi.cpp CameraOriginsBounded).
  // Scenes without such tests (e.g. spheres only) render any camera the reference does.
  bool origins_bounded = false;
  std::vector<uint32_t> lin;      // threaded traversal program (4 words per step), empty if too long
  std::vector<float> lind;        // records of the program's steps, in program order (float4)
  std::vector<uint32_t> lin_wide; // 16 words per step: the lin entry + the first 12 words of its record,
                                  // then one kProgramEnd entry
};
// accelerate_lists = false keeps every list a linear child loop (the reference's own order).
bool CompileScene(const Scene& s, CompiledScene& out, std::string& err, bool accelerate_lists = true);
// Accelerated-list trees built by SAH splits are at most this many levels deeper than balanced ones
// (compile.cpp BuildAcc); CompileSceneWith(..., 0) builds them balanced (depth ceil(log2 n)).
constexpr int kAccDepthSlack = 2;
bool CompileSceneWith(const Scene& s, CompiledScene& out, std::string& err, bool accelerate_lists,
                      int acc_depth_slack);
// The 8 QUADAA test words of QUAD record r (20 floats, rt2_layout.h) with axis code k + 4, or false when
// the quad takes the general path (compile.cpp RectAAWords; for tests/cpp/quadaa_bounds.cpp).
bool QuadAATestWords(const float* r, int k, float out[8]);
// The box record's six planes and margin constant (boxaa.h) of six QUAD records in MakeBox order, or
// false when they are not a box the box-level test can take (compile.cpp BoxAAWordsOf; for
// tests/cpp/box_cert.cpp).
bool BoxAAWords(const float* const faces[6], float out[6], float& mB);

// Philox4x32-10 (shared constants with the kernel; see render.hip)
void Philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1);
constexpr uint32_t kTagPath = 0x52543250u;    // "RT2P": per-(pixel, frame) path streams
constexpr uint32_t kTagPerlin = 0x52543254u;  // "RT2T": per-noise-texture table streams

}  // namespace rt2
