// scene.cpp — SceneLoader (Serialize.cpp:32-360), Camera::Update (Camera.hpp:16-48),
// geometry constructors (Quad.hpp, Sphere.hpp, Transform.cpp, ConstantMedium.cpp, BVH.cpp).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>

#include "json.h"
#include "scene.h"

namespace rt2 {

// ---------------------------------------------------------------------------------------------
// Interval / AABB (Interval.hpp:6-31, AABB.hpp:9-65)
Interval::Interval(const Interval& a, const Interval& b)
    : min(std::fmin(a.min, b.min)), max(std::fmax(a.max, b.max)) {}

AABB::AABB(vec3 a, vec3 b)
    : x(std::fmin(a.x, b.x), std::fmax(a.x, b.x)),
      y(std::fmin(a.y, b.y), std::fmax(a.y, b.y)),
      z(std::fmin(a.z, b.z), std::fmax(a.z, b.z)) {
  PadToMinimums();
}
AABB::AABB(const AABB& a, const AABB& b) : x(a.x, b.x), y(a.y, b.y), z(a.z, b.z) { PadToMinimums(); }

int AABB::LongestAxis() const {
  if (x.Size() > y.Size()) return x.Size() > z.Size() ? 0 : 2;
  return y.Size() > z.Size() ? 1 : 2;
}

void AABB::PadToMinimums() {
  const float kDelta = 0.0001f;
  auto expand = [](Interval& i, float delta) {
    float padding = delta / 2.0f;
    i = Interval(i.min - padding, i.max + padding);
  };
  if (x.Size() < kDelta) expand(x, kDelta);
  if (y.Size() < kDelta) expand(y, kDelta);
  if (z.Size() < kDelta) expand(z, kDelta);
}

// ---------------------------------------------------------------------------------------------
mat4 inverse(const mat4& m) {
  float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
  float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
  float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
  float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
  float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
  float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
  float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
  float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
  float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
  float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
  float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
  float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
  float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
  float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
  float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
  float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
  float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
  float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
  vec4 Fac0{{Coef00, Coef00, Coef02, Coef03}}, Fac1{{Coef04, Coef04, Coef06, Coef07}};
  vec4 Fac2{{Coef08, Coef08, Coef10, Coef11}}, Fac3{{Coef12, Coef12, Coef14, Coef15}};
  vec4 Fac4{{Coef16, Coef16, Coef18, Coef19}}, Fac5{{Coef20, Coef20, Coef22, Coef23}};
  vec4 Vec0{{m[1][0], m[0][0], m[0][0], m[0][0]}}, Vec1{{m[1][1], m[0][1], m[0][1], m[0][1]}};
  vec4 Vec2{{m[1][2], m[0][2], m[0][2], m[0][2]}}, Vec3{{m[1][3], m[0][3], m[0][3], m[0][3]}};
  vec4 Inv0 = (Vec1 * Fac0 - Vec2 * Fac1) + Vec3 * Fac2;
  vec4 Inv1 = (Vec0 * Fac0 - Vec2 * Fac3) + Vec3 * Fac4;
  vec4 Inv2 = (Vec0 * Fac1 - Vec1 * Fac3) + Vec3 * Fac5;
  vec4 Inv3 = (Vec0 * Fac2 - Vec1 * Fac4) + Vec2 * Fac5;
  vec4 SignA{{+1, -1, +1, -1}}, SignB{{-1, +1, -1, +1}};
  mat4 r;
  r[0] = Inv0 * SignA;
  r[1] = Inv1 * SignB;
  r[2] = Inv2 * SignA;
  r[3] = Inv3 * SignB;
  vec4 Row0{{r[0][0], r[1][0], r[2][0], r[3][0]}};
  vec4 Dot0 = m[0] * Row0;
  float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
  float OneOverDeterminant = 1.0f / Dot1;
  for (int c = 0; c < 4; c++) r[c] = r[c] * OneOverDeterminant;
  return r;
}

void Philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

namespace {

// Host RNG stream for scene-load draws (PerlinNoiseGen.cpp:41-103 draws from RandReal()).
struct LoadRng {
  uint32_t k0, k1, a, b = 0xFFFFFFFFu, block = 0, buf[4] = {0, 0, 0, 0};
  int idx = 4;
  LoadRng(uint64_t seed, uint32_t ordinal) : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), a(ordinal) {}
  float Uniform() {
    if (idx == 4) {
      buf[0] = a;
      buf[1] = b;
      buf[2] = block++;
      buf[3] = kTagPerlin;
      Philox4x32_10(buf, k0, k1);
      idx = 0;
    }
    return (float)(buf[idx++] >> 8) * (1.0f / 16777216.0f);
  }
  float Uniform(float mn, float mx) { return mn + Uniform() * (mx - mn); }
  int Int(int mn, int mx) { return (int)Uniform((float)mn, (float)(mx + 1)); }
};

void GeneratePerlin(TextureDesc& t, uint64_t seed, uint32_t ordinal) {
  LoadRng g(seed, ordinal);
  t.perlin_vec.resize((size_t)t.point_count);
  for (int i = 0; i < t.point_count; i++) {
    float x = g.Uniform(-1, 1), y = g.Uniform(-1, 1), z = g.Uniform(-1, 1);
    t.perlin_vec[(size_t)i] = normalize(vec3{x, y, z});
  }
  auto perm = [&](std::vector<int>& p) {
    p.resize((size_t)t.point_count);
    for (int i = 0; i < t.point_count; i++) p[(size_t)i] = i;
    for (int i = t.point_count - 1; i > 0; i--) std::swap(p[(size_t)i], p[(size_t)g.Int(0, i)]);
  };
  perm(t.perm_x);
  perm(t.perm_y);
  perm(t.perm_z);
}

// nlohmann value(key, default) with the reference's default types
int GetInt(const Json& o, const char* k, int d) {
  const Json* v = o.find(k);
  return (v && (v->is_number() || v->is_bool())) ? (int)v->as_number() : d;
}
float GetFloat(const Json& o, const char* k, float d) {
  const Json* v = o.find(k);
  return (v && (v->is_number() || v->is_bool())) ? (float)v->as_number() : d;
}
// keys whose reference default is a double literal (value("radius", 0.5), value("density", 0.01))
float GetDoubleAsFloat(const Json& o, const char* k, double d) {
  const Json* v = o.find(k);
  return (float)((v && (v->is_number() || v->is_bool())) ? v->as_number() : d);
}
bool GetBool(const Json& o, const char* k, bool d) {
  const Json* v = o.find(k);
  return (v && (v->is_number() || v->is_bool())) ? v->as_bool() : d;
}
bool GetVec3(const Json& o, const char* k, vec3 d, vec3& out, std::string& err) {
  const Json* v = o.find(k);
  if (!v || v->is_null()) {
    out = d;
    return true;
  }
  if (!v->is_array() || v->items().size() < 3) {
    err = std::string("'") + k + "' must be an array of 3 numbers";
    return false;
  }
  out = vec3{(float)v->items()[0].as_number(), (float)v->items()[1].as_number(), (float)v->items()[2].as_number()};
  return true;
}

int AddObj(Scene& s, Obj o) {
  s.objs.push_back(std::move(o));
  return (int)s.objs.size() - 1;
}

// Quad.hpp:14-26
int MakeQuad(Scene& s, vec3 q, vec3 u, vec3 v, uint32_t mat) {
  Obj o;
  o.kind = kQuad;
  o.q = q;
  o.u = u;
  o.v = v;
  o.material = mat;
  vec3 n = cross(u, v);
  o.n = normalize(n);
  o.d = dot(o.n, q);
  o.w = n / dot(n, n);
  o.aabb = AABB(AABB(q, (q + u) + v), AABB(q + u, q + v));
  return AddObj(s, std::move(o));
}

// HittableList::Add (HittableList.hpp:13-16)
void ListAdd(Scene& s, int list, int child) {
  s.objs[(size_t)list].children.push_back(child);
  s.objs[(size_t)list].aabb = AABB(s.objs[(size_t)list].aabb, s.objs[(size_t)child].aabb);
}
int MakeList(Scene& s) {
  Obj o;
  o.kind = kList;
  return AddObj(s, std::move(o));
}

// Quad.hpp:34-50
int MakeBox(Scene& s, vec3 a, vec3 b, uint32_t mat) {
  vec3 mn{std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)};
  vec3 mx{std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)};
  vec3 dx{mx.x - mn.x, 0, 0}, dy{0, mx.y - mn.y, 0}, dz{0, 0, mx.z - mn.z};
  int l = MakeList(s);
  ListAdd(s, l, MakeQuad(s, vec3{mn.x, mn.y, mx.z}, dx, dy, mat));   // front
  ListAdd(s, l, MakeQuad(s, vec3{mx.x, mn.y, mx.z}, -dz, dy, mat));  // right
  ListAdd(s, l, MakeQuad(s, vec3{mx.x, mn.y, mn.z}, -dx, dy, mat));  // back
  ListAdd(s, l, MakeQuad(s, vec3{mn.x, mn.y, mn.z}, dz, dy, mat));   // left
  ListAdd(s, l, MakeQuad(s, vec3{mn.x, mx.y, mx.z}, dx, -dz, mat));  // top
  ListAdd(s, l, MakeQuad(s, vec3{mn.x, mn.y, mn.z}, dx, dz, mat));   // bottom
  return l;
}

// Sphere.hpp:21-29 (the moving constructor, which the loader always uses)
int MakeSphere(Scene& s, vec3 c0, vec3 disp, float r, uint32_t mat) {
  Obj o;
  o.kind = kSphere;
  o.c0 = c0;
  o.disp = disp;
  o.radius = r;
  o.material = mat;
  vec3 at0 = c0 + disp * 0.0f, at1 = c0 + disp * 1.0f;
  o.aabb = AABB(AABB(at0 - vec3(r), at0 + vec3(r)), AABB(at1 - vec3(r), at1 + vec3(r)));
  return AddObj(s, std::move(o));
}

// Transform.cpp:36-73
int MakeXform(Scene& s, int child, const mat4& model) {
  Obj o;
  o.kind = kXform;
  o.child = child;
  o.model = model;
  o.inv_model = inverse(model);
  const AABB& e = s.objs[(size_t)child].aabb;
  vec3 mn{e.x.min, e.y.min, e.z.min}, mx{e.x.max, e.y.max, e.z.max};
  vec3 corners[8] = {{mn.x, mn.y, mn.z}, {mx.x, mn.y, mn.z}, {mn.x, mx.y, mn.z}, {mx.x, mx.y, mn.z},
                     {mn.x, mn.y, mx.z}, {mx.x, mn.y, mx.z}, {mn.x, mx.y, mx.z}, {mx.x, mx.y, mx.z}};
  vec3 nmin(kInfinity), nmax(-kInfinity);
  for (const vec3& c : corners) {
    vec3 t = transform_point(model, c);
    nmin = vec3{std::fmin(nmin.x, t.x), std::fmin(nmin.y, t.y), std::fmin(nmin.z, t.z)};
    nmax = vec3{std::fmax(nmax.x, t.x), std::fmax(nmax.y, t.y), std::fmax(nmax.z, t.z)};
  }
  o.aabb = AABB(nmin, nmax);
  return AddObj(s, std::move(o));
}

// ConstantMedium.cpp:10-12
int MakeMedium(Scene& s, int boundary, float density, uint32_t mat) {
  Obj o;
  o.kind = kMedium;
  o.child = boundary;
  o.neg_inv_density = (float)(-1.0 / (double)density);
  o.material = mat;
  o.aabb = s.objs[(size_t)boundary].aabb;
  return AddObj(s, std::move(o));
}

// BVH.cpp:10-31
int MakeBvh(Scene& s, std::vector<int>& objects, size_t start, size_t end) {
  Obj node;
  node.kind = kBvh;
  size_t span = end - start;
  for (size_t i = start; i < end; i++) node.aabb = AABB(node.aabb, s.objs[(size_t)objects[i]].aabb);
  if (span == 1) {
    node.left = node.right = objects[start];
  } else if (span == 2) {
    node.left = objects[start];
    node.right = objects[start + 1];
  } else {
    int axis = node.aabb.LongestAxis();
    const std::vector<Obj>& objs = s.objs;
    std::sort(objects.begin() + (long)start, objects.begin() + (long)end, [&objs, axis](int a, int b) {
      return objs[(size_t)a].aabb.Axis(axis).min < objs[(size_t)b].aabb.Axis(axis).min;
    });
    size_t mid = start + span / 2;
    node.left = MakeBvh(s, objects, start, mid);
    node.right = MakeBvh(s, objects, mid, end);
  }
  return AddObj(s, std::move(node));
}

// Serialize.cpp:106-132 (ParseTransform): T * R * S
bool ParseTransform(const Json& tj, mat4& out, std::string& err) {
  vec3 tr, sc;
  if (!GetVec3(tj, "translation", {0, 0, 0}, tr, err)) return false;
  if (!GetVec3(tj, "scale", {1, 1, 1}, sc, err)) return false;
  // Missing "rotation" leaves glm::quat uninitialised in the reference (undefined behaviour,
  // Serialize.cpp:114); defined here as the identity rotation.
  float qw = 1, qx = 0, qy = 0, qz = 0;
  if (const Json* r = tj.find("rotation")) {
    if (!r->is_array() || r->items().size() < 4) {
      err = "'rotation' must be [angle_deg, ax, ay, az]";
      return false;
    }
    float angle = radians((float)r->items()[0].as_number());
    vec3 axis{(float)r->items()[1].as_number(), (float)r->items()[2].as_number(), (float)r->items()[3].as_number()};
    float sn = std::sin(angle * 0.5f);  // glm::angleAxis
    qw = std::cos(angle * 0.5f);
    qx = axis.x * sn;
    qy = axis.y * sn;
    qz = axis.z * sn;
  }
  mat4 T = mat4::identity();
  T[3] = vec4{{tr.x, tr.y, tr.z, 1.0f}};
  float qxx = qx * qx, qyy = qy * qy, qzz = qz * qz, qxz = qx * qz, qxy = qx * qy, qyz = qy * qz;
  float qwx = qw * qx, qwy = qw * qy, qwz = qw * qz;
  mat4 R = mat4::identity();  // glm::toMat4 / mat3_cast
  R[0][0] = 1.f - 2.f * (qyy + qzz);
  R[0][1] = 2.f * (qxy + qwz);
  R[0][2] = 2.f * (qxz - qwy);
  R[1][0] = 2.f * (qxy - qwz);
  R[1][1] = 1.f - 2.f * (qxx + qzz);
  R[1][2] = 2.f * (qyz + qwx);
  R[2][0] = 2.f * (qxz + qwy);
  R[2][1] = 2.f * (qyz - qwx);
  R[2][2] = 1.f - 2.f * (qxx + qyy);
  mat4 S = mat4::identity();
  S[0][0] = sc.x;
  S[1][1] = sc.y;
  S[2][2] = sc.z;
  out = matmul(matmul(T, R), S);
  return true;
}

// Serialize.cpp:161-197 (ParseNode)
int ParseNode(Scene& s, const Json& node, std::string& err, int depth) {
  if (depth > 64) {
    err = "scene graph nested too deeply";
    return -1;
  }
  int ret = -1;
  if (node.contains("primitive")) {
    int idx = GetInt(node, "primitive", -1);
    if (idx < 0) {
      err = "primitive must be a non-negative integer";
      return -1;
    }
    if (idx >= (int)s.primitives.size()) {
      err = "primitive out of range of primitives";
      return -1;
    }
    ret = s.primitives[(size_t)idx];
  }
  if (const Json* children = node.find("children")) {
    if (!children->is_array()) {
      err = "children entry must be an array";
      return -1;
    }
    int l = MakeList(s);
    if (ret >= 0) ListAdd(s, l, ret);
    for (const Json& c : children->items()) {
      int ch = ParseNode(s, c, err, depth + 1);
      if (ch < 0) return -1;
      ListAdd(s, l, ch);
    }
    ret = l;
  }
  if (ret < 0) {
    err = "error parsing node";
    return -1;
  }
  if (const Json* tj = node.find("transform")) {
    if (tj->is_object()) {
      mat4 m;
      if (!ParseTransform(*tj, m, err)) return -1;
      return MakeXform(s, ret, m);
    }
  }
  return ret;
}

std::string DirOf(const std::string& p) {
  size_t k = p.find_last_of('/');
  return k == std::string::npos ? std::string("") : p.substr(0, k + 1);
}

bool CameraFromJson(const Json& o, Camera& cam, std::string& err) {
  cam = Camera();
  cam.SetFOV((float)GetInt(o, "fov", 90));  // value("fov", 90): an int, fractional fov truncates
  vec3 c, l;
  if (!GetVec3(o, "center", {0, 0, 1}, c, err) || !GetVec3(o, "look_at", {0, 0, 0}, l, err)) return false;
  cam.SetCenter(c);
  cam.SetLookAt(l);
  cam.SetDefocusAngle(GetFloat(o, "defocus_angle", 0.0f));
  cam.SetFocusDistance(GetFloat(o, "focus_distance", 1.f));
  return true;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Camera.hpp:16-48
void Camera::Update() {
  if (!dirty_) return;
  dirty_ = false;
  float theta = radians(vfov_);
  float h = std::tan(theta / 2);
  vec3 w = normalize(center_ - lookat_);
  vec3 u = normalize(cross(view_up_, w));
  vec3 v = cross(w, u);
  float viewport_height = (float)(2.0 * (double)h * (double)focus_dist_);
  float viewport_width = viewport_height * ((float)dims_x_ / (float)dims_y_);
  vec3 lu = viewport_width * u;
  vec3 lv = viewport_height * v;
  pixel_delta_u_ = lu / (float)dims_x_;
  pixel_delta_v_ = lv / (float)dims_y_;
  viewport_upper_left_ = ((center_ - (w * focus_dist_)) - lu / 2.0f) - lv / 2.0f;
  pixel00_loc_ = viewport_upper_left_ + 0.5f * (pixel_delta_u_ + pixel_delta_v_);
  float defocus_radius = focus_dist_ * std::tan(radians(defocus_angle_ / 2));
  defocus_disk_u_ = u * defocus_radius;
  defocus_disk_v_ = v * defocus_radius;
  sqrt_spp_ = (int)std::sqrt((double)samples_per_pixel_);
  recip_sqrt_spp_ = (float)(1.0 / (double)sqrt_spp_);
}

CameraParams Camera::Params() {
  Update();
  CameraParams p;
  auto put = [](float* d, vec3 v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
  };
  put(p.pixel00, pixel00_loc_);
  put(p.du, pixel_delta_u_);
  put(p.dv, pixel_delta_v_);
  put(p.center, center_);
  put(p.defocus_u, defocus_disk_u_);
  put(p.defocus_v, defocus_disk_v_);
  p.defocus_angle = defocus_angle_;
  p.recip_sqrt_spp = recip_sqrt_spp_;
  p.sqrt_spp = sqrt_spp_;
  return p;
}

bool LoadCameraFile(const std::string& path, Camera& out, std::string& err) {
  Json o;
  if (!Json::ParseFile(path, o, err)) return false;
  return CameraFromJson(o, out, err);
}

std::string CameraToJson(const Camera& cam) {
  auto arr = [](vec3 v) {
    Json a = Json::array();
    a.push_back(Json::number(v.x));
    a.push_back(Json::number(v.y));
    a.push_back(Json::number(v.z));
    return a;
  };
  Json o = Json::object();  // Serialize.cpp:47-54
  o.set("fov", Json::number(cam.vfov_));
  o.set("center", arr(cam.center_));
  o.set("look_at", arr(cam.lookat_));
  o.set("defocus_angle", Json::number(cam.defocus_angle_));
  o.set("focus_distance", Json::number(cam.focus_dist_));
  return o.Dump(2) + "\n";
}

bool WriteCameraFile(const Camera& cam, const std::string& path, std::string& err) {
  std::ofstream f(path, std::ios::binary);
  if (!f) {
    err = "cannot write " + path;
    return false;
  }
  f << CameraToJson(cam);
  return true;
}

bool LoadAppSettingsFile(const std::string& path, AppSettings& out, std::string& err) {
  Json o;
  if (!Json::ParseFile(path, o, err)) return false;
  out = AppSettings();  // Serialize.cpp:56-65
  out.num_samples = GetInt(o, "num_samples", 1);
  out.render_once = GetBool(o, "render_once", false);
  out.save_after_render_once = GetBool(o, "save_after_render_once", false);
  out.max_depth = GetInt(o, "max_depth", 50);
  out.render_window = GetBool(o, "render_window", true);
  return true;
}

// Serialize.cpp:199-360 + App.cpp:122-126
bool LoadScene(const std::string& path, uint64_t seed, Scene& s, std::string& err) {
  s = Scene();
  Json obj;
  if (!Json::ParseFile(path, obj, err)) return false;
  auto fail = [&](const std::string& m) {
    err = "Failed to parse Scene: " + m + ". " + path;
    return false;
  };
  if (!obj.is_object()) return fail("top level must be an object");
  if (!GetVec3(obj, "background_color", {1, 1, 1}, s.background, err)) return fail(err);

  const Json* cam = obj.find("camera");
  if (cam && cam->is_object()) {
    if (!CameraFromJson(*cam, s.cam, err)) return fail(err);
  } else {
    // A string names data/<name>.json next to the scene. Legacy files have no camera at all:
    // the adapter uses cam1 (the RTIOW book-1 camera its sibling scenes name; SURVEY Finding 3).
    std::string name = (cam && cam->is_string()) ? cam->as_string() : std::string("cam1");
    if (cam && !cam->is_string() && !cam->is_null()) return fail("camera must be an object or a name");
    s.cam_name = name + ".json";
    std::string e2;
    if (!LoadCameraFile(DirOf(path) + s.cam_name, s.cam, e2)) return fail(e2);
  }

  uint32_t noise_ordinal = 0;
  if (const Json* tx = obj.find("textures")) {
    if (tx->is_array()) {
      for (const Json& t : tx->items()) {
        TextureDesc tex;
        const Json* ty = t.find("type");
        std::string type = (ty && ty->is_string()) ? ty->as_string() : "";
        if (type == "solid_color") {
          tex.type = kTexSolid;
          if (!GetVec3(t, "albedo", {1, 1, 1}, tex.albedo, err)) return fail(err);
        } else if (type == "checker") {
          tex.type = kTexChecker;
          tex.inv_scale = 1.f / GetFloat(t, "scale", 1.0f);
          tex.even = (uint32_t)GetInt(t, "even_tex_idx", 0);
          tex.odd = (uint32_t)GetInt(t, "odd_tex_idx", 0);
        } else if (type == "noise") {
          tex.type = kTexNoise;
          tex.point_count = GetInt(t, "point_count", 256);
          if (tex.point_count < 256 || tex.point_count > 4096)
            return fail("noise point_count must be in [256, 4096] (indices are taken & 255)");
          GeneratePerlin(tex, seed, noise_ordinal++);
          if (!GetVec3(t, "albedo", {1, 1, 1}, tex.albedo, err)) return fail(err);
          tex.scale = GetFloat(t, "scale", 1.0f);
          tex.noise_type = GetInt(t, "noise_type", 1);
        } else {
          return fail("Invalid texture type: " + type);
        }
        s.textures.push_back(std::move(tex));
      }
    }
  }

  if (const Json* mats = obj.find("materials")) {
    if (!mats->is_array()) return fail("materials must be an array");
    for (const Json& m : mats->items()) {
      const Json* ty = m.find("type");
      std::string type = (ty && ty->is_string()) ? ty->as_string() : "";
      if (type.empty()) return fail("material type field empty");
      MaterialDesc md;
      if (type == "lambertian") {
        md.type = kMatLambertian;
        if (!GetVec3(m, "albedo", {1, 1, 1}, md.albedo, err)) return fail(err);
      } else if (type == "dielectric") {
        md.type = kMatDielectric;
        md.refraction_index = GetFloat(m, "refraction_index", 1.0f);
      } else if (type == "metal") {
        md.type = kMatMetal;
        if (!GetVec3(m, "albedo", {1, 1, 1}, md.albedo, err)) return fail(err);
        md.fuzz = GetFloat(m, "fuzz", 0.0f);
      } else if (type == "texture" || type == "diffuse_light") {
        md.type = type == "texture" ? kMatTexture : kMatDiffuseLight;
        if (m.contains("tex_idx")) {
          md.tex_idx = (uint32_t)GetInt(m, "tex_idx", 0);
        } else if (m.contains("albedo")) {
          md.tex_idx = (uint32_t)s.textures.size();
          TextureDesc t;
          if (!GetVec3(m, "albedo", {1, 1, 1}, t.albedo, err)) return fail(err);
          s.textures.push_back(std::move(t));
        } else {
          return fail(type == "texture" ? "invalid texture, must contain tex_idx or albedo"
                                        : "invalid diffuse light, must contain tex_idx or albedo");
        }
      } else {
        return fail("Invalid material type");
      }
      s.materials.push_back(md);
    }
  }

  const Json* prims = obj.find("primitives");
  if (prims && prims->is_object()) {
    // Legacy schema (the reference's current loader throws on it, Serialize.cpp:288-290):
    // {"spheres": [{center, radius, material_id, displacement?}], "quads": [{q, u, v, material_id}],
    //  "boxes": [{a, b, material_id}]}. Documented adapter (SURVEY.md Finding 3): the groups in the
    // order the file lists them, each in array order; every primitive is one top-level scene node
    // (a box is MakeBox's 6-quad list, Quad.hpp:34-50).
    s.legacy_schema = true;
    for (const auto& grp : prims->members()) {
      const std::string& kind = grp.first;
      if (kind != "spheres" && kind != "quads" && kind != "boxes")
        return fail("legacy primitives: unknown group '" + kind + "'");
      if (!grp.second.is_array()) return fail("legacy primitives: '" + kind + "' must be an array");
      for (const Json& p : grp.second.items()) {
        const uint32_t mat = (uint32_t)GetInt(p, "material_id", 0);
        int o = -1;
        if (kind == "spheres") {
          vec3 c, d;
          if (!GetVec3(p, "center", {0, 0, 0}, c, err) || !GetVec3(p, "displacement", {0, 0, 0}, d, err))
            return fail(err);
          o = MakeSphere(s, c, d, GetDoubleAsFloat(p, "radius", 0.5), mat);
        } else if (kind == "quads") {
          vec3 q, u, v;
          if (!GetVec3(p, "q", {0, 0, 0}, q, err) || !GetVec3(p, "u", {1, 0, 0}, u, err) ||
              !GetVec3(p, "v", {0, 0, 1}, v, err))
            return fail(err);
          o = MakeQuad(s, q, u, v, mat);
        } else {
          vec3 a, b;
          if (!GetVec3(p, "a", {0, 0, 0}, a, err) || !GetVec3(p, "b", {1, 1, 1}, b, err)) return fail(err);
          o = MakeBox(s, a, b, mat);
        }
        s.primitives.push_back(o);
        s.top.push_back(o);
      }
    }
  } else if (prims && prims->is_array()) {
    for (const Json& p : prims->items()) {
      const Json* ty = p.find("type");
      std::string type = (ty && ty->is_string()) ? ty->as_string() : "";
      if (type.empty()) return fail("Primitive needs type entry");
      uint32_t mat = (uint32_t)GetInt(p, "material", 0);
      int h = -1;
      if (type == "quad") {
        vec3 q, u, v;
        if (!GetVec3(p, "q", {0, 0, 0}, q, err) || !GetVec3(p, "u", {1, 0, 0}, u, err) ||
            !GetVec3(p, "v", {0, 0, 1}, v, err))
          return fail(err);
        h = MakeQuad(s, q, u, v, mat);
      } else if (type == "box") {
        vec3 a, b;
        if (!GetVec3(p, "a", {0, 0, 0}, a, err) || !GetVec3(p, "b", {1, 1, 1}, b, err)) return fail(err);
        h = MakeBox(s, a, b, mat);
      } else if (type == "sphere") {
        vec3 c, d;
        if (!GetVec3(p, "center", {0, 0, 0}, c, err) || !GetVec3(p, "displacement", {0, 0, 0}, d, err))
          return fail(err);
        h = MakeSphere(s, c, d, GetDoubleAsFloat(p, "radius", 0.5), mat);
      } else {
        return fail("invalid primitive type: " + type);
      }
      if (const Json* cm = p.find("constant_medium")) {
        uint32_t midx;
        if (cm->contains("albedo")) {
          MaterialDesc iso;
          iso.type = kMatIsotropic;
          iso.tex_idx = (uint32_t)s.textures.size();
          TextureDesc t;
          if (!GetVec3(*cm, "albedo", {0, 0, 0}, t.albedo, err)) return fail(err);
          s.textures.push_back(std::move(t));
          midx = (uint32_t)s.materials.size();
          s.materials.push_back(iso);
        } else if (cm->contains("material")) {
          midx = (uint32_t)GetInt(*cm, "material", 0);
        } else {
          return fail("constant_medium must contain 'albedo' or 'material'");
        }
        h = MakeMedium(s, h, GetDoubleAsFloat(*cm, "density", 0.01), midx);
      }
      s.primitives.push_back(h);
    }
    if (const Json* nodes = obj.find("scene")) {
      for (const Json& n : nodes->items()) {
        int h = ParseNode(s, n, err, 0);
        if (h < 0) return fail(err);
        s.top.push_back(h);
      }
    }
  }

  if (cam && cam->is_object()) {
    int width = GetInt(*cam, "width", 0);
    float aspect = GetFloat(*cam, "aspect_ratio", 0.0f);
    if (width != 0 && aspect != 0.0f) {
      float height = (float)width / aspect;
      s.dims_x = width;
      s.dims_y = (int)height;
    }
  }
  // index validation (the reference reads out of bounds instead)
  for (const Obj& o : s.objs) {
    if ((o.kind == kQuad || o.kind == kSphere || o.kind == kMedium) && o.material >= s.materials.size())
      return fail("material index " + std::to_string(o.material) + " out of range");
  }
  for (const MaterialDesc& m : s.materials) {
    if ((m.type == kMatTexture || m.type == kMatDiffuseLight || m.type == kMatIsotropic) &&
        m.tex_idx >= s.textures.size())
      return fail("texture index out of range");
  }
  for (const TextureDesc& t : s.textures) {
    if (t.type == kTexChecker && (t.even >= s.textures.size() || t.odd >= s.textures.size()))
      return fail("checker texture index out of range");
  }
  if (s.top.empty()) return fail("scene has no objects (the reference's BVHNode recurses forever on an empty list)");
  std::vector<int> objects = s.top;  // BVHNode(HittableList list) sorts a copy
  s.root = MakeBvh(s, objects, 0, objects.size());
  return true;
}

}  // namespace rt2
