// rt2/RayTracer.hpp — header-only C++ mirror of the reference's hot-path interface over the C ABI
// (include/rt2.h), so reference callers (App::Run, src/App.cpp:81-249) switch by changing includes:
//
//   reference                                   here
//   raytrace2::cpu::RayTracer                   rt2::RayTracer          (RayTracer.hpp:15-42)
//   raytrace2::cpu::Scene (+ App.cpp:126 BVH)   rt2::Scene
//   raytrace2::cpu::Camera (scene.cam)          rt2::Camera (scene.cam, a value type)
//   serialize::SceneLoader::LoadScene           rt2::serialize::SceneLoader::LoadScene
//   serialize::LoadCamera / WriteCamera         rt2::serialize::LoadCamera / WriteCamera
//   serialize::LoadAppSettings                  rt2::serialize::LoadAppSettings
//   util::WriteImage                            rt2::util::WriteImage
//
// Differences a caller sees: the tracer renders on GPUs (device index, or a GPU count, at
// construction) and owns device buffers; Update() takes the scene only for signature compatibility
// (the scene program was uploaded at construction); errors throw rt2::Error (the C ABI itself never
// throws). With n_gpus > 1 the image is split into interleaved row bands over the GPUs and gathered
// over RCCL before every readback (rt2_tracer_create_multi); results are identical to one GPU.
#pragma once

#include <cstdint>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../rt2.h"

namespace rt2 {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void Check(int rc) {
  if (rc < 0) throw Error(rc, rt2_last_error());
}

struct ivec2 {
  int x = 0, y = 0;
};
struct vec3 {
  float x = 0, y = 0, z = 0;
};
struct u8vec4 {
  uint8_t x = 0, y = 0, z = 0, w = 0;
};
using PixelArray = std::vector<u8vec4>;

// The camera fields the scene files carry (Camera.hpp:113-123); Update() happens on the device side.
struct Camera {
  vec3 center_{0, 0, 1}, lookat_{0, 0, 0}, view_up_{0, 1, 0};
  float vfov_ = 90.f, defocus_angle_ = 0, focus_dist_ = 1;
  int samples_per_pixel_ = 1;

  void SetCenter(const vec3& c) { center_ = c; }
  void SetLookAt(const vec3& c) { lookat_ = c; }
  void SetViewUp(const vec3& c) { view_up_ = c; }
  void SetFOV(float f) { vfov_ = f; }
  void SetDefocusAngle(float a) { defocus_angle_ = a; }
  void SetFocusDistance(float d) { focus_dist_ = d; }
  void SetSamplesPerPixel(int s) { samples_per_pixel_ = s; }
  [[nodiscard]] float GetFOV() const { return vfov_; }
  [[nodiscard]] int SamplesPerPixel() const { return samples_per_pixel_; }

  rt2_camera_desc Desc() const {
    rt2_camera_desc d{};
    d.center[0] = center_.x, d.center[1] = center_.y, d.center[2] = center_.z;
    d.look_at[0] = lookat_.x, d.look_at[1] = lookat_.y, d.look_at[2] = lookat_.z;
    d.view_up[0] = view_up_.x, d.view_up[1] = view_up_.y, d.view_up[2] = view_up_.z;
    d.vfov = vfov_, d.defocus_angle = defocus_angle_, d.focus_distance = focus_dist_;
    return d;
  }
  static Camera FromDesc(const rt2_camera_desc& d) {
    Camera c;
    c.center_ = {d.center[0], d.center[1], d.center[2]};
    c.lookat_ = {d.look_at[0], d.look_at[1], d.look_at[2]};
    c.view_up_ = {d.view_up[0], d.view_up[1], d.view_up[2]};
    c.vfov_ = d.vfov, c.defocus_angle_ = d.defocus_angle, c.focus_dist_ = d.focus_distance;
    return c;
  }
};

struct AppSettings {  // Settings.hpp:5-11
  bool render_once = false;
  bool save_after_render_once = false;
  size_t num_samples = 1;
  size_t max_depth = 50;
  bool render_window = true;
};

// A loaded scene: materials, textures, object graph with the top-level BVH (App.cpp:126).
class Scene {
 public:
  explicit Scene(rt2_scene* h) : h_(h, &rt2_scene_free) {
    rt2_camera_desc d{};
    Check(rt2_scene_get_camera(h, &d));
    cam = Camera::FromDesc(d);
    rt2_scene_info info{};
    Check(rt2_scene_get_info(h, &info));
    dims = {info.dims_x, info.dims_y};
    background_color = {info.background[0], info.background[1], info.background[2]};
  }
  rt2_scene* handle() const { return h_.get(); }

  Camera cam;
  ivec2 dims;
  vec3 background_color{1, 1, 1};

 private:
  std::shared_ptr<rt2_scene> h_;
};

namespace serialize {

struct SceneLoader {
  uint64_t seed = 0x5EED2024ull;
  std::string error;
  // Serialize.hpp:22 — std::nullopt on a schema error (message in `error`)
  [[nodiscard]] std::optional<Scene> LoadScene(const std::string& filepath) {
    rt2_scene* h = nullptr;
    if (rt2_scene_load(filepath.c_str(), seed, &h) != RT2_OK) {
      error = rt2_last_error();
      return std::nullopt;
    }
    return Scene(h);
  }
};

inline Camera LoadCamera(const std::string& filepath) {
  rt2_camera_desc d{};
  Check(rt2_camera_load(filepath.c_str(), &d));
  return Camera::FromDesc(d);
}

inline void WriteCamera(const Camera& cam, const std::string& filepath) {
  rt2_camera_desc d = cam.Desc();
  Check(rt2_camera_write(&d, filepath.c_str()));
}

inline AppSettings LoadAppSettings(const std::string& filepath) {
  rt2_app_settings s{};
  Check(rt2_settings_load(filepath.c_str(), &s));
  AppSettings a;
  a.render_once = s.render_once != 0;
  a.save_after_render_once = s.save_after_render_once != 0;
  a.num_samples = (size_t)s.num_samples;
  a.max_depth = (size_t)s.max_depth;
  a.render_window = s.render_window != 0;
  return a;
}

}  // namespace serialize

namespace util {
inline void WriteImage(const std::vector<vec3>& pixels, int width, int height, const std::string& out_path,
                       bool png = true) {
  Check(rt2_write_image(reinterpret_cast<const float*>(pixels.data()), width, height, out_path.c_str(), png ? 1 : 0));
}
}  // namespace util

// cpu::RayTracer (RayTracer.hpp:15-42) on MI355X GPUs: one GPU (`device`; n_gpus 0), or `n_gpus`
// GPUs starting at `device` with an RCCL gather of their row bands (band_h 0 = 2 rows; n_gpus 1
// is the same path with a communicator of size 1).
class RayTracer {
 public:
  explicit RayTracer(const Scene& scene, int device = 0, int n_gpus = 0, int band_h = 0) {
    rt2_tracer* t = nullptr;
    if (n_gpus <= 0) {
      Check(rt2_tracer_create(scene.handle(), device, &t));
    } else {
      std::vector<int> devs((size_t)n_gpus);
      for (int i = 0; i < n_gpus; i++) devs[(size_t)i] = device + i;
      Check(rt2_tracer_create_multi(scene.handle(), n_gpus, devs.data(), band_h, &t));
    }
    t_.reset(t);
  }

  void Update(const Scene& /*scene*/) {  // one frame (RayTracer.cpp:55-70)
    Sync();
    Check(rt2_tracer_update(t_.get()));
  }
  void Render(const Scene& /*scene*/, int n_frames) {  // n x Update in one launch
    Sync();
    Check(rt2_tracer_render(t_.get(), n_frames));
  }
  void OnResize(ivec2 dims) {  // RayTracer.cpp:87-104 (includes Reset)
    dims_ = dims;
    Check(rt2_tracer_on_resize(t_.get(), dims.x, dims.y));
  }
  void Reset() { Check(rt2_tracer_reset(t_.get())); }

  [[nodiscard]] std::vector<vec3> NonConvertedPixels() const {
    std::vector<vec3> out((size_t)dims_.x * LocalRows());
    Check(rt2_tracer_non_converted_pixels(t_.get(), reinterpret_cast<float*>(out.data())));
    return out;
  }
  [[nodiscard]] const PixelArray& Pixels() const {
    pixels_.resize((size_t)dims_.x * LocalRows());
    Check(rt2_tracer_pixels(t_.get(), reinterpret_cast<uint8_t*>(pixels_.data())));
    return pixels_;
  }
  [[nodiscard]] size_t FrameIdx() const { return (size_t)rt2_tracer_frame_idx(t_.get()); }
  [[nodiscard]] ivec2 Dims() const { return dims_; }
  bool OnEvent(const void* /*sdl_event*/) { return false; }  // no window on the GPU path
  void OnImGui() {}

  // Like the reference (RayTracer.hpp:31-32): `camera` points at scene.cam and is read at every
  // Update (camera->Update(), RayTracer.cpp:56), so moving it between Update() calls takes effect
  // at the next frame; max_depth likewise.
  Camera* camera = nullptr;
  size_t max_depth = 50;

  rt2_tracer* handle() const { return t_.get(); }
  [[nodiscard]] int NumGpus() const { return rt2_tracer_n_gpus(t_.get()); }

 private:
  struct Deleter {
    void operator()(rt2_tracer* t) const { rt2_tracer_destroy(t); }
  };
  void Sync() {
    Check(rt2_tracer_set_max_depth(t_.get(), (int)max_depth));
    if (camera) {
      Check(rt2_tracer_set_samples_per_pixel(t_.get(), camera->samples_per_pixel_));
      rt2_camera_desc d = camera->Desc();
      Check(rt2_tracer_set_camera(t_.get(), &d));
    }
  }
  std::unique_ptr<rt2_tracer, Deleter> t_;
  ivec2 dims_;
  mutable PixelArray pixels_;
  int LocalRows() const { return rt2_tracer_local_rows(t_.get()); }
};

}  // namespace rt2
