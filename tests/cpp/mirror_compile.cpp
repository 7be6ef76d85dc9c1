// Compile-only check of include/rt2/RayTracer.hpp: the headless App::Run sequence
// (src/App.cpp:115-174) written against the mirror.
#include <rt2/RayTracer.hpp>

int HeadlessRun(const char* scene_path, const char* out_png) {
  rt2::AppSettings settings;
  settings.num_samples = 64;
  rt2::serialize::SceneLoader loader;
  auto scene_opt = loader.LoadScene(scene_path);
  if (!scene_opt.has_value()) return 1;
  rt2::Scene& scene = scene_opt.value();
  rt2::ivec2 dims{1600, 900};
  if (scene.dims.x != 0 && scene.dims.y != 0) dims = scene.dims;
  rt2::RayTracer tracer(scene, 0);
  tracer.max_depth = settings.max_depth;
  scene.cam.SetSamplesPerPixel((int)settings.num_samples);
  tracer.camera = &scene.cam;
  tracer.OnResize(dims);
  for (size_t i = 0; i < settings.num_samples; i++) tracer.Update(scene);
  rt2::util::WriteImage(tracer.NonConvertedPixels(), tracer.Dims().x, tracer.Dims().y, out_png);
  return tracer.FrameIdx() == settings.num_samples ? 0 : 2;
}
