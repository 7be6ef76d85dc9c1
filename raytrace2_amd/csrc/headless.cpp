// headless.cpp — the reference's headless App::Run path (src/App.cpp:81-174, 243-248) written against
// the C++ mirror include/rt2/RayTracer.hpp: load the settings and the scene, num_samples x
// Update(), WriteImage(NonConvertedPixels()). It is the integration check of the C++ drop-in
// boundary (tests/test_gpu_headless.py runs it and compares its PNG with the Python path's).
//
//   rt2_headless <scene.json> <out.png> [--settings settings.json] [--samples N] [--size WxH] [--gpus N]
//
// Without --settings the reference's Settings.hpp defaults apply (num_samples 1, max_depth 50);
// --samples / --size override num_samples and the output dims (App.cpp:115-124: scene dims, else
// 1600x900). --gpus N renders on GPUs 0..N-1 (row bands + RCCL gather, rt2_tracer_create_multi).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include <rt2/RayTracer.hpp>

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <scene.json> <out.png> [--settings f] [--samples N] [--size WxH]\n", argv[0]);
    return 2;
  }
  const std::string scene_path = argv[1], out_path = argv[2];
  rt2::AppSettings settings;
  long samples = -1;
  rt2::ivec2 size{0, 0};
  int gpus = 0;  // 0: the one-GPU tracer; N >= 1: rt2_tracer_create_multi over GPUs 0..N-1
  try {
    for (int i = 3; i + 1 < argc; i += 2) {
      if (!std::strcmp(argv[i], "--settings")) {
        settings = rt2::serialize::LoadAppSettings(argv[i + 1]);
      } else if (!std::strcmp(argv[i], "--samples")) {
        samples = std::atol(argv[i + 1]);
      } else if (!std::strcmp(argv[i], "--gpus")) {
        gpus = std::atoi(argv[i + 1]);
      } else if (!std::strcmp(argv[i], "--size")) {
        if (std::sscanf(argv[i + 1], "%dx%d", &size.x, &size.y) != 2) return 2;
      } else {
        std::fprintf(stderr, "unknown option %s\n", argv[i]);
        return 2;
      }
    }
    if (samples > 0) settings.num_samples = (size_t)samples;

    rt2::serialize::SceneLoader loader;
    auto scene_opt = loader.LoadScene(scene_path);
    if (!scene_opt.has_value()) {
      std::fprintf(stderr, "scene error: %s\n", loader.error.c_str());
      return 1;
    }
    rt2::Scene& scene = scene_opt.value();
    rt2::ivec2 dims{1600, 900};
    if (scene.dims.x != 0 && scene.dims.y != 0) dims = scene.dims;
    if (size.x > 0 && size.y > 0) dims = size;

    rt2::RayTracer tracer(scene, 0, gpus);
    tracer.max_depth = settings.max_depth;
    scene.cam.SetSamplesPerPixel((int)settings.num_samples);
    tracer.camera = &scene.cam;
    tracer.OnResize(dims);

    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < settings.num_samples; i++) tracer.Update(scene);
    const auto pixels = tracer.NonConvertedPixels();  // runs the queued frames
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    rt2::util::WriteImage(pixels, tracer.Dims().x, tracer.Dims().y, out_path);

    rt2_stats st{};
    rt2::Check(rt2_tracer_get_stats(tracer.handle(), &st));
    std::printf("{\"frames\": %zu, \"width\": %d, \"height\": %d, \"rays\": %llu, \"seconds\": %.6f, "
                "\"mray_s\": %.1f, \"launches\": %llu, \"gpus\": %d}\n",
                (size_t)tracer.FrameIdx(), dims.x, dims.y, (unsigned long long)st.rays, s, st.rays / s / 1e6,
                (unsigned long long)st.launches, tracer.NumGpus());
    return tracer.FrameIdx() == settings.num_samples ? 0 : 3;
  } catch (const rt2::Error& e) {
    std::fprintf(stderr, "rt2 error %d: %s\n", e.code, e.what());
    return 1;
  }
}
