// AddressSanitizer + UndefinedBehaviorSanitizer driver for the host code (SURVEY.md §5 "sanitizers";
// the reference's own debug build is -Wall -Werror only, /root/reference/src/CMakeLists.txt:31-37).
// Built by tests/test_sanitize.py with -fsanitize=address,undefined -fno-sanitize-recover=all over
// json.cpp, scene.cpp, compile.cpp, image.cpp (the product's loader, compiler and image writer) and
// oracle/rt_oracle.cpp (the CPU restatement), then run on:
//   --good <scene.json>...   every committed scene: LoadScene (Serialize.cpp:199-360 + the legacy
//                            adapter), CompileScene with and without list trees, Camera::Params at the
//                            BASELINE sizes, the oracle's loader and an 8x8, 2-frame oracle render in both
//                            product orders; every byte prefix of the small ones and single-byte
//                            corruptions of each (all must fail cleanly or load);
//   --bad <doc.json>...      malformed documents: both loaders must refuse them with an error text;
//   --camera <cam.json>...   LoadCamera / WriteCamera round trip (Serialize.cpp:32-54);
//   --out <dir>              scratch directory for the fuzzed documents and WriteImage output.
// Exits non-zero on a contract violation; a sanitizer finding aborts the process (exit 1 + report).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "scene.h"

namespace rt2 {
bool WriteImage(const float* pixels, int w, int h, const std::string& path, bool png, std::string& err);
}

extern "C" {
struct oracle_counters {
  uint64_t rays, bvh, quad, sphere, xform, medium, list, rng_draws;
};
void* oracle_scene_load(const char* path, uint64_t seed);
void oracle_scene_free(void* s);
const char* oracle_last_error();
int oracle_render(void* sp, int W, int H, int spp, int max_depth, uint64_t seed, int frame_begin, int n_frames,
                  int band_h, int rank, int world, float* accum, uint32_t* ray_counts, int threads, int forward,
                  oracle_counters* out_cnt);
}

using namespace rt2;

static int g_fail = 0;
static void Fail(const std::string& what) {
  std::fprintf(stderr, "FAIL: %s\n", what.c_str());
  g_fail = 1;
}

static std::string ReadAll(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}
static void WriteAll(const std::string& p, const std::string& s) {
  std::ofstream f(p, std::ios::binary | std::ios::trunc);
  f << s;
}

// One document through both loaders; returns whether the product loader accepted it. A document the
// product accepts is also compiled (both list modes) and its camera evaluated.
static bool Exercise(const std::string& path, bool render) {
  Scene s;
  std::string err;
  const bool ok = LoadScene(path, 0x5EED2024ull, s, err);
  if (!ok && err.empty()) Fail(path + ": refused without an error text");
  if (ok) {
    for (int accel = 0; accel < 2; accel++) {
      CompiledScene c;
      std::string e2;
      if (!CompileScene(s, c, e2, accel != 0)) Fail(path + ": compile: " + e2);
    }
    const int dims[4][3] = {{400, 400, 64}, {1024, 1024, 1000}, {1920, 1080, 500}, {800, 800, 10000}};
    for (const auto& d : dims) {
      Camera cam = s.cam;
      cam.SetDims(d[0], d[1]);
      cam.SetSamplesPerPixel(d[2]);
      (void)cam.Params();
    }
  }
  void* o = oracle_scene_load(path.c_str(), 0x5EED2024ull);
  if (o == nullptr && std::strlen(oracle_last_error()) == 0) Fail(path + ": oracle refused without an error text");
  if (o != nullptr && render) {
    const int w = 8, h = 8;
    for (int forward = 0; forward < 2; forward++) {
      std::vector<float> acc((size_t)w * h * 3, 0.0f);
      std::vector<uint32_t> rc((size_t)w * h, 0u);
      oracle_counters cnt{};
      oracle_render(o, w, h, 4, 50, 0x5EED2024ull, 0, 2, 0, 0, 1, acc.data(), rc.data(), 2, forward, &cnt);
      if (cnt.rays == 0) Fail(path + ": oracle render issued no rays");
    }
  }
  if (o != nullptr) oracle_scene_free(o);
  return ok;
}

int main(int argc, char** argv) {
  std::vector<std::string> good, bad, cams;
  std::string out = "/tmp";
  std::vector<std::string>* cur = nullptr;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    if (a == "--good") cur = &good;
    else if (a == "--bad") cur = &bad;
    else if (a == "--camera") cur = &cams;
    else if (a == "--out" && i + 1 < argc) out = argv[++i];
    else if (cur != nullptr) cur->push_back(a);
  }
  size_t docs = 0, accepted = 0;
  for (const auto& p : good) {
    if (!Exercise(p, true)) Fail(p + ": a committed scene did not load");
    docs++;
    const std::string text = ReadAll(p);
    const std::string tmp = out + "/fuzz.json";
    // every byte prefix of the small documents (a stride through the large ones)
    const bool small = text.size() <= 4096;
    const size_t stride = small ? 1 : text.size() / 61;
    for (size_t n = 0; n < text.size(); n += stride) {
      WriteAll(tmp, text.substr(0, n));
      accepted += Exercise(tmp, false);
      docs++;
    }
    // single-byte corruptions: structural characters and digits replaced by JSON-significant bytes
    const char subst[] = {'"', '}', ']', '[', '{', ',', ':', '-', 'e', '0', '\\', '\0'};
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < (small ? 400 : 60); k++) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      std::string m = text;
      m[(size_t)(x % m.size())] = subst[(x >> 32) % sizeof(subst)];
      WriteAll(tmp, m);
      accepted += Exercise(tmp, false);
      docs++;
    }
  }
  for (const auto& p : bad) {
    docs++;
    if (Exercise(p, false)) Fail(p + ": a malformed document loaded");
  }
  for (const auto& p : cams) {
    Camera c;
    std::string err;
    if (!LoadCameraFile(p, c, err)) {
      Fail(p + ": camera: " + err);
      continue;
    }
    const std::string w = out + "/cam_rt.json";
    if (!WriteCameraFile(c, w, err)) Fail(p + ": WriteCamera: " + err);
    Camera c2;
    if (!LoadCameraFile(w, c2, err)) Fail(p + ": camera round trip: " + err);
    docs++;
  }
  // util::WriteImage over a ragged image with out-of-range values (clamped), both formats
  {
    const int w = 7, h = 5;
    std::vector<float> px((size_t)w * h * 3);
    for (size_t i = 0; i < px.size(); i++) px[i] = (float)((i * 37) % 23) / 17.0f - 0.1f;
    std::string err;
    if (!WriteImage(px.data(), w, h, out + "/img.png", true, err)) Fail("WriteImage png: " + err);
    if (!WriteImage(px.data(), w, h, out + "/img.ppm", false, err)) Fail("WriteImage ppm: " + err);
    if (WriteImage(px.data(), w, h, out + "/no/such/dir/img.png", true, err) || err.empty())
      Fail("WriteImage into a missing directory did not report an error");
  }
  std::printf("documents=%zu fuzz_accepted=%zu\n", docs, accepted);
  return g_fail;
}
