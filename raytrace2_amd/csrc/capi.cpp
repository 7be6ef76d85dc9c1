// capi.cpp — implementation of include/rt2.h: scene handles, the device-side RayTracer and the
// host utilities. Device memory is owned by the tracer (hipMalloc); the caller owns host buffers.
// A multi-GPU tracer is a facade over one one-GPU tracer per device (rank i = parts[i]) plus the
// RCCL gather of their row bands to rank 0.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt2.h"
#include "scene.h"

namespace rt2 {
hipError_t LaunchRender(const RenderParams& p, int variant, bool stats, int grid, hipStream_t stream);
int RenderBlocksPerCU(int variant, int mode, bool stats, size_t lds_bytes);
hipError_t LaunchAccumulate(const float* samples, float* accum, uint8_t* pixels, uint32_t npix, int n_frames,
                            int frame_idx, hipStream_t stream);
hipError_t LaunchSelftest(int which, unsigned long long n, uint32_t seed, unsigned long long* d_out, hipStream_t stream);
int RenderMode(const RenderParams& p);
int RenderBlockSize();
int RenderVariant(uint32_t features);
uint32_t RenderVariantFeatures(int v);
size_t RenderLdsBytes(const RenderParams& p);
bool WriteImage(const float* pixels, int w, int h, const std::string& path, bool png, std::string& err);
hipError_t LaunchDeinterleave(const float* stacks, float* image, float* image_nc, uint8_t* pixels, int width, int height, int band_h,
                              int world, int max_rows, int frame_idx, hipStream_t stream);
}  // namespace rt2

using namespace rt2;

// Default bound on the per-frame sample buffers of both launch slots together (rt2.h
// rt2_tracer_set_sample_budget). Each slot gets half, so a 1024^2 image runs 1000 frames (11.7 GiB of
// samples) in one launch per slot: the headline renders one launch per step. Measured on the final
// round-6 kernel, one MI355X: DESIGN.md §3 "Sample buffer budget".
constexpr size_t kDefaultSampleBudget = size_t(24) << 30;

struct rt2_scene {
  Scene scene;
  CompiledScene compiled;
};

struct rt2_tracer {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // scene program
  void* d_nodes = nullptr;
  void* d_materials = nullptr;
  void* d_textures = nullptr;
  void* d_perlin_vec = nullptr;
  int* d_perlin_perm = nullptr;
  void* d_lin = nullptr;
  void* d_lin_wide = nullptr;
  void* d_lind = nullptr;
  uint32_t lin_len = 0;
  bool use_linear = true;
  uint32_t root = kRefNone;
  uint32_t node_records = 0;
  uint32_t features = 0;
  int max_stack = 1;
  bool stack_ok = true;  // the scene fits the stack traversal (else only the threaded program runs it)
  bool flat_xforms = true;  // no nested transforms in the threaded program (RenderParams::flat_xforms)
  bool origins_bounded = false;  // CompiledScene::origins_bounded: launches check the camera's range
  bool use_lds = true;
  bool use_hybrid = true;   // stage only the BVH prefix in LDS when the scene is too large
  bool force_hybrid = false;  // tests: hybrid even when the whole scene would fit
  uint32_t hot_records = 0;
  int cus = 0;
  int lds_per_cu = 0;       // bytes of LDS per CU
  int hybrid_cap = -1;      // tests: most BVH records staged by the hybrid mode (-1: no cap)
  int hyb_key = -1;         // cached hybrid prefix for (variant, counting)
  uint32_t hyb_records = 0;
  float background[3] = {0, 0, 0};
  Camera camera;  // RayTracer::camera (a copy of the scene camera)
  // frame buffers (local rows)
  int width = 0, height = 0, local_rows = 0;
  int band_h = 0, rank = 0, world = 1;
  float* d_accum = nullptr;
  uint8_t* d_pixels = nullptr;
  uint32_t* d_ray_counts = nullptr;
  bool ray_counts_on = false;
  uint32_t* d_work = nullptr;  // one work counter per launch slot (words 0 and 16)
  unsigned long long* d_stats = nullptr;
  bool stats_on = false;
  int64_t frame_idx = 0;  // frames launched (FrameIdx() = frame_idx + queued)
  int queued = 0;         // Update()/Render() frames not launched yet (lazy, see rt2_tracer_render)
  int lazy_max = 4096;    // launch once this many frames are queued (0: launch at every call)
  int max_depth = 50;
  uint64_t seed = 0x5EED2024ull;
  int launch_frames = 0;
  // Launch slots: a render launch runs on one of two render streams with that slot's per-frame
  // sample buffer ([frames][local pixels] float3, which lets a pixel's frames be split into chunks
  // rendered by different lanes and still be summed in frame order), chunk table and work counter;
  // its accumulate_kernel runs on the tracer's stream after it. Consecutive launches alternate
  // slots, so a launch does not wait for the previous one: its waves take the CUs the previous
  // launch's tail leaves idle (LaunchFrames).
  struct Slot {
    hipStream_t stream = nullptr;
    float* samples = nullptr;
    size_t samples_bytes = 0;
    uint32_t* chunks = nullptr;         // this slot's chunk table (ChunkSchedule)
    size_t chunks_bytes = 0;
    std::vector<uint32_t> chunks_host;  // what `chunks` holds (renders repeat one schedule: no upload)
    hipEvent_t rendered = nullptr;      // the slot's last render launch finished (tracer stream waits)
    hipEvent_t consumed = nullptr;      // the accumulate that last read `samples` finished
    bool consumed_set = false;
  };
  Slot slots[2];
  int next_slot = 0;
  bool pipeline = true;  // RT2_PIPELINE=0: every launch waits for the tracer stream (no overlap)
  // bytes: the bound on both launch slots' sample buffers together (each slot gets half; a render
  // needing more runs as several launches, rt2.h rt2_tracer_set_sample_budget)
  size_t sample_budget = kDefaultSampleBudget;
  size_t scene_bytes = 0;         // scene program, tables and small per-tracer buffers on the device
  size_t device_bytes_peak = 0;   // high-water mark of DeviceBytes()
  // chunk schedule: work left split into >= k items per lane (0: one chunk). 4 since round 6: a launch with
  // few pixels per lane (an 8-way rank) gets 60-frame chunks instead of 12 (emulated 8-way C2 job +4.8 %);
  // full-size launches are capped at 64-frame chunks either way
  int work_split = 4;
  int chunk_max = 64;                      // longest chunk (frames)
  int frame_tiles_env = -1;                // RT2_FRAME_TILES: -1 auto, 0 off, 1 on
  bool frame_tiles = false;                // this launch: items = one pixel x 64 short chunks per wave
  int frame_tile_len = 8;                  // most frames per chunk in frame-tile mode (RT2_FRAME_TILE_LEN)
  bool chunk_align = true;                 // chunks of >= kOctet frames: multiples of 4 frames
  struct Staging {                         // pinned host copies of uploaded tables, reusable once copied
    uint32_t* p;
    size_t bytes;
    hipEvent_t done;
  };
  std::vector<Staging> staging;
  int batch_max = 64;                      // most work items a wave reserves with one atomic
  int last_chunk_frames = 0;
  int occ_key = -1, occ_blocks = 1;  // cached occupancy of the last kernel instantiation
  size_t occ_lds = 0;
  int last_variant = -1;
  int last_grid = 0;
  uint64_t launches = 0;
  uint64_t paths = 0;
  // Render-kernel time, from the launches' own clocks (RenderParams::launch_clock): a ring of
  // kClockRing (start complement, end) pairs on the device, read back at the next synchronization.
  // kernel_ms is the time at least one render launch of this tracer ran (the union of the launches'
  // first-wave-to-last-wave intervals: consecutive launches overlap in a launch's tail);
  // launch_ms_sum adds the intervals up (the overlap counted twice).
  double kernel_ms = 0;
  double launch_ms_sum = 0;
  unsigned long long* d_clock = nullptr;  // [kClockRing][2]
  unsigned long long* h_clock = nullptr;  // pinned copy
  uint32_t clock_next = 0;                // next ring entry
  std::vector<uint32_t> pending;          // ring entries of launches not yet read back
  double clock_khz = 100000.0;            // hipDeviceAttributeWallClockRate
  unsigned long long busy_end = 0;        // end of the union so far (clock ticks)
  std::vector<hipEvent_t> event_pool;
  // ---- multi-GPU ----
  std::vector<rt2_tracer*> parts;  // multi tracer: one one-GPU tracer per device, parts[i] = rank i
  bool loopback = false;           // the parts share one GPU: device-local copies instead of RCCL
  ncclComm_t comm = nullptr;       // this tracer's rank in an RCCL communicator (a part, or joined)
  // root (rank 0) image: the gathered band stacks and the de-interleaved full image
  float* d_stacks = nullptr;      // [world][max_rows][W] float3
  float* d_image = nullptr;       // [H][W] float3
  float* d_image_nc = nullptr;    // [H][W] float3 NonConvertedPixels() = image / frame_idx
  uint8_t* d_image_px = nullptr;  // [H][W] RGBA8
  size_t stacks_bytes = 0, image_pixels = 0;
  int64_t image_frame = -1;  // frame index of the last gather (-1: none since the last resize/reset)
  uint64_t gathers = 0;
  double gather_ms = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> gpending;  // per-gather timing events
  // image readbacks to the host (rt2_tracer_image_*): count and device-to-host copy time
  uint64_t readbacks = 0;
  double readback_ms = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> rpending;  // async readbacks' timing events
  double enqueue_ms = 0;  // host time spent enqueueing this tracer's renders (LaunchFrames)
  uint64_t host_waits = 0;  // times the library blocked the host on this GPU (stream / event syncs, sync copies)
};

namespace {

// Row-band height of the multi-GPU partitions (band_h 0). Measured, 8-way split emulated rank by rank
// on one MI355X (job rate = all ranks' rays / the slowest rank's time), band heights 8 / 4 / 2 / 1:
// Cornell 190 / 193 / 197 / 198 k Mray/s, book 1 55.9 / 57.5 / 54.9 / 54.6 k, Cornell volume
// 119.6 / - / 121.5 / 122.4 k, book 2 9.89 / - / 10.15 / 9.81 k. Narrow bands balance the ranks
// (image cost varies smoothly with the row); 2 rows (32x2 work tiles) is within 1-5 % of the best.
constexpr int kDefaultBandH = 2;

thread_local std::string g_err;

int Fail(int code, const std::string& m) {
  g_err = m;
  return code;
}
int HipFail(hipError_t e, const char* what) {
  return Fail(RT2_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t _e = (expr);                            \
    if (_e != hipSuccess) return HipFail(_e, #expr);   \
  } while (0)

#define NCCL_TRY(expr)                                                                     \
  do {                                                                                     \
    ncclResult_t _r = (expr);                                                              \
    if (_r != ncclSuccess) return Fail(RT2_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

int LocalRows(int h, int band_h, int rank, int world) {
  int n = 0;
  for (int y = 0; y < h; y++)
    if (BandRank(y / band_h, world) == rank) n++;
  return n;
}

int BandH(const rt2_tracer* t) { return t->band_h > 0 ? t->band_h : (t->height > 0 ? t->height : 1); }

// Rows of the largest rank's band stack (every rank's accumulation is allocated this tall, so the
// gather sends equal counts; the padding rows stay zero).
int BandRowsMax(const rt2_tracer* t) { return rt2::BandRowsMax(t->height, t->band_h, t->world); }

// Rows of the accumulation buffer: the gather sends BandRowsMax rows from every rank, also at world 1
// (a band height that does not divide the image height leaves padding rows), so every buffer is that
// tall; the rows past local_rows stay zero.
int AllocRows(const rt2_tracer* t) { return BandRowsMax(t); }

void FreeImage(rt2_tracer* t) {
  (void)hipFree(t->d_stacks);
  (void)hipFree(t->d_image);
  (void)hipFree(t->d_image_nc);
  (void)hipFree(t->d_image_px);
  t->d_stacks = nullptr;
  t->d_image = nullptr;
  t->d_image_nc = nullptr;
  t->d_image_px = nullptr;
  t->stacks_bytes = 0;
  t->image_pixels = 0;
  t->image_frame = -1;
}

void FreeFrame(rt2_tracer* t) {
  for (auto& sl : t->slots) {
    if (sl.samples) (void)hipFreeAsync(sl.samples, sl.stream);  // stream-ordered (LaunchFrames)
    sl.samples = nullptr;
    sl.samples_bytes = 0;
  }
  (void)hipFree(t->d_accum);
  (void)hipFree(t->d_pixels);
  (void)hipFree(t->d_ray_counts);
  t->d_accum = nullptr;
  t->d_pixels = nullptr;
  t->d_ray_counts = nullptr;
  FreeImage(t);
}

// Device bytes this tracer holds now: the scene program and small buffers, the frame buffers, both
// launch slots' sample buffers and chunk tables, and a root's gathered image.
size_t DeviceBytes(const rt2_tracer* t) {
  const size_t n = (size_t)t->width * (size_t)AllocRows(t);
  size_t b = t->scene_bytes + (t->d_accum ? n * 12 : 0) + (t->d_pixels ? n * 4 : 0) + (t->d_ray_counts ? n * 4 : 0);
  for (const auto& sl : t->slots) b += sl.samples_bytes + sl.chunks_bytes;
  if (t->d_image) b += t->stacks_bytes + t->image_pixels * (12 + 12 + 4);
  return b;
}
void NoteDeviceBytes(rt2_tracer* t) { t->device_bytes_peak = std::max(t->device_bytes_peak, DeviceBytes(t)); }

int Realloc(rt2_tracer* t) {
  FreeFrame(t);
  t->local_rows = t->height > 0 ? LocalRows(t->height, BandH(t), t->rank, t->world) : 0;
  size_t n = (size_t)t->width * (size_t)AllocRows(t);
  if (n == 0) return RT2_OK;
  HIP_TRY(hipMalloc(&t->d_accum, n * 3 * sizeof(float)));
  HIP_TRY(hipMalloc(&t->d_pixels, n * 4));
  if (t->ray_counts_on) HIP_TRY(hipMalloc(&t->d_ray_counts, n * sizeof(uint32_t)));
  NoteDeviceBytes(t);
  return RT2_OK;
}

int ResetFrame(rt2_tracer* t) {
  size_t n = (size_t)t->width * (size_t)AllocRows(t);
  t->frame_idx = 0;
  t->queued = 0;  // queued frames would only be accumulated and zeroed again
  t->image_frame = -1;
  if (n == 0) return RT2_OK;
  HIP_TRY(hipSetDevice(t->device));
  HIP_TRY(hipMemsetAsync(t->d_accum, 0, n * 3 * sizeof(float), t->stream));
  HIP_TRY(hipMemsetAsync(t->d_pixels, 0, n * 4, t->stream));
  if (t->d_ray_counts) HIP_TRY(hipMemsetAsync(t->d_ray_counts, 0, n * sizeof(uint32_t), t->stream));
  return RT2_OK;
}

hipEvent_t TakeEvent(rt2_tracer* t) {
  if (!t->event_pool.empty()) {
    hipEvent_t e = t->event_pool.back();
    t->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int DrainEvents(rt2_tracer* t) {
  if (!t->pending.empty() || !t->gpending.empty() || !t->rpending.empty()) t->host_waits++;
  if (!t->pending.empty()) {
    // every render launch is followed by its accumulate on the tracer stream, so a copy queued there
    // reads the clocks of all of them
    HIP_TRY(hipSetDevice(t->device));
    HIP_TRY(hipMemcpyAsync(t->h_clock, t->d_clock, 2 * sizeof(unsigned long long) * kClockRing,
                           hipMemcpyDeviceToHost, t->stream));
    HIP_TRY(hipStreamSynchronize(t->stream));
    std::vector<std::pair<unsigned long long, unsigned long long>> iv;
    for (uint32_t k : t->pending) {
      const unsigned long long s = ~t->h_clock[2 * k], e = t->h_clock[2 * k + 1];
      if (t->h_clock[2 * k] != 0ull && e >= s) iv.emplace_back(s, e);
    }
    std::sort(iv.begin(), iv.end());
    const double ms_per_tick = 1.0 / t->clock_khz;
    for (const auto& x : iv) {
      t->launch_ms_sum += (double)(x.second - x.first) * ms_per_tick;
      const unsigned long long from = std::max(x.first, t->busy_end);
      if (x.second > from) t->kernel_ms += (double)(x.second - from) * ms_per_tick;
      t->busy_end = std::max(t->busy_end, x.second);
    }
  }
  t->pending.clear();
  for (auto& pr : t->gpending) {
    HIP_TRY(hipEventSynchronize(pr.second));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    t->gather_ms += ms;
    t->event_pool.push_back(pr.first);
    t->event_pool.push_back(pr.second);
  }
  t->gpending.clear();
  for (auto& pr : t->rpending) {
    HIP_TRY(hipEventSynchronize(pr.second));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
    t->readback_ms += ms;
    t->event_pool.push_back(pr.first);
    t->event_pool.push_back(pr.second);
  }
  t->rpending.clear();
  return RT2_OK;
}

int Flush(rt2_tracer* t);  // launches the queued frames (rt2_tracer_render)

// Flush before a setting that changes how the queued frames render.
template <typename T>
int FlushIfChanged(rt2_tracer* t, const T& cur, const T& next) {
  return cur == next ? RT2_OK : Flush(t);
}

int Sync(rt2_tracer* t) {
  int rc = Flush(t);
  if (rc != RT2_OK) return rc;
  HIP_TRY(hipSetDevice(t->device));
  t->host_waits++;
  HIP_TRY(hipStreamSynchronize(t->stream));
  return DrainEvents(t);
}

template <typename T>
int Upload(T** dst, const void* src, size_t bytes) {
  HIP_TRY(hipMalloc((void**)dst, bytes));
  HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return RT2_OK;
}

void Put3(float* d, vec3 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}

}  // namespace

extern "C" {

const char* rt2_last_error(void) { return g_err.c_str(); }
#ifndef RT2_KERNEL_SHA
#define RT2_KERNEL_SHA "unknown"
#endif
// "rt2-mi355x 0.1 (gfx950) kernel <sha1 of render.hip + rt2_layout.h, 12 hex digits>"
const char* rt2_version(void) { return "rt2-mi355x 0.1 (gfx950) kernel " RT2_KERNEL_SHA; }

int rt2_scene_load(const char* path, uint64_t seed, rt2_scene** out) {
  if (!path || !out) return Fail(RT2_ERR_INVALID, "rt2_scene_load: null argument");
  *out = nullptr;
  auto s = std::make_unique<rt2_scene>();
  std::string err;
  if (!LoadScene(path, seed, s->scene, err)) {
    bool io = err.rfind("Failed to open", 0) == 0;
    return Fail(io ? RT2_ERR_IO : RT2_ERR_SCENE, err);
  }
  const char* na = getenv("RT2_NO_LIST_ACCEL");
  const bool accel = !(na && na[0] == '1');
  if (!CompileScene(s->scene, s->compiled, err, accel)) return Fail(RT2_ERR_SCENE, err);
  *out = s.release();
  return RT2_OK;
}

void rt2_scene_free(rt2_scene* s) { delete s; }

int rt2_scene_get_info(const rt2_scene* s, rt2_scene_info* o) {
  if (!s || !o) return Fail(RT2_ERR_INVALID, "rt2_scene_get_info: null argument");
  const Scene& sc = s->scene;
  const CompiledScene& c = s->compiled;
  o->dims_x = sc.dims_x;
  o->dims_y = sc.dims_y;
  o->n_materials = (int)sc.materials.size();
  o->n_textures = (int)sc.textures.size();
  o->n_primitives = (int)sc.primitives.size();
  o->n_top_nodes = (int)sc.top.size();
  Put3(o->background, sc.background);
  o->legacy_schema = sc.legacy_schema ? 1 : 0;
  o->bvh_nodes = c.bvh_nodes;
  o->quads = c.quads;
  o->spheres = c.spheres;
  o->lists = c.lists;
  o->xforms = c.xforms;
  o->media = c.media;
  o->max_stack = c.max_stack;
  o->bvh_depth = c.bvh_depth;
  o->node_bytes = (uint64_t)c.nodes.size() * sizeof(float);
  o->acc_lists = c.acc_lists;
  o->acc_nodes = c.acc_nodes;
  o->linear_steps = (int)(c.lin.size() / 4);
  o->origins_bounded = c.origins_bounded ? 1 : 0;
  o->box_steps = c.box_steps;
  return RT2_OK;
}

int rt2_scene_materials(const rt2_scene* s, float* out, int cap) {
  if (!s) return Fail(RT2_ERR_INVALID, "null scene");
  int n = (int)s->scene.materials.size();
  for (int i = 0; i < n && i < cap && out; i++) {
    const MaterialDesc& m = s->scene.materials[(size_t)i];
    float* r = out + 8 * i;
    r[0] = (float)m.type;
    r[1] = m.albedo.x;
    r[2] = m.albedo.y;
    r[3] = m.albedo.z;
    r[4] = m.fuzz;
    r[5] = m.refraction_index;
    r[6] = (float)m.tex_idx;
    r[7] = 0;
  }
  return n;
}

int rt2_scene_textures(const rt2_scene* s, float* out, int cap) {
  if (!s) return Fail(RT2_ERR_INVALID, "null scene");
  int n = (int)s->scene.textures.size();
  for (int i = 0; i < n && i < cap && out; i++) {
    const TextureDesc& t = s->scene.textures[(size_t)i];
    float* r = out + 8 * i;
    r[0] = (float)t.type;
    r[1] = t.albedo.x;
    r[2] = t.albedo.y;
    r[3] = t.albedo.z;
    r[4] = t.type == kTexChecker ? t.inv_scale : t.scale;
    r[5] = (float)t.even;
    r[6] = (float)t.odd;
    r[7] = (float)t.noise_type;
  }
  return n;
}

int rt2_scene_perlin(const rt2_scene* s, int tex, float* vec, int* perm) {
  if (!s || tex < 0 || tex >= (int)s->scene.textures.size()) return Fail(RT2_ERR_INVALID, "bad texture index");
  const TextureDesc& t = s->scene.textures[(size_t)tex];
  if (t.type != kTexNoise) return Fail(RT2_ERR_INVALID, "not a noise texture");
  int pc = t.point_count;
  for (int i = 0; i < pc; i++) {
    if (vec) Put3(vec + 3 * i, t.perlin_vec[(size_t)i]);
    if (perm) {
      perm[i] = t.perm_x[(size_t)i];
      perm[pc + i] = t.perm_y[(size_t)i];
      perm[2 * pc + i] = t.perm_z[(size_t)i];
    }
  }
  return pc;
}

int rt2_scene_get_camera(const rt2_scene* s, rt2_camera_desc* o) {
  if (!s || !o) return Fail(RT2_ERR_INVALID, "null argument");
  const Camera& c = s->scene.cam;
  Put3(o->center, c.center_);
  Put3(o->look_at, c.lookat_);
  Put3(o->view_up, c.view_up_);
  o->vfov = c.vfov_;
  o->defocus_angle = c.defocus_angle_;
  o->focus_distance = c.focus_dist_;
  return RT2_OK;
}

int rt2_scene_set_camera(rt2_scene* s, const rt2_camera_desc* c) {
  if (!s || !c) return Fail(RT2_ERR_INVALID, "null argument");
  Camera& cam = s->scene.cam;
  cam.SetCenter(vec3{c->center[0], c->center[1], c->center[2]});
  cam.SetLookAt(vec3{c->look_at[0], c->look_at[1], c->look_at[2]});
  cam.SetViewUp(vec3{c->view_up[0], c->view_up[1], c->view_up[2]});
  cam.SetFOV(c->vfov);
  cam.SetDefocusAngle(c->defocus_angle);
  cam.SetFocusDistance(c->focus_distance);
  return RT2_OK;
}

int rt2_camera_params(const rt2_scene* s, int w, int h, int spp, float* out) {
  if (!s || !out || w <= 0 || h <= 0 || spp <= 0) return Fail(RT2_ERR_INVALID, "bad camera query");
  Camera c = s->scene.cam;
  c.SetDims(w, h);
  c.SetSamplesPerPixel(spp);
  CameraParams p = c.Params();
  memcpy(out, p.pixel00, 3 * sizeof(float));
  memcpy(out + 3, p.du, 3 * sizeof(float));
  memcpy(out + 6, p.dv, 3 * sizeof(float));
  memcpy(out + 9, p.center, 3 * sizeof(float));
  memcpy(out + 12, p.defocus_u, 3 * sizeof(float));
  memcpy(out + 15, p.defocus_v, 3 * sizeof(float));
  out[18] = p.defocus_angle;
  out[19] = p.recip_sqrt_spp;
  out[20] = (float)p.sqrt_spp;
  return RT2_OK;
}

int rt2_camera_load(const char* path, rt2_camera_desc* o) {
  if (!path || !o) return Fail(RT2_ERR_INVALID, "null argument");
  Camera c;
  std::string err;
  if (!LoadCameraFile(path, c, err)) return Fail(RT2_ERR_IO, err);
  Put3(o->center, c.center_);
  Put3(o->look_at, c.lookat_);
  Put3(o->view_up, c.view_up_);
  o->vfov = c.vfov_;
  o->defocus_angle = c.defocus_angle_;
  o->focus_distance = c.focus_dist_;
  return RT2_OK;
}

int rt2_camera_write(const rt2_camera_desc* d, const char* path) {
  if (!d || !path) return Fail(RT2_ERR_INVALID, "null argument");
  Camera c;
  c.SetCenter(vec3{d->center[0], d->center[1], d->center[2]});
  c.SetLookAt(vec3{d->look_at[0], d->look_at[1], d->look_at[2]});
  c.SetViewUp(vec3{d->view_up[0], d->view_up[1], d->view_up[2]});
  c.SetFOV(d->vfov);
  c.SetDefocusAngle(d->defocus_angle);
  c.SetFocusDistance(d->focus_distance);
  std::string err;
  if (!WriteCameraFile(c, path, err)) return Fail(RT2_ERR_IO, err);
  return RT2_OK;
}

int rt2_settings_load(const char* path, rt2_app_settings* o) {
  if (!path || !o) return Fail(RT2_ERR_INVALID, "null argument");
  AppSettings a;
  std::string err;
  if (!LoadAppSettingsFile(path, a, err)) return Fail(RT2_ERR_IO, err);
  o->render_once = a.render_once;
  o->save_after_render_once = a.save_after_render_once;
  o->num_samples = a.num_samples;
  o->max_depth = a.max_depth;
  o->render_window = a.render_window;
  return RT2_OK;
}

int rt2_tracer_create(const rt2_scene* s, int device, rt2_tracer** out) {
  if (!s || !out) return Fail(RT2_ERR_INVALID, "rt2_tracer_create: null argument");
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return Fail(RT2_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return Fail(RT2_ERR_INVALID, "device index out of range");
  auto t = std::make_unique<rt2_tracer>();
  t->device = device;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&t->own_stream, hipStreamNonBlocking));
  t->stream = t->own_stream;
  for (auto& sl : t->slots) {
    HIP_TRY(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&sl.rendered, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&sl.consumed, hipEventDisableTiming));
  }
  if (const char* e = getenv("RT2_PIPELINE")) t->pipeline = e[0] != '0';
  const CompiledScene& c = s->compiled;
  int rc;
  if ((rc = Upload(&t->d_nodes, c.nodes.data(), c.nodes.size() * sizeof(float))) != RT2_OK) return rc;
  std::vector<float> mats = c.materials;
  if (mats.empty()) mats.assign(8, 0.0f);
  if ((rc = Upload(&t->d_materials, mats.data(), mats.size() * sizeof(float))) != RT2_OK) return rc;
  if ((rc = Upload(&t->d_textures, c.textures.data(), c.textures.size() * sizeof(float))) != RT2_OK) return rc;
  if ((rc = Upload(&t->d_perlin_vec, c.perlin_vec.data(), c.perlin_vec.size() * sizeof(float))) != RT2_OK) return rc;
  if ((rc = Upload(&t->d_perlin_perm, c.perlin_perm.data(), c.perlin_perm.size() * sizeof(int))) != RT2_OK) return rc;
  if (!c.lin.empty()) {
    if ((rc = Upload(&t->d_lin, c.lin.data(), c.lin.size() * sizeof(uint32_t))) != RT2_OK) return rc;
    if ((rc = Upload(&t->d_lin_wide, c.lin_wide.data(), c.lin_wide.size() * sizeof(uint32_t))) != RT2_OK) return rc;
    if ((rc = Upload(&t->d_lind, c.lind.data(), c.lind.size() * sizeof(float))) != RT2_OK) return rc;
    t->lin_len = (uint32_t)(c.lin.size() / 4);
  }
  HIP_TRY(hipMalloc(&t->d_work, 128));
  HIP_TRY(hipMalloc(&t->d_clock, 2 * sizeof(unsigned long long) * kClockRing));
  HIP_TRY(hipMemset(t->d_clock, 0, 2 * sizeof(unsigned long long) * kClockRing));
  HIP_TRY(hipHostMalloc((void**)&t->h_clock, 2 * sizeof(unsigned long long) * kClockRing, hipHostMallocDefault));
  {
    int khz = 0;  // the constant clock s_memrealtime counts (100 MHz on MI355X)
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
      t->clock_khz = (double)khz;
  }
  HIP_TRY(hipMalloc(&t->d_stats, kStatsSlots * sizeof(unsigned long long)));
  HIP_TRY(hipMemset(t->d_stats, 0, kStatsSlots * sizeof(unsigned long long)));
  t->scene_bytes = c.nodes.size() * sizeof(float) + std::max<size_t>(mats.size(), 8) * sizeof(float) +
                   c.textures.size() * sizeof(float) + c.perlin_vec.size() * sizeof(float) +
                   c.perlin_perm.size() * sizeof(int) + c.lin.size() * sizeof(uint32_t) +
                   c.lin_wide.size() * sizeof(uint32_t) + c.lind.size() * sizeof(float) + 128 +
                   2 * sizeof(unsigned long long) * kClockRing + kStatsSlots * sizeof(unsigned long long);
  t->root = c.root;
  t->node_records = (uint32_t)(c.nodes.size() / 4);
  t->hot_records = c.hot_records;
  t->features = c.features;
  t->max_stack = c.max_stack;
  t->stack_ok = c.stack_ok;
  t->flat_xforms = c.lin_xform_depth <= 1;
  t->origins_bounded = c.origins_bounded;
  Put3(t->background, s->scene.background);
  t->camera = s->scene.cam;
  HIP_TRY(hipDeviceGetAttribute(&t->cus, hipDeviceAttributeMultiprocessorCount, device));
  HIP_TRY(hipDeviceGetAttribute(&t->lds_per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device));
  if (const char* e = getenv("RT2_NO_LDS")) t->use_lds = e[0] == '0';
  if (const char* e = getenv("RT2_NO_LINEAR")) t->use_linear = e[0] == '0';
  if (const char* e = getenv("RT2_NO_HYBRID")) t->use_hybrid = e[0] == '0';
  if (const char* e = getenv("RT2_FORCE_HYBRID")) t->force_hybrid = e[0] == '1';
  if (const char* e = getenv("RT2_HYBRID_RECORDS")) t->hybrid_cap = atoi(e);
  if (const char* e = getenv("RT2_CHUNK_MAX")) t->chunk_max = std::max(1, atoi(e));
  if (const char* e = getenv("RT2_CHUNK_ALIGN")) t->chunk_align = e[0] != '0';
  if (const char* e = getenv("RT2_FRAME_TILES")) t->frame_tiles_env = e[0] == '1' ? 1 : 0;
  if (const char* e = getenv("RT2_FRAME_TILE_LEN")) t->frame_tile_len = std::max(1, std::min(atoi(e), 64));
  // App.cpp:122-125,157: scene dims when present, else the window default 1600x900
  int w = s->scene.dims_x > 0 && s->scene.dims_y > 0 ? s->scene.dims_x : 1600;
  int h = s->scene.dims_x > 0 && s->scene.dims_y > 0 ? s->scene.dims_y : 900;
  rt2_tracer* raw = t.release();
  rc = rt2_tracer_on_resize(raw, w, h);
  if (rc != RT2_OK) {
    rt2_tracer_destroy(raw);
    return rc;
  }
  *out = raw;
  return RT2_OK;
}

void rt2_tracer_destroy(rt2_tracer* t) {
  if (!t) return;
  if (!t->parts.empty()) {
    for (rt2_tracer* p : t->parts) rt2_tracer_destroy(p);
    delete t;
    return;
  }
  (void)hipSetDevice(t->device);
  if (t->stream) (void)hipStreamSynchronize(t->stream);
  if (t->comm) (void)ncclCommDestroy(t->comm);
  for (auto& pr : t->gpending) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  for (auto& pr : t->rpending) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (t->stream) (void)hipStreamSynchronize(t->stream);
  for (hipEvent_t e : t->event_pool) (void)hipEventDestroy(e);
  (void)hipFree(t->d_clock);
  if (t->h_clock) (void)hipHostFree(t->h_clock);
  FreeFrame(t);
  (void)hipFree(t->d_nodes);
  (void)hipFree(t->d_materials);
  (void)hipFree(t->d_textures);
  (void)hipFree(t->d_perlin_vec);
  (void)hipFree(t->d_perlin_perm);
  (void)hipFree(t->d_lin);
  (void)hipFree(t->d_lin_wide);
  (void)hipFree(t->d_lind);
  (void)hipFree(t->d_work);
  (void)hipFree(t->d_stats);
  for (auto& sl : t->slots) {
    if (sl.chunks) (void)hipFreeAsync(sl.chunks, sl.stream);
    if (sl.stream) (void)hipStreamSynchronize(sl.stream);
  }
  if (t->stream) (void)hipStreamSynchronize(t->stream);
  for (auto& st : t->staging) {
    (void)hipEventDestroy(st.done);
    (void)hipHostFree(st.p);
  }
  if (t->own_stream) (void)hipStreamDestroy(t->own_stream);
  for (auto& sl : t->slots) {
    if (sl.rendered) (void)hipEventDestroy(sl.rendered);
    if (sl.consumed) (void)hipEventDestroy(sl.consumed);
    if (sl.stream) (void)hipStreamDestroy(sl.stream);
  }
  delete t;
}

}  // extern "C"

namespace {
bool IsMulti(const rt2_tracer* t) { return !t->parts.empty(); }

// Applies f to every part of a multi tracer (stops at the first error).
template <typename Fn>
int ForParts(rt2_tracer* t, Fn&& f) {
  for (rt2_tracer* p : t->parts) {
    int rc = f(p);
    if (rc != RT2_OK) return rc;
  }
  return RT2_OK;
}

// Forwards a setter to every part of a multi tracer.
#define RT2_FORWARD(t, call)                                           \
  do {                                                                 \
    if (IsMulti(t)) return ForParts(t, [&](rt2_tracer* p) { return call; }); \
  } while (0)
}  // namespace

extern "C" {

int rt2_tracer_set_stream(rt2_tracer* t, void* s) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  if (IsMulti(t)) {
    if (t->parts.size() != 1) return Fail(RT2_ERR_INVALID, "set_stream: a multi-GPU tracer owns one stream per GPU");
    return rt2_tracer_set_stream(t->parts[0], s);
  }
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  t->stream = s ? (hipStream_t)s : t->own_stream;
  return RT2_OK;
}

int rt2_tracer_set_max_depth(rt2_tracer* t, int d) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_set_max_depth(p, d));
  // RayTracer::max_depth is a size_t (RayTracer.hpp:32); the kernel keeps it in 16 bits
  if (d > 0xFFFF) return Fail(RT2_ERR_INVALID, "max_depth must be at most 65535");
  int rc = FlushIfChanged(t, t->max_depth, d < 0 ? 0 : d);
  if (rc != RT2_OK) return rc;
  t->max_depth = d < 0 ? 0 : d;
  return RT2_OK;
}

int rt2_tracer_set_samples_per_pixel(rt2_tracer* t, int spp) {
  if (!t || spp <= 0) return Fail(RT2_ERR_INVALID, "samples_per_pixel must be positive");
  RT2_FORWARD(t, rt2_tracer_set_samples_per_pixel(p, spp));
  int rc = FlushIfChanged(t, t->camera.SamplesPerPixel(), spp);
  if (rc != RT2_OK) return rc;
  t->camera.SetSamplesPerPixel(spp);
  return RT2_OK;
}

int rt2_tracer_set_seed(rt2_tracer* t, uint64_t seed) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_set_seed(p, seed));
  int rc = FlushIfChanged(t, t->seed, seed);
  if (rc != RT2_OK) return rc;
  t->seed = seed;
  return RT2_OK;
}

int rt2_tracer_set_partition(rt2_tracer* t, int band_h, int rank, int world) {
  if (!t || band_h < 0 || world < 1 || rank < 0 || rank >= world)
    return Fail(RT2_ERR_INVALID, "bad partition (need band_h >= 0, 0 <= rank < world)");
  if (IsMulti(t)) return Fail(RT2_ERR_INVALID, "set_partition: a multi-GPU tracer partitions itself");
  if (t->comm && (rank != t->rank || world != t->world || band_h != t->band_h))
    return Fail(RT2_ERR_INVALID, "set_partition: the tracer is joined to a communicator with another partition");
  t->queued = 0;  // the partition change resets the frame
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  t->band_h = band_h;
  t->rank = rank;
  t->world = world;
  if ((rc = Realloc(t)) != RT2_OK) return rc;
  return ResetFrame(t);
}

int rt2_tracer_set_launch_frames(rt2_tracer* t, int n) {
  if (!t || n < 0) return Fail(RT2_ERR_INVALID, "frames_per_launch must be >= 0");
  RT2_FORWARD(t, rt2_tracer_set_launch_frames(p, n));
  t->launch_frames = n;
  return RT2_OK;
}

int rt2_tracer_set_work_split(rt2_tracer* t, int items_per_lane) {
  if (!t || items_per_lane < 0) return Fail(RT2_ERR_INVALID, "items_per_lane must be >= 0");
  RT2_FORWARD(t, rt2_tracer_set_work_split(p, items_per_lane));
  t->work_split = items_per_lane;
  return RT2_OK;
}

int rt2_tracer_set_batch_max(rt2_tracer* t, int items) {
  if (!t || items < 1) return Fail(RT2_ERR_INVALID, "batch must be >= 1");
  RT2_FORWARD(t, rt2_tracer_set_batch_max(p, items));
  t->batch_max = items;
  return RT2_OK;
}

int rt2_tracer_set_sample_budget(rt2_tracer* t, uint64_t bytes) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_set_sample_budget(p, bytes));
  t->sample_budget = (size_t)bytes;
  return RT2_OK;
}

int rt2_tracer_last_launch(const rt2_tracer* t, int* grid, int* chunk_frames, int* variant) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  if (IsMulti(t)) return rt2_tracer_last_launch(t->parts[0], grid, chunk_frames, variant);
  if (grid) *grid = t->last_grid;
  if (chunk_frames) *chunk_frames = t->last_chunk_frames;
  if (variant) *variant = t->last_variant;
  return RT2_OK;
}

int rt2_tracer_on_resize(rt2_tracer* t, int w, int h) {
  if (!t || w <= 0 || h <= 0) return Fail(RT2_ERR_INVALID, "dims must be positive");
  if (w > 65535 || h > 65535) return Fail(RT2_ERR_INVALID, "dims must be at most 65535");
  // the kernel's pixel index (Philox pixel word, magic division by the width) stays below 2^31
  if ((int64_t)w * h >= (int64_t)1 << 31) return Fail(RT2_ERR_INVALID, "width * height must be below 2^31");
  if (IsMulti(t)) {
    t->width = w;
    t->height = h;
    return ForParts(t, [&](rt2_tracer* p) { return rt2_tracer_on_resize(p, w, h); });
  }
  t->queued = 0;  // OnResize resets the frame
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  t->width = w;
  t->height = h;
  t->camera.SetDims(w, h);
  if ((rc = Realloc(t)) != RT2_OK) return rc;
  return ResetFrame(t);
}

int rt2_tracer_reset(rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_reset(p));
  return ResetFrame(t);
}

int rt2_tracer_set_camera(rt2_tracer* t, const rt2_camera_desc* c) {
  if (!t || !c) return Fail(RT2_ERR_INVALID, "null argument");
  RT2_FORWARD(t, rt2_tracer_set_camera(p, c));
  const Camera& cur = t->camera;
  const vec3 center{c->center[0], c->center[1], c->center[2]};
  const vec3 look{c->look_at[0], c->look_at[1], c->look_at[2]};
  const vec3 up{c->view_up[0], c->view_up[1], c->view_up[2]};
  auto same3 = [](vec3 a, vec3 b) { return memcmp(&a, &b, sizeof(vec3)) == 0; };
  const bool same = same3(cur.center_, center) && same3(cur.lookat_, look) && same3(cur.view_up_, up) &&
                    memcmp(&cur.vfov_, &c->vfov, 4) == 0 && memcmp(&cur.defocus_angle_, &c->defocus_angle, 4) == 0 &&
                    memcmp(&cur.focus_dist_, &c->focus_distance, 4) == 0;
  if (same) return RT2_OK;  // the reference's lazy camera: nothing dirty, nothing to recompute
  int rc = Flush(t);        // queued frames render with the camera they were queued under
  if (rc != RT2_OK) return rc;
  t->camera.SetCenter(center);
  t->camera.SetLookAt(look);
  t->camera.SetViewUp(up);
  t->camera.SetFOV(c->vfov);
  t->camera.SetDefocusAngle(c->defocus_angle);
  t->camera.SetFocusDistance(c->focus_distance);
  return RT2_OK;
}

int rt2_tracer_get_camera(const rt2_tracer* t, rt2_camera_desc* o) {
  if (!t || !o) return Fail(RT2_ERR_INVALID, "null argument");
  if (IsMulti(t)) return rt2_tracer_get_camera(t->parts[0], o);
  const Camera& c = t->camera;
  Put3(o->center, c.center_);
  Put3(o->look_at, c.lookat_);
  Put3(o->view_up, c.view_up_);
  o->vfov = c.vfov_;
  o->defocus_angle = c.defocus_angle_;
  o->focus_distance = c.focus_dist_;
  return RT2_OK;
}

}  // extern "C"

namespace {
constexpr uint32_t kFrameTileMinSteps = 256;  // threaded programs longer than this use frame tiles

// Camera rays start within +-2^64 on every axis (center + the defocus disk's two half-axes): the
// kernel's rectangle test (compile.cpp RectAAWords) is exact for ray origins within +-2^100, and a
// scene the compiler gives that test lies within +-2^64 (Flattener::QuadAASpace). Checked only for
// scenes whose threaded program holds such a test (CompiledScene::origins_bounded).
bool CameraOriginsBounded(const CameraParams& c) {
  for (int k = 0; k < 3; k++)
    if (!(std::fabs((double)c.center[k]) + std::fabs((double)c.defocus_u[k]) + std::fabs((double)c.defocus_v[k]) <=
          0x1p64))
      return false;
  return true;
}
constexpr const char* kCameraRangeMsg = "camera origin or defocus disk outside +-2^64";

Magic MakeMagic(uint32_t d) {  // rt2_layout.h Magic: floor(n / d) for n < 2^31
  uint32_t l = 0;
  while ((1ull << l) < (uint64_t)d) l++;
  const uint64_t m = ((1ull << (31 + l)) + d - 1) / d;
  return Magic{(uint32_t)m, 31 + l};
}

// Frame chunks of one launch: frames [fb, fb + n) cut into chunks, every pixel's chunk c one work
// item (chunk-major). A chunk starting with R frames left holds about R * T / (k * L) frames (T =
// items per chunk, L = resident lanes, k = work_split), at least 1 and at most chunk_max: early
// items are long (few item setups per sample) and the last ones short, so the launch's tail — the
// time in which lanes run out of work while others finish their item — stays short. k = 0: one
// chunk (each pixel's frames in one item). Appends the table (first frame, stratum) per chunk and
// the sentinel to `tab`; returns the number of chunks and the first chunk's length.
void ChunkSchedule(const rt2_tracer* t, int fb, int n, uint32_t tile_items, int64_t lanes, int sq,
                   std::vector<uint32_t>& tab, uint32_t* n_chunks, int* first_len) {
  const size_t start = tab.size();
  // items must stay below 2^31 (kernel index arithmetic): shortest chunk that allows it
  const int64_t max_chunks = std::max<int64_t>(1, (int64_t)0x7FFFFFFF / tile_items);
  const int lo = (int)std::max<int64_t>(1, ((int64_t)n + max_chunks - 1) / max_chunks);
  int first = 0;
  // frame tiles: chunks of up to frame_tile_len frames, as even as the 64-chunk groups allow (the
  // last group is padded with empty chunks, whose lanes fetch again)
  int ft_len = 1;
  if (t->frame_tiles) {
    const int groups = (n + 64 * t->frame_tile_len - 1) / (64 * t->frame_tile_len);
    ft_len = (n + 64 * groups - 1) / (64 * groups);
  }
  for (int s = 0; s < n;) {
    int len = n - s;
    if (t->frame_tiles) {
      len = ft_len;  // frame tiles: short chunks of one pixel (RenderParams::frame_tiles)
    } else if (t->work_split > 0) {
      const double want = (double)(n - s) * (double)tile_items / ((double)t->work_split * (double)lanes);
      len = (int)std::min<double>(want, (double)t->chunk_max);
    }
    // long chunks start on a 4-frame group of the sample octets (the 8-wave kernels stage samples
    // by 4 frames; whole octets would cut a 15-frame chunk to 8)
    if (t->chunk_align && len >= (int)kOctet) len -= len % 4;
    if (!t->frame_tiles) len = std::max(len, lo);
    len = std::min({len, n - s, kChunkMaxFrames});
    const uint32_t f = (uint32_t)(fb + s), usq = (uint32_t)sq;
    tab.push_back(f);
    tab.push_back((f % usq) | (((f / usq) % usq) << 16));  // RayTracer.cpp:59-60
    if (s == 0) first = len;
    s += len;
  }
  if (t->frame_tiles) {  // padding chunks up to a multiple of 64 (empty: first frame = the launch end)
    while (((tab.size() - start) / 2) % 64 != 0) {
      tab.push_back((uint32_t)(fb + n));
      tab.push_back(0u);
    }
  }
  tab.push_back((uint32_t)(fb + n));
  tab.push_back(0u);
  *n_chunks = (uint32_t)((tab.size() - start) / 2 - 1);
  *first_len = first;
}

// Puts a launch's chunk table in its slot's table, ordered on the slot's render stream: the copy runs
// after the launches already queued there (which may still read the old table), from pinned staging
// memory, so the host never waits for the GPU (a multi-GPU tracer enqueues every GPU's launches at
// once). A launch repeating the slot's last schedule (the bench, a progressive loop's steady state)
// uploads nothing.
int UploadChunks(rt2_tracer* t, rt2_tracer::Slot& sl, const std::vector<uint32_t>& tab) {
  if (sl.chunks && tab == sl.chunks_host) return RT2_OK;
  const size_t bytes = tab.size() * sizeof(uint32_t);
  if (bytes > sl.chunks_bytes) {
    // grow geometrically; stream-ordered free and allocation: the queued launches that read the old
    // table run first, and the host does not wait (hipFree would synchronize the device)
    const size_t cap = std::max(bytes, 2 * sl.chunks_bytes);
    if (sl.chunks) HIP_TRY(hipFreeAsync(sl.chunks, sl.stream));
    sl.chunks = nullptr;
    sl.chunks_bytes = 0;
    sl.chunks_host.clear();
    HIP_TRY(hipMallocAsync((void**)&sl.chunks, cap, sl.stream));
    sl.chunks_bytes = cap;
  }
  // a staging buffer whose previous copy has run, else a new one
  rt2_tracer::Staging* st = nullptr;
  for (auto& c : t->staging) {
    if (c.bytes < bytes) continue;
    const hipError_t q = hipEventQuery(c.done);
    if (q == hipSuccess) {
      st = &c;
      break;
    }
    if (q != hipErrorNotReady) return HipFail(q, "hipEventQuery");
  }
  if (!st) {
    rt2_tracer::Staging c{nullptr, std::max<size_t>(bytes, 4096), nullptr};
    HIP_TRY(hipHostMalloc((void**)&c.p, c.bytes, hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&c.done, hipEventDisableTiming));
    t->staging.push_back(c);
    st = &t->staging.back();
  }
  memcpy(st->p, tab.data(), bytes);
  HIP_TRY(hipMemcpyAsync(sl.chunks, st->p, bytes, hipMemcpyHostToDevice, sl.stream));
  HIP_TRY(hipEventRecord(st->done, sl.stream));
  sl.chunks_host = tab;
  return RT2_OK;
}

// Launches frames [frame_idx, frame_idx + n_frames) now.
int LaunchFrames(rt2_tracer* t, int n_frames) {
  if (n_frames == 0 || t->local_rows == 0) {
    t->frame_idx += n_frames;
    return RT2_OK;
  }
  HIP_TRY(hipSetDevice(t->device));
  RenderParams p;
  memset(&p, 0, sizeof(p));
  p.nodes = t->d_nodes;
  p.materials = t->d_materials;
  p.textures = t->d_textures;
  p.perlin_vec = t->d_perlin_vec;
  p.perlin_perm = t->d_perlin_perm;
  p.root = t->root;
  memcpy(p.background, t->background, sizeof(p.background));
  p.cam = t->camera.Params();  // RayTracer::Update → camera->Update() (RayTracer.cpp:56)
  if (p.cam.sqrt_spp <= 0) return Fail(RT2_ERR_INVALID, "samples_per_pixel gives sqrt_spp = 0");
  if (t->origins_bounded && !CameraOriginsBounded(p.cam)) return Fail(RT2_ERR_INVALID, kCameraRangeMsg);
  p.width = t->width;
  p.height = t->height;
  p.local_rows = t->local_rows;
  p.band_h = t->band_h > 0 ? t->band_h : t->height;
  p.rank = t->rank;
  p.world = t->world;
  // work tiles of 64 pixels: 8x8, or as tall as a row band narrower than 8 rows (16x4, 32x2, 64x1)
  // so that a wave's pixels stay in one band (neighbouring pixels, coherent primary rays)
  const int tile_rows = t->world > 1 && p.band_h < 8 ? (p.band_h >= 4 ? 4 : p.band_h >= 2 ? 2 : 1) : 8;
  p.tile_shift = tile_rows == 8 ? 3u : tile_rows == 4 ? 4u : tile_rows == 2 ? 5u : 6u;
  p.tiles_x = (t->width + (1 << p.tile_shift) - 1) >> p.tile_shift;
  p.tile_items = (uint32_t)p.tiles_x * (uint32_t)((t->local_rows + tile_rows - 1) / tile_rows) * 64u;
  p.div_tile_items = MakeMagic(p.tile_items);
  p.div_tiles_x = MakeMagic((uint32_t)p.tiles_x);
  p.div_band_h = MakeMagic((uint32_t)p.band_h);
  p.div_band_w = MakeMagic((uint32_t)p.band_h * (uint32_t)p.world);
  p.div_world = MakeMagic((uint32_t)p.world);
  p.local_pixels = (uint32_t)t->width * (uint32_t)t->local_rows;
  if (p.tile_items > 0x7FFFFFFFu)  // work items (and pixel indices) must stay below 2^31
    return Fail(RT2_ERR_INVALID, "image too large for one GPU (more than 2^31 pixels in a partition)");
  p.max_depth = t->max_depth;
  p.seed_lo = (uint32_t)t->seed;
  p.seed_hi = (uint32_t)(t->seed >> 32);
  for (uint32_t r = 0; r < 10; r++) {
    p.philox_keys[2 * r] = p.seed_lo + r * 0x9E3779B9u;
    p.philox_keys[2 * r + 1] = p.seed_hi + r * 0xBB67AE85u;
  }
  p.ray_counts = t->d_ray_counts;
  p.work_counter = t->d_work;
  p.stats = t->d_stats;
  p.stack_depth = t->max_stack;
  p.lin = t->d_lin;
  p.lin_wide = t->d_lin_wide;
  p.lind = t->d_lind;
  p.lin_len = t->use_linear ? t->lin_len : 0u;
  p.flat_xforms = t->flat_xforms ? 1u : 0u;
  if (!p.lin_len && !t->stack_ok)
    return Fail(RT2_ERR_INVALID, "scene needs a traversal stack of " + std::to_string(t->max_stack) +
                                     " entries (kernel has " + std::to_string(kTraversalStack) +
                                     "): only the threaded traversal can render it");
  // Frame tiles (a wave's lanes trace one pixel's consecutive frames: paths from one pixel share
  // their first hit and start their secondary rays from nearly one point, so the lockstep walk of
  // a deep program serves more lanes per step) for deep threaded programs: measured with chunks of
  // up to 8 frames, book 2 (4,922 steps) +4 %, book 1 (995 steps) +4.5 %; Cornell (29 steps) -2 %,
  // where 8x8 pixel tiles are as coherent and the shorter chunks cost more item fetches.
  t->frame_tiles = t->frame_tiles_env >= 0 ? t->frame_tiles_env == 1 : (p.lin_len > kFrameTileMinSteps);
  // frame-tile items are g * 64 * local_pixels + ...: at least one 64-chunk group must stay below 2^31
  if ((uint64_t)p.local_pixels * 64u > 0x7FFFFFFFull) t->frame_tiles = false;
  uint32_t feats = t->features | (p.cam.defocus_angle > 0.0f ? (uint32_t)kFeatDefocus : 0u);
  int variant = RenderVariant(feats);
  // per-record counters and per-pixel ray counts come from the counting kernel instantiation (same
  // arithmetic, extra counters); the product kernel keeps only the wave ray totals
  const bool counting = t->stats_on || t->ray_counts_on;
  // Scene records in LDS: the whole scene when it fits; otherwise (stack traversal) the top levels
  // of the BVH — its node records are a breadth-first prefix of the record array — as many as fit
  // beside the traversal stack without lowering the occupancy the registers allow.
  // LDS room per workgroup that keeps the occupancy the registers allow (beside the stack)
  uint32_t room = 0;  // float4 records
  if (t->use_lds && !p.lin_len) {
    const int hkey = variant * 2 + (counting ? 1 : 0);
    if (t->hyb_key != hkey) {
      const size_t stack_bytes = (size_t)p.stack_depth * (size_t)RenderBlockSize() * 4;
      const int blocks = RenderBlocksPerCU(variant, kModeStackHybrid, counting, stack_bytes);
      const size_t per_block = (size_t)t->lds_per_cu / (size_t)std::max(1, blocks);
      t->hyb_records = (uint32_t)(per_block > stack_bytes ? (per_block - stack_bytes) / 16 : 0);
      t->hyb_key = hkey;
    }
    room = t->hyb_records;
  }
  // whole scene in LDS only when that costs no occupancy (measured on book 1 in stack mode: the
  // 32 KB scene in LDS limited it to 3 workgroups per CU, 3.9 Grays/s; the hybrid prefix 5.0)
  const bool lds = t->use_lds && !t->force_hybrid && !p.lin_len && t->node_records <= room &&
                   (size_t)t->node_records * 16 <= (size_t)kLdsSceneBytesMax;
  // Hybrid prefix: measured +20% on a 10^5-sphere field, but -15% on book 2, whose all-features
  // kernel already spills at its occupancy target; used for variants without media and transforms
  // unless forced (RT2_FORCE_HYBRID).
  const bool hybrid_variant = t->force_hybrid || !(RenderVariantFeatures(variant) & (kFeatMedium | kFeatXform));
  uint32_t hot = 0;
  if (!lds && hybrid_variant && t->use_lds && t->use_hybrid && t->hot_records > 0 && !p.lin_len) {
    hot = std::min<uint32_t>(std::min<uint32_t>(room, (uint32_t)(kLdsHotBytesMax / 16)), t->hot_records) & ~1u;
    if (t->hybrid_cap >= 0) hot = std::min(hot, (uint32_t)t->hybrid_cap & ~1u);
    if (hot < 2) hot = 0;
  }
  p.lds_nodes = lds ? t->node_records : hot;
  p.lds_partial = (!lds && hot) ? 1u : 0u;
  // resident lanes of this kernel instantiation (occupancy query cached: it costs far more than
  // a one-frame launch)
  const size_t lds_bytes = RenderLdsBytes(p);
  const int okey = variant * 16 + RenderMode(p) * 2 + (counting ? 1 : 0);
  if (t->occ_key != okey || t->occ_lds != lds_bytes) {
    t->occ_blocks = RenderBlocksPerCU(variant, RenderMode(p), counting, lds_bytes);
    t->occ_key = okey;
    t->occ_lds = lds_bytes;
  }
  const int64_t resident = (int64_t)t->cus * t->occ_blocks * RenderBlockSize();
  // frames per launch: the caller's launch_frames, bounded by the sample-buffer budget
  const size_t frame_bytes = (size_t)p.local_pixels * 3 * sizeof(float);
  int per_launch = t->launch_frames > 0 ? std::min(t->launch_frames, n_frames) : n_frames;
  // (the buffer holds whole octets of frames, rt2_layout.h kOctet; each of the two slots gets half the
  // budget, so both together stay within it)
  const size_t budget_frames = std::max<size_t>(1, t->sample_budget / 2 / frame_bytes);
  per_launch = (int)std::min<size_t>((size_t)per_launch, budget_frames < kOctet ? budget_frames : budget_frames - budget_frames % kOctet);
  if (t->frame_tiles) {  // items (64-frame groups x 64 x local pixels) stay below 2^31
    const size_t groups = std::max<size_t>(1, (size_t)0x7FFFFFFF / (64u * (size_t)p.local_pixels));
    per_launch = (int)std::min<size_t>((size_t)per_launch, groups * 64u);
  }
  const auto octets = [](size_t frames) { return (frames + kOctet - 1) / kOctet * kOctet; };
  t->last_variant = variant;
  struct Launch {
    int frame_begin, n_frames, first_len;
    uint32_t n_chunks;
    size_t table;  // offset in `tabs` (words)
  };
  std::vector<Launch> launches;
  std::vector<uint32_t> tabs;
  for (int done = 0, fb = (int)t->frame_idx; done < n_frames;) {
    Launch L{fb, std::min(per_launch, n_frames - done), 0, 0, tabs.size()};
    // Split each pixel's frames into chunks so that the launch has about work_split items per
    // resident lane: a persistent lane's last item is then short, and a small partition (a row
    // band of an 8-GPU split) still fills every CU. Samples land in the per-frame buffer, so the
    // accumulation order does not depend on the split.
    ChunkSchedule(t, L.frame_begin, L.n_frames, p.tile_items, resident, p.cam.sqrt_spp, tabs, &L.n_chunks,
                  &L.first_len);
    launches.push_back(L);
    done += L.n_frames;
    fb += L.n_frames;
  }
  // The counting kernels add per-pixel ray counts that Reset() zeroes on the tracer stream: those
  // launches wait for it, as every launch does with RT2_PIPELINE=0.
  const bool serial = !t->pipeline || counting;
  for (const Launch& L : launches) {
    rt2_tracer::Slot& sl = t->slots[t->next_slot];
    t->next_slot ^= 1;
    // the slot's render stream waits for the accumulate that last read its sample buffer (or, serial,
    // for everything queued on the tracer stream so far); never for the other slot's render
    if (serial) {
      hipEvent_t e = TakeEvent(t);
      if (!e) return Fail(RT2_ERR_HIP, "event create failed");
      HIP_TRY(hipEventRecord(e, t->stream));
      HIP_TRY(hipStreamWaitEvent(sl.stream, e, 0));
      t->event_pool.push_back(e);
    } else if (sl.consumed_set) {
      HIP_TRY(hipStreamWaitEvent(sl.stream, sl.consumed, 0));
    }
    size_t need = octets((size_t)L.n_frames) * frame_bytes;
    if (need > sl.samples_bytes) {
      // grow geometrically (progressive loops raise their frames per call a little at a time)
      need = std::max(need, std::min(2 * sl.samples_bytes, octets((size_t)per_launch) * frame_bytes));
      // stream-ordered: the queued work still using the old buffer runs first; the host does not
      // wait (a multi-GPU tracer enqueues every GPU's render before any of them finishes)
      if (sl.samples) HIP_TRY(hipFreeAsync(sl.samples, sl.stream));
      sl.samples = nullptr;
      sl.samples_bytes = 0;
      HIP_TRY(hipMallocAsync((void**)&sl.samples, need, sl.stream));
      sl.samples_bytes = need;
      NoteDeviceBytes(t);
    }
    p.samples = sl.samples;
    const std::vector<uint32_t> tab(tabs.begin() + (long)L.table, tabs.begin() + (long)L.table + 2 * (L.n_chunks + 1));
    int rc = UploadChunks(t, sl, tab);
    if (rc != RT2_OK) return rc;
    p.frame_begin = L.frame_begin;
    p.n_frames = L.n_frames;
    p.chunks = sl.chunks;
    p.n_chunks = L.n_chunks;
    p.div_width = MakeMagic((uint32_t)t->width);  // pixel index -> (x, y)
    if (t->frame_tiles) {
      p.frame_tiles = 1u;
      p.frame_tile = 64u * p.local_pixels;
      p.div_frame_tile = MakeMagic(p.frame_tile);
      p.n_items = (L.n_chunks / 64u) * p.frame_tile;
    } else {
      p.n_items = L.n_chunks * p.tile_items;
    }
    p.batch_max = (uint32_t)t->batch_max;
    p.batch_div = (uint32_t)std::max<int64_t>(1, (resident / 64) * 2);  // half of the left work / waves
    int grid = (int)std::min<int64_t>(resident, (int64_t)p.n_items) / RenderBlockSize();
    grid = std::max(grid, 1);
    t->last_grid = grid;
    t->last_chunk_frames = L.first_len;
    p.work_counter = t->d_work + 16 * (&sl - t->slots);
    HIP_TRY(hipMemsetAsync(p.work_counter, 0, sizeof(uint32_t), sl.stream));
    // the launch's clock pair (RenderParams::launch_clock; read back by DrainEvents)
    const uint32_t ck = t->clock_next;
    t->clock_next = (t->clock_next + 1u) % (uint32_t)kClockRing;
    p.launch_clock = t->d_clock + 2u * ck;
    HIP_TRY(hipMemsetAsync(p.launch_clock, 0, 2 * sizeof(unsigned long long), sl.stream));
    HIP_TRY(LaunchRender(p, variant, counting, grid, sl.stream));
    t->pending.push_back(ck);
    // accumulate in frame order on the tracer stream, after this launch (RayTracer.cpp:64)
    HIP_TRY(hipEventRecord(sl.rendered, sl.stream));
    HIP_TRY(hipStreamWaitEvent(t->stream, sl.rendered, 0));
    HIP_TRY(LaunchAccumulate(sl.samples, t->d_accum, t->d_pixels, p.local_pixels, p.n_frames,
                             p.frame_begin + p.n_frames, t->stream));
    HIP_TRY(hipEventRecord(sl.consumed, t->stream));
    sl.consumed_set = true;
    t->launches++;
    t->paths += (uint64_t)p.n_frames * p.local_pixels;
    t->frame_idx += p.n_frames;
    // the ring's entries of unread launches must not be reused: read them back at half the ring
    if (t->pending.size() >= (size_t)kClockRing / 2) {
      int rc2 = DrainEvents(t);
      if (rc2 != RT2_OK) return rc2;
    }
  }
  return RT2_OK;
}

int Flush(rt2_tracer* t) {
  if (t->queued == 0) return RT2_OK;
  const int n = t->queued;
  t->queued = 0;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = LaunchFrames(t, n);
  t->enqueue_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

// ---- multi-GPU gather ----
// Sizes the root's gathered band stacks and full-image buffers for its current dims and world.
int EnsureImage(rt2_tracer* root) {
  const size_t npix = (size_t)root->width * (size_t)root->height;
  const size_t stacks = (size_t)root->world * (size_t)BandRowsMax(root) * (size_t)root->width * 3 * sizeof(float);
  if (root->d_image && root->image_pixels == npix && root->stacks_bytes == stacks) return RT2_OK;
  FreeImage(root);
  HIP_TRY(hipSetDevice(root->device));
  HIP_TRY(hipMalloc(&root->d_stacks, std::max<size_t>(stacks, 4)));
  HIP_TRY(hipMalloc(&root->d_image, std::max<size_t>(npix * 3 * sizeof(float), 4)));
  HIP_TRY(hipMalloc(&root->d_image_nc, std::max<size_t>(npix * 3 * sizeof(float), 4)));
  HIP_TRY(hipMalloc(&root->d_image_px, std::max<size_t>(npix * 4, 4)));
  root->stacks_bytes = stacks;
  root->image_pixels = npix;
  NoteDeviceBytes(root);
  return RT2_OK;
}

// Gathers the band stacks of `ranks` (every rank this thread drives: a multi tracer's parts, or
// one joined tracer) to rank 0 and de-interleaves them there. RCCL unless `loopback` (the ranks
// share one GPU and their stacks are copied on it). Enqueued on the streams; does not wait.
int GatherRanks(const std::vector<rt2_tracer*>& ranks, bool loopback) {
  rt2_tracer* root = nullptr;
  for (rt2_tracer* p : ranks) {
    int rc = Flush(p);
    if (rc != RT2_OK) return rc;
    if (p->rank == 0) root = p;
  }
  const rt2_tracer* r0 = ranks[0];
  for (rt2_tracer* p : ranks)
    if (p->width != r0->width || p->height != r0->height || p->frame_idx != r0->frame_idx)
      return Fail(RT2_ERR_INVALID, "gather: the ranks disagree on dims or frame index");
  const size_t count = (size_t)BandRowsMax(r0) * (size_t)r0->width * 3;  // floats per rank
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (root) {
    int rc = EnsureImage(root);
    if (rc != RT2_OK) return rc;
    HIP_TRY(hipSetDevice(root->device));
    e0 = TakeEvent(root);
    e1 = TakeEvent(root);
    if (e0) HIP_TRY(hipEventRecord(e0, root->stream));
  }
  if (count > 0) {
    if (loopback) {
      for (rt2_tracer* p : ranks) {
        HIP_TRY(hipSetDevice(p->device));
        if (p != root) {
          hipEvent_t e = TakeEvent(p);
          if (!e) return Fail(RT2_ERR_HIP, "event create failed");
          HIP_TRY(hipEventRecord(e, p->stream));
          HIP_TRY(hipStreamWaitEvent(root->stream, e, 0));
          p->event_pool.push_back(e);
        }
        HIP_TRY(hipMemcpyAsync(root->d_stacks + (size_t)p->rank * count, p->d_accum, count * sizeof(float),
                               hipMemcpyDeviceToDevice, root->stream));
      }
      // later work on a part's stream (Render, Reset) must not overwrite its accumulation while the
      // root's copy may still read it: every part stream waits for the copies
      if (ranks.size() > 1) {
        HIP_TRY(hipSetDevice(root->device));
        hipEvent_t e = TakeEvent(root);
        if (!e) return Fail(RT2_ERR_HIP, "event create failed");
        HIP_TRY(hipEventRecord(e, root->stream));
        for (rt2_tracer* p : ranks)
          if (p != root) HIP_TRY(hipStreamWaitEvent(p->stream, e, 0));
        root->event_pool.push_back(e);
      }
    } else {
      for (rt2_tracer* p : ranks)
        if (!p->comm) return Fail(RT2_ERR_INVALID, "gather: tracer is not part of a communicator");
      NCCL_TRY(ncclGroupStart());
      for (rt2_tracer* p : ranks) {
        ncclResult_t r = ncclGather(p->d_accum, p == root ? root->d_stacks : nullptr, count, ncclFloat32, 0, p->comm,
                                    p->stream);
        if (r != ncclSuccess) {
          (void)ncclGroupEnd();
          return Fail(RT2_ERR_HIP, std::string("ncclGather: ") + ncclGetErrorString(r));
        }
      }
      NCCL_TRY(ncclGroupEnd());
    }
  }
  if (root) {
    HIP_TRY(hipSetDevice(root->device));
    HIP_TRY(LaunchDeinterleave(root->d_stacks, root->d_image, root->d_image_nc, root->d_image_px, root->width,
                               root->height,
                               BandH(root), root->world, BandRowsMax(root), (int)root->frame_idx, root->stream));
    if (e1) HIP_TRY(hipEventRecord(e1, root->stream));
    if (e0 && e1) root->gpending.emplace_back(e0, e1);
    root->image_frame = root->frame_idx;
    root->gathers++;
  }
  return RT2_OK;
}

int GatherMulti(rt2_tracer* t) {
  if (IsMulti(t)) return GatherRanks(t->parts, t->loopback);
  if (t->comm) return GatherRanks({t}, false);
  if (t->world > 1) return Fail(RT2_ERR_INVALID, "gather: a partitioned tracer must be joined to a communicator");
  return GatherRanks({t}, true);  // one GPU, whole image: the "gather" is a device-local copy
}

// The root tracer holding the gathered image (rank 0), after a gather.
int ImageRoot(rt2_tracer* t, rt2_tracer** root) {
  rt2_tracer* r = IsMulti(t) ? t->parts[0] : t;
  if (r->rank != 0) return Fail(RT2_ERR_INVALID, "the gathered image lives on rank 0");
  if (r->image_frame < 0) return Fail(RT2_ERR_INVALID, "no gathered image (call rt2_tracer_gather first)");
  int rc = Sync(r);
  if (rc != RT2_OK) return rc;
  *root = r;
  return RT2_OK;
}
}  // namespace

extern "C" {

// Update()/Render() only queue frames: the queued frames are launched together when a result is
// read (any readback, query, synchronize, stats), when a setting that affects them changes, or
// when lazy_max frames are queued. Results cannot tell the difference (samples are summed in frame
// order), but App::Run's headless pattern — num_samples x Update() then one readback
// (App.cpp:243-248) — then runs as one launch instead of num_samples one-frame launches, each
// of which would be as long as its longest path.
int rt2_tracer_render(rt2_tracer* t, int n_frames) {
  if (!t || n_frames < 0) return Fail(RT2_ERR_INVALID, "n_frames must be >= 0");
  RT2_FORWARD(t, rt2_tracer_render(p, n_frames));
  if ((int64_t)t->frame_idx + t->queued + n_frames > 0x7FFFFFFF)
    return Fail(RT2_ERR_INVALID, "frame index overflow");
  if (t->camera.Params().sqrt_spp <= 0) return Fail(RT2_ERR_INVALID, "samples_per_pixel gives sqrt_spp = 0");
  if (t->origins_bounded && !CameraOriginsBounded(t->camera.Params())) return Fail(RT2_ERR_INVALID, kCameraRangeMsg);
  t->queued += n_frames;
  if (t->lazy_max > 0 && t->queued < t->lazy_max) return RT2_OK;
  return Flush(t);
}

int rt2_tracer_set_lazy_frames(rt2_tracer* t, int max_queued) {
  if (!t || max_queued < 0) return Fail(RT2_ERR_INVALID, "max_queued must be >= 0");
  RT2_FORWARD(t, rt2_tracer_set_lazy_frames(p, max_queued));
  t->lazy_max = max_queued;
  if (max_queued == 0 || t->queued >= max_queued) return Flush(t);
  return RT2_OK;
}

int rt2_tracer_update(rt2_tracer* t) { return rt2_tracer_render(t, 1); }

int rt2_tracer_flush(rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_flush(p));
  return Flush(t);
}

int rt2_tracer_synchronize(rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_synchronize(p));
  return Sync(t);
}

int64_t rt2_tracer_frame_idx(const rt2_tracer* t) {
  if (!t) return -1;
  if (IsMulti(t)) return rt2_tracer_frame_idx(t->parts[0]);
  return t->frame_idx + t->queued;
}

int rt2_tracer_dims(const rt2_tracer* t, int* w, int* h) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  if (w) *w = t->width;
  if (h) *h = t->height;
  return RT2_OK;
}

int rt2_tracer_local_rows(const rt2_tracer* t) {
  if (!t) return -1;
  return IsMulti(t) ? t->height : t->local_rows;
}

int rt2_tracer_n_gpus(const rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  return IsMulti(t) ? (int)t->parts.size() : 1;
}

int rt2_tracer_accumulation(rt2_tracer* t, float* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  if (IsMulti(t)) {
    int rc = GatherMulti(t);
    return rc != RT2_OK ? rc : rt2_tracer_image_accumulation(t, out);
  }
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  size_t n = (size_t)t->width * (size_t)t->local_rows;
  if (n) HIP_TRY(hipMemcpy(out, t->d_accum, n * 3 * sizeof(float), hipMemcpyDeviceToHost));
  return RT2_OK;
}

int rt2_tracer_non_converted_pixels(rt2_tracer* t, float* out) {
  int rc = rt2_tracer_accumulation(t, out);
  if (rc != RT2_OK) return rc;
  size_t n = (size_t)t->width * (size_t)rt2_tracer_local_rows(t) * 3;
  float f = (float)rt2_tracer_frame_idx(t);  // accumulation / frame_idx_ (RayTracer.cpp:108-109)
  for (size_t i = 0; i < n; i++) out[i] = out[i] / f;
  return RT2_OK;
}

int rt2_tracer_pixels(rt2_tracer* t, uint8_t* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  if (IsMulti(t)) {
    int rc = GatherMulti(t);
    return rc != RT2_OK ? rc : rt2_tracer_image_pixels(t, out);
  }
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  size_t n = (size_t)t->width * (size_t)t->local_rows;
  if (n) HIP_TRY(hipMemcpy(out, t->d_pixels, n * 4, hipMemcpyDeviceToHost));
  return RT2_OK;
}

int rt2_tracer_pixels_async(rt2_tracer* t, uint8_t* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  if (IsMulti(t)) {
    int rc = GatherMulti(t);
    if (rc != RT2_OK) return rc;
    rt2_tracer* r = t->parts[0];
    HIP_TRY(hipSetDevice(r->device));
    size_t n = (size_t)t->width * (size_t)t->height;
    if (n) HIP_TRY(hipMemcpyAsync(out, r->d_image_px, n * 4, hipMemcpyDeviceToHost, r->stream));
    return RT2_OK;
  }
  int rc = Flush(t);
  if (rc != RT2_OK) return rc;
  HIP_TRY(hipSetDevice(t->device));
  size_t n = (size_t)t->width * (size_t)t->local_rows;
  if (n) HIP_TRY(hipMemcpyAsync(out, t->d_pixels, n * 4, hipMemcpyDeviceToHost, t->stream));
  return RT2_OK;
}

int rt2_tracer_query(rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  if (IsMulti(t)) {
    int all = 1;
    for (rt2_tracer* p : t->parts) {
      int q = rt2_tracer_query(p);
      if (q < 0) return q;
      all &= q;
    }
    return all;
  }
  int rc = Flush(t);
  if (rc != RT2_OK) return rc;
  HIP_TRY(hipSetDevice(t->device));
  hipError_t e = hipStreamQuery(t->stream);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return HipFail(e, "hipStreamQuery");
}

int rt2_host_alloc(size_t bytes, void** out) {
  if (!out) return Fail(RT2_ERR_INVALID, "null argument");
  *out = nullptr;
  HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return RT2_OK;
}

void rt2_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int rt2_tracer_copy_accum_device(rt2_tracer* t, void* dst, void* stream) {
  if (!t || !dst) return Fail(RT2_ERR_INVALID, "null argument");
  const float* src;
  size_t n;
  rt2_tracer* o = t;  // the tracer whose stream orders the copy
  if (IsMulti(t)) {
    int rc = GatherMulti(t);
    if (rc != RT2_OK) return rc;
    o = t->parts[0];
    src = o->d_image;
    n = (size_t)t->width * (size_t)t->height;
  } else {
    int rc = Flush(t);
    if (rc != RT2_OK) return rc;
    src = t->d_accum;
    n = (size_t)t->width * (size_t)t->local_rows;
  }
  HIP_TRY(hipSetDevice(o->device));
  hipStream_t s = stream ? (hipStream_t)stream : o->stream;
  if (s != o->stream) {
    hipEvent_t e = TakeEvent(o);
    if (!e) return Fail(RT2_ERR_HIP, "event create failed");
    HIP_TRY(hipEventRecord(e, o->stream));
    HIP_TRY(hipStreamWaitEvent(s, e, 0));
    o->event_pool.push_back(e);
  }
  if (n) HIP_TRY(hipMemcpyAsync(dst, src, n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
  return RT2_OK;
}

int rt2_tracer_enable_ray_counts(rt2_tracer* t, int on) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_enable_ray_counts(p, on));
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  t->ray_counts_on = on != 0;
  if ((rc = Realloc(t)) != RT2_OK) return rc;
  return ResetFrame(t);
}

int rt2_tracer_ray_counts(rt2_tracer* t, uint32_t* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  if (IsMulti(t)) {  // a diagnostic: each GPU's rows read back and placed on the host
    std::vector<uint32_t> part;
    for (rt2_tracer* p : t->parts) {
      part.resize((size_t)p->width * (size_t)p->local_rows);
      int rc = rt2_tracer_ray_counts(p, part.data());
      if (rc != RT2_OK) return rc;
      const int bh = BandH(p);
      for (int r = 0; r < p->local_rows; r++) {
        const int period = r / bh;  // the rank's band of this period (rt2_layout.h BandRank)
        const int phase = ((p->rank - period) % p->world + p->world) % p->world;
        const int y = (period * p->world + phase) * bh + r % bh;
        memcpy(out + (size_t)y * p->width, part.data() + (size_t)r * p->width, (size_t)p->width * sizeof(uint32_t));
      }
    }
    return RT2_OK;
  }
  if (!t->d_ray_counts) return Fail(RT2_ERR_INVALID, "ray counts not enabled");
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  size_t n = (size_t)t->width * (size_t)t->local_rows;
  if (n) HIP_TRY(hipMemcpy(out, t->d_ray_counts, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return RT2_OK;
}

int rt2_tracer_enable_stats(rt2_tracer* t, int on) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_enable_stats(p, on));
  int rc = FlushIfChanged(t, t->stats_on, on != 0);
  if (rc != RT2_OK) return rc;
  t->stats_on = on != 0;
  return RT2_OK;
}

int rt2_tracer_get_stats(rt2_tracer* t, rt2_stats* o) {
  if (!t || !o) return Fail(RT2_ERR_INVALID, "null argument");
  if (IsMulti(t)) {  // sums over the GPUs; launches per GPU, kernel_ms of the busiest GPU
    rt2_stats sum;
    memset(&sum, 0, sizeof(sum));
    for (rt2_tracer* p : t->parts) {
      rt2_stats s;
      int rc = rt2_tracer_get_stats(p, &s);
      if (rc != RT2_OK) return rc;
      sum.rays += s.rays;
      sum.paths += s.paths;
      sum.bvh_tests += s.bvh_tests;
      sum.quad_tests += s.quad_tests;
      sum.sphere_tests += s.sphere_tests;
      sum.xform_visits += s.xform_visits;
      sum.medium_tests += s.medium_tests;
      sum.list_visits += s.list_visits;
      sum.overflow += s.overflow;
      sum.box_tests += s.box_tests;
      sum.box_certified += s.box_certified;
      sum.box_wave_visits += s.box_wave_visits;
      sum.box_wave_runs += s.box_wave_runs;
      sum.launches = std::max(sum.launches, s.launches);
      sum.kernel_ms = std::max(sum.kernel_ms, s.kernel_ms);
      sum.launch_ms_sum = std::max(sum.launch_ms_sum, s.launch_ms_sum);
      for (int k = 0; k < 4; k++) sum.stamps[k] += s.stamps[k];
      for (int k = 0; k < 8; k++) sum.diag[k] += s.diag[k];
      sum.gathers += s.gathers;
      sum.gather_ms += s.gather_ms;
      sum.enqueue_ms += s.enqueue_ms;
      sum.readbacks += s.readbacks;
      sum.readback_ms += s.readback_ms;
      sum.host_waits += s.host_waits;
      sum.sample_buffer_bytes = std::max(sum.sample_buffer_bytes, s.sample_buffer_bytes);
      sum.device_bytes_peak = std::max(sum.device_bytes_peak, s.device_bytes_peak);
    }
    *o = sum;
    return RT2_OK;
  }
  const uint64_t waits = t->host_waits;  // (this diagnostic's own synchronization is not counted)
  int rc = Sync(t);
  t->host_waits = waits;
  if (rc != RT2_OK) return rc;
  unsigned long long s[kStatsSlots];
  HIP_TRY(hipSetDevice(t->device));
  HIP_TRY(hipMemcpy(s, t->d_stats, sizeof(s), hipMemcpyDeviceToHost));
  o->rays = s[StatsCounters::kRays];
  o->paths = t->paths;  // every (pixel, frame) of a launch finishes exactly one camera path
  o->bvh_tests = s[StatsCounters::kBvhTests];
  o->quad_tests = s[StatsCounters::kQuadTests];
  o->sphere_tests = s[StatsCounters::kSphereTests];
  o->xform_visits = s[StatsCounters::kXformVisits];
  o->medium_tests = s[StatsCounters::kMediumTests];
  o->list_visits = s[StatsCounters::kListVisits];
  o->overflow = s[StatsCounters::kCount];
  o->box_tests = s[StatsCounters::kBoxTests];
  o->box_certified = s[StatsCounters::kBoxCertified];
  o->box_wave_visits = s[StatsCounters::kBoxWaveVisits];
  o->box_wave_runs = s[StatsCounters::kBoxWaveRuns];
  for (int k = 0; k < 4; k++) o->stamps[k] = s[StatsCounters::kStamps + k];
  for (int k = 0; k < 8; k++) o->diag[k] = s[StatsCounters::kDiag + k];
  o->launches = t->launches;
  o->kernel_ms = t->kernel_ms;
  o->launch_ms_sum = t->launch_ms_sum;
  o->gathers = t->gathers;
  o->gather_ms = t->gather_ms;
  o->enqueue_ms = t->enqueue_ms;
  o->readbacks = t->readbacks;
  o->readback_ms = t->readback_ms;
  o->host_waits = t->host_waits;
  o->sample_buffer_bytes = t->slots[0].samples_bytes + t->slots[1].samples_bytes;
  o->device_bytes_peak = std::max(t->device_bytes_peak, DeviceBytes(t));
  return RT2_OK;
}

int rt2_tracer_part_stats(rt2_tracer* t, int part, rt2_stats* o) {
  if (!t || !o) return Fail(RT2_ERR_INVALID, "null argument");
  const int n = IsMulti(t) ? (int)t->parts.size() : 1;
  if (part < 0 || part >= n) return Fail(RT2_ERR_INVALID, "rt2_tracer_part_stats: part out of range");
  return rt2_tracer_get_stats(IsMulti(t) ? t->parts[(size_t)part] : t, o);
}

// ---- multi-GPU entry points ----
int rt2_multi_plan(int n, const int* devices, int band_h, int width, int height, rt2_part_plan* out, int* loopback) {
  if (n < 1 || band_h < 0) return Fail(RT2_ERR_INVALID, "rt2_tracer_create_multi: need n_gpus >= 1, band_h >= 0");
  if (width < 0 || height < 0) return Fail(RT2_ERR_INVALID, "rt2_multi_plan: negative dims");
  std::vector<int> devs((size_t)n);
  for (int i = 0; i < n; i++) devs[(size_t)i] = devices ? devices[i] : i;
  for (int d : devs)
    if (d < 0) return Fail(RT2_ERR_INVALID, "rt2_tracer_create_multi: negative device id");
  const bool all_same = std::all_of(devs.begin(), devs.end(), [&](int d) { return d == devs[0]; });
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (!distinct && !all_same)
    return Fail(RT2_ERR_INVALID, "rt2_tracer_create_multi: devices must be distinct (or all one GPU, for tests)");
  const int bh = band_h > 0 ? band_h : kDefaultBandH;
  if (loopback) *loopback = n > 1 && all_same ? 1 : 0;
  if (out) {
    for (int i = 0; i < n; i++) {
      rt2_part_plan& q = out[i];
      q.device = devs[(size_t)i];
      q.rank = i;
      q.world = n;
      q.band_h = bh;
      q.local_rows = height > 0 ? LocalRows(height, bh, i, n) : 0;
      q.rows_max = rt2::BandRowsMax(height, bh, n);
    }
  }
  return RT2_OK;
}

int rt2_tracer_create_multi(const rt2_scene* s, int n, const int* devices, int band_h, rt2_tracer** out) {
  if (!s || !out) return Fail(RT2_ERR_INVALID, "rt2_tracer_create_multi: null argument");
  *out = nullptr;
  int lb = 0;
  int prc = rt2_multi_plan(n, devices, band_h, 0, 0, nullptr, &lb);
  if (prc != RT2_OK) return prc;
  std::vector<int> devs((size_t)n);
  for (int i = 0; i < n; i++) devs[(size_t)i] = devices ? devices[i] : i;
  auto m = std::make_unique<rt2_tracer>();
  m->loopback = lb != 0;
  const int bh = band_h > 0 ? band_h : kDefaultBandH;
  auto cleanup = [&](int rc) {
    for (rt2_tracer* p : m->parts) rt2_tracer_destroy(p);
    m->parts.clear();
    return rc;
  };
  for (int i = 0; i < n; i++) {
    rt2_tracer* p = nullptr;
    int rc = rt2_tracer_create(s, devs[(size_t)i], &p);
    if (rc != RT2_OK) return cleanup(rc);
    m->parts.push_back(p);
    if ((rc = rt2_tracer_set_partition(p, bh, i, n)) != RT2_OK) return cleanup(rc);
  }
  if (!m->loopback) {  // one communicator per device (rank i on devs[i]), RCCL over xGMI
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
    if (r != ncclSuccess) return cleanup(Fail(RT2_ERR_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r)));
    for (int i = 0; i < n; i++) m->parts[(size_t)i]->comm = comms[(size_t)i];
  }
  m->device = devs[0];
  m->width = m->parts[0]->width;
  m->height = m->parts[0]->height;
  m->band_h = bh;
  m->world = n;
  *out = m.release();
  return RT2_OK;
}

int rt2_comm_unique_id(uint8_t* out, size_t cap) {
  if (!out || cap < sizeof(ncclUniqueId)) return Fail(RT2_ERR_INVALID, "rt2_comm_unique_id: need RT2_UNIQUE_ID_BYTES");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof(id));
  return RT2_OK;
}

int rt2_tracer_join(rt2_tracer* t, const uint8_t* unique_id, int world, int rank, int band_h) {
  if (!t || !unique_id) return Fail(RT2_ERR_INVALID, "rt2_tracer_join: null argument");
  if (IsMulti(t)) return Fail(RT2_ERR_INVALID, "rt2_tracer_join: a multi-GPU tracer has its own communicators");
  if (t->comm) return Fail(RT2_ERR_INVALID, "rt2_tracer_join: already joined");
  int rc = rt2_tracer_set_partition(t, band_h > 0 ? band_h : kDefaultBandH, rank, world);
  if (rc != RT2_OK) return rc;
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  HIP_TRY(hipSetDevice(t->device));
  NCCL_TRY(ncclCommInitRank(&t->comm, world, id, rank));
  return RT2_OK;
}

int rt2_tracer_gather(rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  return GatherMulti(t);
}

int rt2_tracer_image_accumulation(rt2_tracer* t, float* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  rt2_tracer* r = nullptr;
  int rc = ImageRoot(t, &r);
  if (rc != RT2_OK) return rc;
  size_t n = (size_t)r->width * (size_t)r->height;
  if (n) HIP_TRY(hipMemcpy(out, r->d_image, n * 3 * sizeof(float), hipMemcpyDeviceToHost));
  return RT2_OK;
}

// NonConvertedPixels() of the gathered image: accumulation / frame_idx_ (RayTracer.cpp:108-109),
// divided on the GPU by the de-interleave kernel (the same IEEE quotient as the host's)
int rt2_tracer_image_non_converted_pixels(rt2_tracer* t, float* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  rt2_tracer* r = nullptr;
  int rc = ImageRoot(t, &r);
  if (rc != RT2_OK) return rc;
  const size_t n = (size_t)r->width * (size_t)r->height;
  const auto t0 = std::chrono::steady_clock::now();
  if (n) HIP_TRY(hipMemcpy(out, r->d_image_nc, n * 3 * sizeof(float), hipMemcpyDeviceToHost));
  r->readback_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  r->readbacks++;
  return RT2_OK;
}

// The same, enqueued on the root's stream (out: pinned host memory, rt2_host_alloc); complete once
// rt2_tracer_query returns 1 or after rt2_tracer_synchronize. Needs a gather enqueued before it.
int rt2_tracer_image_non_converted_pixels_async(rt2_tracer* t, float* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  rt2_tracer* r = IsMulti(t) ? t->parts[0] : t;
  if (r->rank != 0) return Fail(RT2_ERR_INVALID, "the gathered image lives on rank 0");
  if (r->image_frame < 0) return Fail(RT2_ERR_INVALID, "no gathered image (call rt2_tracer_gather first)");
  HIP_TRY(hipSetDevice(r->device));
  const size_t n = (size_t)r->width * (size_t)r->height;
  hipEvent_t e0 = TakeEvent(r), e1 = TakeEvent(r);
  if (e0) HIP_TRY(hipEventRecord(e0, r->stream));
  if (n) HIP_TRY(hipMemcpyAsync(out, r->d_image_nc, n * 3 * sizeof(float), hipMemcpyDeviceToHost, r->stream));
  if (e1) HIP_TRY(hipEventRecord(e1, r->stream));
  if (e0 && e1) r->rpending.emplace_back(e0, e1);
  r->readbacks++;
  return RT2_OK;
}

int rt2_tracer_image_pixels(rt2_tracer* t, uint8_t* out) {
  if (!t || !out) return Fail(RT2_ERR_INVALID, "null argument");
  rt2_tracer* r = nullptr;
  int rc = ImageRoot(t, &r);
  if (rc != RT2_OK) return rc;
  size_t n = (size_t)r->width * (size_t)r->height;
  if (n) HIP_TRY(hipMemcpy(out, r->d_image_px, n * 4, hipMemcpyDeviceToHost));
  return RT2_OK;
}

int rt2_selftest(int device, int which, uint64_t n, uint64_t seed, uint64_t* mismatches, uint64_t* checked) {
  if (!mismatches || !checked) return Fail(RT2_ERR_INVALID, "null argument");
  if (which < 0 || which > 9) return Fail(RT2_ERR_INVALID, "unknown self-test");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return Fail(RT2_ERR_HIP, "no HIP device available");
  HIP_TRY(hipSetDevice(device));
  unsigned long long* d = nullptr;
  HIP_TRY(hipMalloc(&d, 2 * sizeof(unsigned long long)));
  unsigned long long h[2] = {0, 0};
  hipError_t e = hipMemset(d, 0, sizeof(h));
  if (e == hipSuccess) e = LaunchSelftest(which, (unsigned long long)n, (uint32_t)seed, d, nullptr);
  if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return HipFail(e, "self-test");
  *mismatches = h[0];
  *checked = h[1];
  return RT2_OK;
}

int rt2_tracer_reset_stats(rt2_tracer* t) {
  if (!t) return Fail(RT2_ERR_INVALID, "null tracer");
  RT2_FORWARD(t, rt2_tracer_reset_stats(p));
  int rc = Sync(t);
  if (rc != RT2_OK) return rc;
  HIP_TRY(hipSetDevice(t->device));
  HIP_TRY(hipMemset(t->d_stats, 0, kStatsSlots * sizeof(unsigned long long)));
  t->launches = 0;
  t->paths = 0;
  t->kernel_ms = 0;
  t->launch_ms_sum = 0;
  t->busy_end = 0;
  t->gathers = 0;
  t->gather_ms = 0;
  t->enqueue_ms = 0;
  t->readbacks = 0;
  t->readback_ms = 0;
  t->host_waits = 0;
  return RT2_OK;
}

int rt2_band_rows_max(int height, int band_h, int world) {
  if (height < 0 || band_h < 0 || world < 1) return Fail(RT2_ERR_INVALID, "bad band layout");
  return rt2::BandRowsMax(height, band_h, world);
}

int rt2_deinterleave_host(const float* stacks, float* image, int width, int height, int band_h, int world,
                          int max_rows, int channels) {
  if (!stacks || !image || width < 0 || height < 0 || band_h < 0 || world < 1 || channels < 1)
    return Fail(RT2_ERR_INVALID, "bad de-interleave arguments");
  if (max_rows < rt2::BandRowsMax(height, band_h, world))
    return Fail(RT2_ERR_INVALID, "max_rows is below the largest rank's band stack");
  const size_t row = (size_t)width * (size_t)channels;
  for (int y = 0; y < height; y++) {
    const BandRow src = BandSource(y, band_h, world);
    memcpy(image + (size_t)y * row, stacks + ((size_t)src.rank * (size_t)max_rows + (size_t)src.row) * row,
           row * sizeof(float));
  }
  return RT2_OK;
}

int rt2_runtime_info(char* out, size_t cap) {
  if (!out || cap == 0) return Fail(RT2_ERR_INVALID, "null argument");
  int v = 0;
  (void)ncclGetVersion(&v);
  auto path_of = [](const void* sym) {
    Dl_info di;
    return dladdr(sym, &di) && di.dli_fname ? std::string(di.dli_fname) : std::string("?");
  };
  const std::string s = "rccl " + std::to_string(v) + " " + path_of((const void*)&ncclGetVersion) + "; hip " +
                        path_of((const void*)&hipGetDeviceCount);
  snprintf(out, cap, "%s", s.c_str());
  return RT2_OK;
}

int rt2_write_image(const float* pixels, int w, int h, const char* path, int png) {
  if (!pixels || !path || w <= 0 || h <= 0) return Fail(RT2_ERR_INVALID, "bad image arguments");
  std::string err;
  if (!WriteImage(pixels, w, h, path, png != 0, err)) return Fail(RT2_ERR_IO, err);
  return RT2_OK;
}

}  // extern "C"
