/* rt2.h — C ABI of the MI355X (gfx950) replacement for the reference renderer's hot path.
 *
 * Drop-in boundary for tonadr1022/Raytrace2 `raytrace2::cpu::RayTracer` (src/cpu_raytrace/
 * RayTracer.hpp:15-42) and the host surface that stays around it: `serialize::SceneLoader`,
 * `LoadCamera`, `WriteCamera`, `LoadAppSettings` (src/Serialize.hpp:21-35) and
 * `util::WriteImage` (src/Util.hpp:11-12). Plain pointers and sizes only; no HIP or torch types in
 * the signatures (streams are passed as void*). Every function returns RT2_OK (0) or a negative
 * status and never throws; rt2_last_error() has the message (thread-local).
 *
 * Pixel layout: row-major, row 0 = bottom image row (RayTracer.cpp:97-102). With a row-band
 * partition (rt2_tracer_set_partition) a tracer owns the "local rows" y whose band b = y / band_h
 * has (b % world + b / world) % world == rank (one band per period of `world` bands, the phase
 * rotating by one each period), stored compactly in increasing y.
 */
#ifndef RT2_H_
#define RT2_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT2_API __attribute__((visibility("default")))

enum {
  RT2_OK = 0,
  RT2_ERR_INVALID = -1, /* bad argument or call order */
  RT2_ERR_IO = -2,      /* file missing / unreadable / unwritable */
  RT2_ERR_SCENE = -3,   /* scene schema or compile error */
  RT2_ERR_HIP = -4,     /* HIP runtime error (no device, out of memory, launch failure) */
};

typedef struct rt2_scene rt2_scene;
typedef struct rt2_tracer rt2_tracer;

RT2_API const char* rt2_last_error(void);
/* "rt2-mi355x <version> (gfx950) kernel <12 hex digits>": the last field identifies the kernel sources
 * (render.hip + rt2_layout.h) the library was built from */
RT2_API const char* rt2_version(void);

/* ---- SceneLoader::LoadScene (Serialize.cpp:199-360) + App.cpp:126 (top-level BVHNode) ----
 * Accepts the v2 schema and the legacy {"primitives":{"spheres":[...]}} schema (documented
 * adapter: each sphere is a top-level node; a missing camera means "cam1"). Camera names resolve
 * to <scene dir>/<name>.json. `seed` keys the Perlin-table random streams (the reference draws them
 * from its unseeded RNG at load, PerlinNoiseGen.cpp:41-50). */
RT2_API int rt2_scene_load(const char* path, uint64_t seed, rt2_scene** out);
/* The environment variable RT2_NO_LIST_ACCEL=1 at load keeps every list a linear child loop. */
RT2_API void rt2_scene_free(rt2_scene* scene);

typedef struct {
  int dims_x, dims_y; /* Scene::dims (camera width / aspect), 0 when absent */
  int n_materials, n_textures, n_primitives, n_top_nodes;
  float background[3];
  int legacy_schema;
  int bvh_nodes, quads, spheres, lists, xforms, media; /* flattened records */
  int max_stack, bvh_depth;
  uint64_t node_bytes;
  int acc_lists, acc_nodes; /* sphere lists given an exact acceleration tree, and its nodes */
  int linear_steps;         /* threaded-program length (0: the scene uses the stack traversal) */
  int origins_bounded;      /* 1: the threaded program's exact tests need camera rays starting within
                             * +-2^64 (rectangle quads, box boundaries, transforms about y); a launch
                             * refuses a camera beyond that (RT2_ERR_INVALID). 0: any camera renders */
  int box_steps;            /* MakeBox runs and MakeBox medium boundaries given the box-level test */
} rt2_scene_info;
RT2_API int rt2_scene_get_info(const rt2_scene* scene, rt2_scene_info* out);
/* Material table, 8 floats per material: type, albedo.xyz, fuzz, refraction_index, tex_idx, 0.
 * type: 0 metal, 1 lambertian, 2 dielectric, 3 texture, 4 diffuse_light, 5 isotropic
 * (variant order of Fwd.hpp:13-14). Returns the material count. */
RT2_API int rt2_scene_materials(const rt2_scene* scene, float* out, int cap);
/* Texture table, 8 floats: type (0 solid, 1 checker, 2 noise), albedo.xyz, inv_scale|scale,
 * even, odd, noise_type. Returns the texture count. */
RT2_API int rt2_scene_textures(const rt2_scene* scene, float* out, int cap);
/* Perlin tables of noise texture `tex`: vec = point_count*3 floats, perm = 3*point_count ints
 * (perm_x, perm_y, perm_z). Returns point_count. */
RT2_API int rt2_scene_perlin(const rt2_scene* scene, int tex, float* vec, int* perm);

/* ---- Camera (Camera.hpp:10-137) ---- */
typedef struct {
  float center[3], look_at[3], view_up[3];
  float vfov, defocus_angle, focus_distance;
} rt2_camera_desc;
RT2_API int rt2_scene_get_camera(const rt2_scene* scene, rt2_camera_desc* out);
RT2_API int rt2_scene_set_camera(rt2_scene* scene, const rt2_camera_desc* cam);
/* Camera::Update for (w, h, spp): out[21] = pixel00(3) du(3) dv(3) center(3) defocus_u(3)
 * defocus_v(3) defocus_angle recip_sqrt_spp sqrt_spp */
RT2_API int rt2_camera_params(const rt2_scene* scene, int w, int h, int spp, float* out);
RT2_API int rt2_camera_load(const char* path, rt2_camera_desc* out);         /* LoadCamera */
RT2_API int rt2_camera_write(const rt2_camera_desc* cam, const char* path);  /* WriteCamera */

/* ---- LoadAppSettings (Serialize.cpp:56-65) ---- */
typedef struct {
  int render_once, save_after_render_once;
  int64_t num_samples, max_depth;
  int render_window;
} rt2_app_settings;
RT2_API int rt2_settings_load(const char* path, rt2_app_settings* out);

/* ---- RayTracer (RayTracer.hpp:15-42) on one GPU ----
 * create:   compiles the scene program and uploads it to `device` (the scene may be freed after).
 * on_resize:OnResize(dims) (RayTracer.cpp:87-104): sets camera dims, reallocates, Reset().
 * update:   Update(scene) (RayTracer.cpp:55-70): one frame, stratum (f % sq, f / sq % sq).
 * render:   n consecutive Update() calls, executed as ceil(n / launch_frames) kernel launches.
 * Update()/render() queue their frames; queued frames are launched together at the next readback,
 * query, synchronize or stats call, before a change of max_depth / spp / seed / stats mode, or once
 * `lazy_frames` (default 4096; 0 = launch at every call) are queued. Reset/OnResize drop queued
 * frames. Results are identical either way; FrameIdx() counts queued frames. Launched frames run on
 * the tracer's stream; readbacks synchronise it. */
RT2_API int rt2_tracer_create(const rt2_scene* scene, int device, rt2_tracer** out); /* n GPUs: see below */
RT2_API void rt2_tracer_destroy(rt2_tracer* tr);
RT2_API int rt2_tracer_set_stream(rt2_tracer* tr, void* hip_stream); /* NULL = own stream */
RT2_API int rt2_tracer_set_max_depth(rt2_tracer* tr, int max_depth); /* RayTracer::max_depth, <= 65535 */
RT2_API int rt2_tracer_set_samples_per_pixel(rt2_tracer* tr, int spp); /* App.cpp:129 */
RT2_API int rt2_tracer_set_seed(rt2_tracer* tr, uint64_t seed);
RT2_API int rt2_tracer_set_partition(rt2_tracer* tr, int band_h, int rank, int world);
RT2_API int rt2_tracer_set_launch_frames(rt2_tracer* tr, int frames_per_launch); /* 0 = all */
/* Work split: a launch's frames are cut into chunks and every (pixel, chunk) is one work item. A
 * chunk starting with R frames left holds about R * pixels / (k * resident GPU lanes) frames, k =
 * `items_per_lane` (default 4), at least 1 and at most 64 (RT2_CHUNK_MAX): long items early, short
 * ones at the end of the launch. 0 = one chunk (each pixel's frames in one item). Every frame's
 * sample goes to a per-frame buffer and is summed in frame order after the launch, so results do
 * not depend on the split. `bytes` bounds the device memory the samples take on each GPU in total
 * (default 24 GiB of the MI355X's 288 GB): consecutive launches alternate between two launch slots,
 * each with its own sample buffer of at most bytes / 2, so that a launch's tail overlaps the next
 * launch; a render needing more than bytes / 2 of samples runs as several launches (at least one
 * 8-frame octet each). rt2_stats.sample_buffer_bytes / device_bytes_peak report what is held. */
RT2_API int rt2_tracer_set_lazy_frames(rt2_tracer* tr, int max_queued);
RT2_API int rt2_tracer_flush(rt2_tracer* tr); /* launch the queued frames now (does not wait) */
RT2_API int rt2_tracer_set_work_split(rt2_tracer* tr, int items_per_lane);
RT2_API int rt2_tracer_set_sample_budget(rt2_tracer* tr, uint64_t bytes);
/* Most work items a GPU wave reserves with one atomic (default 64); batches shrink as the launch
 * drains. */
RT2_API int rt2_tracer_set_batch_max(rt2_tracer* tr, int items);
/* Launch shape of the last render: persistent workgroups, frames of its first chunk, kernel variant. */
RT2_API int rt2_tracer_last_launch(const rt2_tracer* tr, int* grid, int* chunk_frames, int* variant);
RT2_API int rt2_tracer_on_resize(rt2_tracer* tr, int width, int height);
RT2_API int rt2_tracer_reset(rt2_tracer* tr);
RT2_API int rt2_tracer_update(rt2_tracer* tr);
RT2_API int rt2_tracer_render(rt2_tracer* tr, int n_frames);
RT2_API int rt2_tracer_synchronize(rt2_tracer* tr);
RT2_API int64_t rt2_tracer_frame_idx(const rt2_tracer* tr); /* FrameIdx */
RT2_API int rt2_tracer_dims(const rt2_tracer* tr, int* width, int* height); /* Dims */
RT2_API int rt2_tracer_local_rows(const rt2_tracer* tr);
/* NonConvertedPixels (RayTracer.cpp:105-112): accum / frame_idx, float3 per local pixel */
RT2_API int rt2_tracer_non_converted_pixels(rt2_tracer* tr, float* out);
RT2_API int rt2_tracer_accumulation(rt2_tracer* tr, float* out); /* raw float3 sums */
RT2_API int rt2_tracer_pixels(rt2_tracer* tr, uint8_t* out_rgba); /* Pixels(): RGBA8 */
/* Progressive display (App.cpp:176-242 without the window): enqueue the Pixels() readback after the
 * frames already enqueued and return at once; the buffer is complete when rt2_tracer_query returns
 * 1 (all enqueued work done; 0 = still running) or after rt2_tracer_synchronize. Pinned host memory
 * from rt2_host_alloc makes the copy a DMA that does not stall the host. */
RT2_API int rt2_tracer_pixels_async(rt2_tracer* tr, uint8_t* out_rgba);
RT2_API int rt2_tracer_query(rt2_tracer* tr);
RT2_API int rt2_host_alloc(size_t bytes, void** out);
RT2_API void rt2_host_free(void* ptr);
/* Device-to-device copy of the local accumulation (float3 per local pixel) into `dst_device`,
 * ordered on `hip_stream` (NULL = tracer stream) — used for the multi-GPU gather. */
RT2_API int rt2_tracer_copy_accum_device(rt2_tracer* tr, void* dst_device, void* hip_stream);
/* ---- RayTracer::camera (RayTracer.hpp:31) ----
 * The reference borrows `Camera* camera` (= &scene.cam, App.cpp:130) and calls camera->Update() at
 * every Update() (RayTracer.cpp:56): a camera moved between Update() calls takes effect at the next
 * frame and does not reset the accumulation. set_camera gives the tracer the setter fields of
 * Camera.hpp:69-101 (center, look_at, view_up, vfov, defocus_angle, focus_distance; dims and
 * samples_per_pixel stay as on_resize / set_samples_per_pixel set them). When they change, frames
 * queued so far are launched first, with the camera they were queued under. Rendering refuses, with
 * RT2_ERR_INVALID, a camera whose rays would start beyond +-2^64 on an axis (center plus the defocus
 * disk): the kernel's exact axis-aligned rectangle test assumes ray origins within +-2^100. */
RT2_API int rt2_tracer_set_camera(rt2_tracer* tr, const rt2_camera_desc* cam);
RT2_API int rt2_tracer_get_camera(const rt2_tracer* tr, rt2_camera_desc* out);

/* ---- Multi-GPU; replaces the reference's data-parallel pixel loop
 * std::for_each(std::execution::par, ...) (RayTracer.cpp:69) ----
 * Pixels are independent and sample streams are keyed by (seed, global pixel, frame), so the image
 * is split into interleaved row bands (band b -> GPU b % n) and rendered with no communication. The
 * one exchange is an RCCL gather (ncclGather over xGMI) of every GPU's band stack to the root GPU,
 * where a kernel de-interleaves it into the full image. The result is bit-identical to one GPU.
 *
 * (1) One process driving n GPUs: rt2_tracer_create_multi (devices NULL = 0..n-1; band_h 0 = 2),
 *     one RCCL communicator per device (ncclCommInitAll). Every rt2_tracer_* function works on it as
 *     on a one-GPU tracer; readbacks (accumulation, non_converted_pixels, pixels, pixels_async,
 *     ray_counts, copy_accum_device) return the FULL image (local_rows = height), gathering first.
 *     set_stream, set_partition and join are refused. A device listed more than once runs several
 *     partitions on one GPU with device-local copies in place of RCCL (a test configuration).
 * (2) One process per GPU (torchrun / MPI style): each process creates a one-GPU tracer; rank 0 makes
 *     an id with rt2_comm_unique_id, the caller broadcasts it, and every rank calls rt2_tracer_join
 *     (= set_partition(band_h, rank, world) + ncclCommInitRank). Readbacks stay local (the rank's
 *     bands); rt2_tracer_gather is the collective that assembles the full image on rank 0, read
 *     there with rt2_tracer_image_*.
 * rt2_tracer_gather works in both modes. It is enqueued on the tracers' streams and does not wait. */
#define RT2_UNIQUE_ID_BYTES 128
RT2_API int rt2_tracer_create_multi(const rt2_scene* scene, int n_gpus, const int* devices, int band_h,
                                    rt2_tracer** out);
RT2_API int rt2_tracer_n_gpus(const rt2_tracer* tr); /* devices of a multi tracer, else 1 */
/* rt2_tracer_create_multi's argument checks and partition, on the host only (no GPU, no RCCL): part
 * i = rank i on devices[i] renders local_rows rows of the image in bands of band_h rows (0 = 2), and
 * every part sends rows_max rows in the gather. loopback = 1 when every device is one GPU (the tests'
 * configuration: device-local copies instead of RCCL). out may be NULL (checks only). */
typedef struct {
  int device, rank, world, band_h;
  int local_rows; /* image rows this part renders */
  int rows_max;   /* rows of the largest part's band stack: what every part sends */
} rt2_part_plan;
RT2_API int rt2_multi_plan(int n_gpus, const int* devices, int band_h, int width, int height, rt2_part_plan* out,
                           int* loopback);
RT2_API int rt2_comm_unique_id(uint8_t* out, size_t cap); /* cap >= RT2_UNIQUE_ID_BYTES */
RT2_API int rt2_tracer_join(rt2_tracer* tr, const uint8_t* unique_id, int world, int rank, int band_h);
RT2_API int rt2_tracer_gather(rt2_tracer* tr);
/* Root (rank 0 / a multi tracer) after a gather: the full image, rows bottom-up, H x W. */
RT2_API int rt2_tracer_image_accumulation(rt2_tracer* tr, float* out);        /* raw float3 sums */
RT2_API int rt2_tracer_image_non_converted_pixels(rt2_tracer* tr, float* out); /* accum / frame_idx */
/* NonConvertedPixels of the gathered image enqueued on the root's stream into pinned host memory
 * (rt2_host_alloc); complete when rt2_tracer_query returns 1 or after rt2_tracer_synchronize. */
RT2_API int rt2_tracer_image_non_converted_pixels_async(rt2_tracer* tr, float* out);
RT2_API int rt2_tracer_image_pixels(rt2_tracer* tr, uint8_t* out_rgba);       /* Pixels(): RGBA8 */
/* The gather's layout, for callers that move the band stacks themselves (e.g. over another
 * collective library): every rank sends rt2_band_rows_max(height, band_h, world) rows of its band
 * stack (padding rows zero); rt2_deinterleave_host turns the rank-major stacks
 * [world][max_rows][width][channels] (what ncclGather delivers on the root) into the image
 * [height][width][channels] on the host, with the same index map as the root's de-interleave
 * kernel (rt2_layout.h BandSource). No GPU needed. */
RT2_API int rt2_band_rows_max(int height, int band_h, int world);
RT2_API int rt2_deinterleave_host(const float* stacks, float* image, int width, int height, int band_h, int world,
                                  int max_rows, int channels);
/* The RCCL and HIP runtime this process runs (the first library of each name loaded wins: under
 * PyTorch that is torch's bundled copy, in a plain C++ process the one librt2.so was linked with):
 * writes "rccl <version> <path>; hip <path>" into out. */
RT2_API int rt2_runtime_info(char* out, size_t cap);

RT2_API int rt2_tracer_enable_ray_counts(rt2_tracer* tr, int on);
RT2_API int rt2_tracer_ray_counts(rt2_tracer* tr, uint32_t* out); /* rays per local pixel */
RT2_API int rt2_tracer_enable_stats(rt2_tracer* tr, int on);      /* per-record test counters */

typedef struct {
  uint64_t rays;      /* closest-hit queries issued by RayColor (depth > 0) */
  uint64_t paths;     /* camera samples finished */
  uint64_t bvh_tests, quad_tests, sphere_tests, xform_visits, medium_tests, list_visits;
  uint64_t overflow;  /* lanes that hit the traversal-stack bound (must be 0) */
  uint64_t launches;
  /* render-kernel GPU time: the time in which at least one render launch ran, each launch timed by
   * its own clock from its first wave's start to its last wave's end (queue time excluded;
   * consecutive launches overlap in the previous launch's tail, counted once) */
  double kernel_ms;
  uint64_t stamps[4]; /* diagnostic builds only: s_memtime sums (fetch, trace, shade, finish) */
  uint64_t diag[8];   /* diagnostic builds only: per-wave traversal step counts */
  /* multi-GPU (root): gathers done, and the sum of their root-stream durations (HIP events from the
   * root's last render kernel to the de-interleaved image; waiting for the slowest GPU included).
   * For a multi-GPU tracer the counters above are sums over its GPUs, except launches (per GPU)
   * and kernel_ms (the largest per-GPU sum). */
  uint64_t gathers;
  double gather_ms;
  /* host time spent enqueueing renders (a multi-GPU tracer: sum over its GPUs); image readbacks to
   * the host (rt2_tracer_image_*) on the root and their device-to-host copy time */
  double enqueue_ms;
  uint64_t readbacks;
  double readback_ms;
  /* times the library blocked the host on the GPU (stream / event synchronizations); the launch path
   * (Render, flush, gather, the async readbacks) adds none */
  uint64_t host_waits;
  /* the sum of the render launches' first-wave-to-last-wave times (>= kernel_ms: overlaps counted
   * once per launch) */
  double launch_ms_sum;
  /* device memory: both launch slots' per-frame sample buffers now (<= the sample budget), and the
   * high-water mark of everything this tracer holds on its GPU (scene program, frame buffers, sample
   * buffers, chunk tables, a root's gathered image). A multi-GPU tracer: the largest GPU's. */
  uint64_t sample_buffer_bytes;
  uint64_t device_bytes_peak;
  /* stats mode, the box-level test of MakeBox runs (sphere scenes): lanes tested and certified (the others
   * fall back to the six-face run), wave visits of a flagged run and those in which the wave ran the six
   * faces for its uncertified lanes */
  uint64_t box_tests, box_certified, box_wave_visits, box_wave_runs;
} rt2_stats;
RT2_API int rt2_tracer_get_stats(rt2_tracer* tr, rt2_stats* out);
/* The stats of GPU `part` of a multi-GPU tracer (part 0 of a one-GPU tracer is itself). */
RT2_API int rt2_tracer_part_stats(rt2_tracer* tr, int part, rt2_stats* out);
RT2_API int rt2_tracer_reset_stats(rt2_tracer* tr);

/* Diagnostic: checks the kernel's exact arithmetic shortcuts against their reference form on n
 * random inputs on `device` (which 0: division by a correctly rounded reciprocal, accepted quad
 * distances; which 1: the NaN-free slab test; which 2: reciprocal and square root without range
 * scaling; which 3: division by a correctly rounded reciprocal over any quotient, numerators down to
 * 2^-100; which 4: the accelerated-list padded slab test culls no box the exact padded slab accepts,
 * zero direction components included; which 5: the reciprocal without range scaling for every float
 * bit pattern below n, n = 2^32 for all of them; which 6: division by a correctly rounded reciprocal
 * for the first n pairs of significands, n = 2^46 for all of them; which 7: the same for every
 * numerator significand against n / 2^23 divisor significands each; which 8: sphere roots by the
 * reciprocal against IEEE division on rays from near a sphere's surface, `checked` = the admitted
 * inputs whose smaller numerator cancelled; which 9: the square root without range scaling at the
 * samplers' inputs for every 24-bit uniform, n = 2^24). Writes the number of mismatches and of inputs checked. */
RT2_API int rt2_selftest(int device, int which, uint64_t n, uint64_t seed, uint64_t* mismatches, uint64_t* checked);

/* ---- util::WriteImage (Util.cpp:39-79): sqrt gamma, clamp(x*255.999), vertical flip ---- */
RT2_API int rt2_write_image(const float* pixels, int width, int height, const char* path, int png);

#ifdef __cplusplus
}
#endif

#endif /* RT2_H_ */
