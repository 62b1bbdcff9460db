/*
 * rt_mi355x.h — C-ABI boundary of the MI355X path tracer (librt_mi355x.so).
 *
 * Plain C: pointers, sizes and the byte-exact structs of rt_abi.h. No torch, no
 * HIP types in the signatures (streams travel as void*).
 *
 * What each entry point replaces in the reference (water-chika/ray-tracing-gpu-vulkan):
 *
 *   ray_trace()              src/ray_trace.h:5-15 / src/ray_trace.cpp:922-972 — same symbol and
 *                            signature; headless, renders once, honours `storeRenderResult`
 *                            (the reference accepts but ignores it, src/ray_trace.cpp:928) and
 *                            RETURNS (the reference loops until its window closes, :88/:567).
 *   rt_generate_scene()      src/scene.h:79-157 generateRandomScene(), with the wall-clock time
 *                            (:82-83) made an explicit argument and the 22x22 grid generalised to
 *                            a (2K)x(2K) grid (K = 11 is the reference scene; K = 158 is config 5).
 *   rt_canonical_render_call_info()
 *                            the RenderCallInfo the reference fills per frame,
 *                            src/ray_trace.cpp:660-676 (number 0, camera (13,11,-3) -> origin).
 *   rt_context_create() + rt_set_scene()
 *                            the per-frame scene upload + acceleration-structure build:
 *                            AABBs src/ray_trace.cpp:583-599, BLAS src/vulkan.h:395-453,
 *                            TLAS src/vulkan.h:463-554, rebuild src/vulkan.h:1020-1059,
 *                            UBO upload src/vulkan.h:1239-1254.
 *   rt_render_device()       the per-frame GPU work of one device: clear accumulator
 *                            (src/vulkan.h:1061-1106) + vkCmdTraceRaysKHR(W, band_h, 1)
 *                            (src/vulkan.h:994-995) executing shaders/shader.{rgen,rint,rchit,rmiss}.
 *                            Device pointers, caller's stream, asynchronous.
 *   rt_multi_*()             one process driving N devices (src/ray_trace.cpp:42-105 creates one
 *                            Vulkan device per GPU, :74-93 splits the image into bands): one RCCL
 *                            communicator over the devices (ncclCommInitAll; none for one device,
 *                            whose frame has no collective), the image tiled into row-exact
 *                            interleaved 8-row strips, every device's rows gathered to
 *                            device 0 over xGMI (grouped ncclSend/ncclRecv) and reordered there,
 *                            the rows re-dealt from measured device times between frames.
 *   rt_partition_*()         the row split and its re-deal (src/ray_trace.cpp:74-81 band extents,
 *                            src/workload_tuner.hpp:38-104 get_workload fed by the per-GPU frame
 *                            times of src/ray_trace.cpp:750-762), host only, for callers that run
 *                            one process per GPU (rtvk/dist.py).
 *   rt_render()              host-pointer convenience wrapper (one call = one frame); rci_count > 1
 *                            renders one band per GPU like src/ray_trace.cpp:74-93, gathered by RCCL.
 *
 * Error model: every rt_* call returns RT_OK (0) or a negative rt_status; the message of the
 * calling thread's last failure is rt_last_error(). Exceptions never cross this boundary (the
 * reference lets C++ exceptions escape its extern "C" function). ray_trace() has
 * no return value in the reference; it prints the error to stderr, as src/main.cpp:61-63 does.
 *
 * Threading: a context is thread-compatible (one call at a time per context); distinct contexts
 * may be used concurrently from distinct threads.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stdbool.h>
#include <stdint.h>
#include "rt_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 2u

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARGUMENT = -1,
    RT_ERR_DEVICE = -2,       /* a HIP runtime call failed                         */
    RT_ERR_OUT_OF_MEMORY = -3,
    RT_ERR_NO_SCENE = -4,     /* rt_render_device() before rt_set_scene()          */
    RT_ERR_IO = -5,           /* image store failed                                */
    RT_ERR_NO_DEVICE = -6     /* no HIP device visible                             */
} rt_status;

/* Per-pixel seed coordinates. */
typedef enum rt_seed_mode {
    RT_SEED_GLOBAL = 0,        /* seed = TEA(TEA(x_global, y_global), number): image independent of GPU count */
    RT_SEED_LAUNCH_LOCAL = 1   /* seed = TEA(TEA(launchID.x, launchID.y), number): shader.rgen:40 verbatim  */
} rt_seed_mode;

/* Random stream layout. */
typedef enum rt_rng_mode {
    RT_RNG_PIXEL_STREAM = 0,   /* reference: one LCG stream per pixel runs through every sample (random.glsl)   */
    RT_RNG_SAMPLE_COUNTER = 1, /* counter-based: sample s of a pixel starts at TEA(pixel_seed, s): samples of a
                                  pixel are independent and may be split across launches                        */
    RT_RNG_SAMPLE_HASH = 2     /* counter-based (the north star's RNG): sample s starts its LCG at
                                  lowbias32(pixel_seed + 0x9E3779B9 * s) and per-sample colours are summed in
                                  8.24 fixed point, so the library splits a pixel's samples into chunks run
                                  by any lanes in any order with bit-identical results;
                                  samplesPerRenderCall <= 2^19. The fixed point holds a sample colour
                                  channel in [0, 1] (a NaN channel counts 0): every sample colour is a
                                  product of sphere colours and the sky (0.7, 0.8, 1), so it lies in
                                  [0, 1] exactly when every colour a sphere can return does (colors[0],
                                  and colors[1] of checkered spheres). rt_render_device refuses a scene
                                  with a colour channel outside [0, 1] in this mode
                                  (RT_ERR_INVALID_ARGUMENT) instead of clipping it; the reference sums
                                  unclamped (shader.rgen:55-59): render such scenes with
                                  RT_RNG_PIXEL_STREAM.                                                      */
} rt_rng_mode;

/* Closest-hit search structure (the reference uses the driver's BVH, src/vulkan.h:395-554). */
typedef enum rt_accel {
    RT_ACCEL_AUTO = 0,         /* LBVH                                                   */
    RT_ACCEL_BRUTE = 1,        /* every sphere per segment, sphere list from the scalar cache */
    RT_ACCEL_LBVH = 2          /* linear BVH (Morton order, Karras hierarchy)            */
} rt_accel;

typedef struct rt_options {
    uint32_t max_depth;   /* segments per sample; 0 -> 50 (shader.rgen:27)                       */
    uint32_t seed_mode;   /* rt_seed_mode                                                        */
    uint32_t rng_mode;    /* rt_rng_mode                                                         */
    uint32_t accel;       /* rt_accel                                                            */
    uint32_t accumulate;  /* 0: clear the accumulator first (src/vulkan.h:1081-1086); 1: add on top */
    uint32_t sample_base; /* counter modes only: index of this launch's first sample               */
    uint32_t reserved[2]; /* 0 for production. Diagnostics / A/B only: reserved[0] bit 0 = count box
                             and sphere tests (slower instrumented build, rt_get_stats); bit 1 =
                             recompute every segment's closest hit by the gated brute force that
                             backs the deferred AABB gate (tests);
                             reserved[1] = LBVH walk form: 0 automatic (octant node copies in LDS
                             when they fit, else one copy in LDS, else an LDS treelet over L2
                             subtrees), 6 one LDS node copy, 8 octant copies, 10 every node from
                             L2, 12 the uniform grid, 14 the uniform grid in LDS with the
                             wave-cooperative walk, 16 the uniform grid in LDS
                             with the wave-wide candidate queue */
} rt_options;

/* Statistics of the last rt_render_device() on a context (valid after its stream completes). */
typedef struct rt_stats {
    uint64_t segments;      /* traced segments (one traceRayEXT each, shader.rgen:75)              */
    uint64_t samples;       /* camera samples                                                     */
    uint64_t box_tests;     /* LBVH node-box tests (0 for brute force)                             */
    uint64_t sphere_tests;  /* ray-sphere tests (shader.rint:44-60 evaluations)                    */
} rt_stats;

typedef struct rt_context rt_context;

/* ---- library ---------------------------------------------------------------------- */
uint32_t    rt_abi_version(void);
const char* rt_last_error(void);
int         rt_device_count(int* count);

/* ---- host data API (scene.h / render_call_info.h) --------------------------------- */
/* generateRandomScene(t) with a (2K)x(2K) grid: writes 4 + 4K^2 spheres (488 for K = 11). */
int rt_generate_scene(float t, uint32_t grid_half_extent, Sphere* out, uint32_t capacity,
                      uint32_t* count);
int rt_canonical_render_call_info(uint32_t spp, uint32_t width, uint32_t height,
                                  RenderCallInfo* out);

/* ---- device API ------------------------------------------------------------------- */
int rt_context_create(int device, rt_context** out);
int rt_context_destroy(rt_context* ctx);
/* Uploads `count` spheres (host memory) and builds the closest-hit structure: a binned-SAH tree
 * built on the host for scenes of up to 1024 spheres (the cheaper walk), the parallel device
 * LBVH build (rt_build.hip) + device grid above that. RT_BVH_BUILD=gpu|sah|morton forces one
 * builder (A/B). `spheres` may be reused as soon as it returns. Launches already queued render
 * the old scene; every later launch of ctx renders the new one, on any stream. Host-built scenes
 * are built while queued launches execute and uploaded in order on `stream`. Device builds run on
 * the context's own build stream into the one of two scene arenas that no queued launch reads
 * (the one used two scenes ago, whose launches they wait for), so frame k + 1's build overlaps
 * frame k's tail; the call returns once the build's summary is back on the host (no wait for
 * queued launches) and its grid build is queued. */
int rt_set_scene(rt_context* ctx, const Sphere* spheres, uint32_t count, void* stream);
/* As rt_set_scene, spheres already in DEVICE memory, written by earlier work on `stream` (the
 * build copies them after that work; the caller may reuse them once the call returns). */
int rt_set_scene_device(rt_context* ctx, const Sphere* d_spheres, uint32_t count, void* stream);
/*
 * Per-frame update of an animated scene (the reference rebuilds BLAS/TLAS every frame,
 * src/vulkan.h:1020-1059, because spheres move with t, src/scene.h:94-111): same count, new
 * positions / radii / materials; keeps the tree topology of the last device build and refits its
 * boxes, records and padding on the device. Without a device-built tree of the same count it
 * performs a full rt_set_scene. Rendering stays exact (any topology is), only walk cost changes.
 */
int rt_refit_scene(rt_context* ctx, const Sphere* spheres, uint32_t count, void* stream);
int rt_refit_scene_device(rt_context* ctx, const Sphere* d_spheres, uint32_t count, void* stream);
/*
 * Render one band on ctx's device, asynchronously on `stream` (hipStream_t; NULL = default).
 *   rci          host pointer; rci->offset / rci->image_size / camera / spp / number as in the UBO.
 *   rows         optional DEVICE array of band_height global row indices (strip tiling across
 *                GPUs); NULL means rows rci->offset.y + [0, band_height).
 *   accum_rgba32f / out_rgba8   DEVICE arrays of band_width * band_height texels, row-major by
 *                band row (the reference's per-band storage images, bindings 3 and 0).
 *   band_width, band_height < 65536 (RT_ERR_INVALID_ARGUMENT otherwise); 0 renders nothing.
 */
int rt_render_device(rt_context* ctx, const RenderCallInfo* rci, const uint32_t* rows,
                     uint32_t band_width, uint32_t band_height, float* accum_rgba32f,
                     uint8_t* out_rgba8, const rt_options* opt, void* stream);
/* Statistics of the last completed rt_render_device (synchronises ctx's last stream). */
int rt_get_stats(rt_context* ctx, rt_stats* out);
/* Trace-kernel duration (ms, HIP events on the launch stream) of ctx's launch `back` launches
 * before its most recent one (0 = the most recent; the last 64 are kept). Waits for that launch's
 * end only, not for launches queued after it: a frame loop reads the launch of two frames ago
 * without draining its queue (the per-GPU frame times the reference's tuner reads,
 * src/ray_trace.cpp:636-644, :750-762). */
int rt_launch_ms(rt_context* ctx, uint32_t back, float* ms);
/* Per band row of the same launch (one of ctx's last 4 grid / LBVH launches; band_rows = its band
 * height), the row's share of the launch's work as its 8x8 tile-cost record estimates it (each
 * tile's longest unit chain x the sample chunks it ran in, split evenly over the tile's rows; the
 * unit is arbitrary, only ratios matter). Waits for that launch's record copy only. A context
 * copies its launches' records (two small device-to-host copies after each kernel) only from the
 * first call on, so the first call finds none (RT_ERR_INVALID_ARGUMENT); rt_multi's contexts keep
 * them from the start when it drives more than one device. */
int rt_launch_row_weights(rt_context* ctx, uint32_t back, double* weights, uint32_t band_rows);
/*
 * Scatter band rows into a full image on the device: dst_row[rows[i]] = src_row[i]
 * (the reorder after the multi-GPU gather). dst has dst_rows rows of `width`
 * texels; map entries >= dst_rows are skipped.
 */
int rt_scatter_rows(rt_context* ctx, const float* src_accum, const uint8_t* src_rgba8,
                    const uint32_t* rows, uint32_t n_rows, uint32_t width, uint32_t dst_rows,
                    float* dst_accum, uint8_t* dst_rgba8, void* stream);

/*
 * Gather full-image rows into a band on the device: dst_row[i] = src_row[rows[i]] (the inverse
 * of rt_scatter_rows: the running sums an accumulating multi-GPU frame hands each device). src
 * has src_rows rows of `width` float4 texels; map entries >= src_rows leave their band row as is.
 */
int rt_gather_rows(rt_context* ctx, const float* src_accum, const uint32_t* rows, uint32_t n_rows,
                   uint32_t width, uint32_t src_rows, float* dst_accum, void* stream);

/*
 * Tonemap a summed accumulator to rgba8 on the device, exactly as the trace kernel's store
 * (shader.rgen:65-66): rgba8 = round(clamp(sqrt(sum / spp), 0, 1) * 255) per channel, alpha 255.
 * spp 0 is accepted and gives the bytes the trace kernel stores for a 0-sample frame.
 * accum_rgba32f: n_texels float4 (DEVICE); out_rgba8: n_texels x 4 bytes (DEVICE).
 */
int rt_resolve_rgba8(rt_context* ctx, const float* accum_rgba32f, uint64_t n_texels, uint32_t spp,
                     uint8_t* out_rgba8, void* stream);

/* ---- multi-device (one process, N GPUs, RCCL over xGMI) ----------------------------- */
typedef struct rt_multi rt_multi;
/* Devices 0 .. n-1, n = min(gpu_count, visible devices) (>= 1): one context and one stream per
 * device and, for n > 1, one RCCL communicator over them (ncclCommInitAll); one device renders
 * straight into the caller's buffers and builds no communicator. */
int rt_multi_create(uint32_t gpu_count, rt_multi** out);
int rt_multi_destroy(rt_multi* m);
int rt_multi_device_count(const rt_multi* m, uint32_t* n);
/* The scene on every device (host spheres), as rt_set_scene: every device's build is issued before
 * any is waited for (device builds run on all GPUs at once), and a host-built scene is built once
 * and uploaded to every device. */
int rt_multi_set_scene(rt_multi* m, const Sphere* spheres, uint32_t count);
/*
 * One frame of the whole image rci->image_size (rci->offset ignored). The rows start as
 * rt_partition_strips' row-exact strips (device d renders its rows through rt_render_device with
 * a rows map, global seeds) and are re-dealt between frames: each frame reads every device's
 * trace-kernel time of the frame two before (rt_launch_ms), rescales per-row cost estimates to
 * them and moves band-end rows from the slowest device to the fastest (rt_partition_rebalance's
 * rule; the move rewrites rows maps only, waiting for queued frames once); every other device's
 * float4 accumulator rows travel to device 0 in one RCCL group
 * (ncclSend / ncclRecv; device 0's own strips never go through RCCL) and are reordered into
 * accum_rgba32f, then device 0 tonemaps the whole accumulator into out_rgba8 (rt_resolve_rgba8:
 * the rgba8 bytes are a function of the float sum, so they are not sent). accum_rgba32f /
 * out_rgba8: DEVICE pointers on device 0, W*H texels. Asynchronous on `stream` (a hipStream_t of
 * device 0; NULL = the legacy stream): the call returns once everything is queued. The image
 * equals the one-device image bit for bit.
 * opt->accumulate: as rt_render_device, the frame adds to what accum_rgba32f holds when the call's
 * work starts on `stream`, at every device count (device 0 sends each device the running sums of
 * its strips first). One device holding every row renders straight into the caller's buffers (no
 * strip copy, no reorder, no resolve). The frame plan is rt_debug_multi_plan's
 * (include/rt_mi355x_debug.h).
 */
int rt_multi_render(rt_multi* m, const RenderCallInfo* rci, const rt_options* opt,
                    float* accum_rgba32f, uint8_t* out_rgba8, void* stream);
/* Sum over the devices of the last frame's statistics (synchronises). */
int rt_multi_stats(rt_multi* m, rt_stats* out);
/* {devices, ranks of the RCCL communicator (ncclCommCount; 0 for one device: no communicator),
 * rows per strip, devices that rendered rows in the last frame}. */
int rt_multi_info(const rt_multi* m, uint32_t* out4);
/* Trace-kernel duration (ms, HIP events on the launch stream) of the last frame on each device
 * that rendered rows, in device order; *count = devices written (synchronises). */
int rt_multi_kernel_times(rt_multi* m, float* out_ms, uint32_t capacity, uint32_t* count);
/* The same for each of the last `frames` frames (at most 64): out_ms[f * devices + d], oldest frame
 * first; *count = frames x devices that rendered rows (synchronises). */
int rt_multi_kernel_times_frames(rt_multi* m, uint32_t frames, float* out_ms, uint32_t capacity, uint32_t* count);
/* The partition the next frame renders with: counts[d] rows on device d (n entries), and with rows
 * non-NULL (capacity >= image height) the rows, device 0's first, each device's in band order.
 * Set up by the first rt_multi_render of an image size (all counts 0 before it). */
int rt_multi_partition(const rt_multi* m, uint32_t* rows, uint32_t* counts, uint32_t capacity);

/* ---- row partition across devices (host only, no device needed) --------------------- */
/* A partition of `height` rows over n devices is rows[] (height entries: device 0's rows, then
 * device 1's, ...; each device's in band order) + counts[] (n entries).
 * rt_partition_strips: the row-exact interleaved strips every multi-device frame starts from: the
 * rows of the R = floor(height / (8 n)) full rounds are 8-row strips dealt round robin (strip k on
 * device k % n), the rest are n contiguous runs (the first (rest % n) one row longer), run d on
 * device d; every device holds floor(height / n) or ceil(height / n) rows (the reference gives the
 * remainder to the first band, src/ray_trace.cpp:74-81). */
int rt_partition_strips(uint32_t n_devices, uint32_t height, uint32_t* rows, uint32_t* counts);
/* One balancing step (src/workload_tuner.hpp:38-104, without its random moves and without the
 * teardown, src/ray_trace.cpp:774): with a measurement (meas_rows / meas_counts: the partition a
 * frame ran with, meas_ms: each device's trace-kernel ms of that frame; all three NULL for none),
 * row_cost (height doubles, ms per row; <= 0: unknown, in / out) is rescaled so that each measured
 * device's rows sum to its time (unknown rows at the mean of its known ones). Then rows / counts
 * (the current partition, in / out) are re-dealt: while the most loaded device is above
 * (1 + tolerance) x the mean load, one of its last min(8, rows) band rows moves to the end of
 * another device's band, or is swapped with one of that band's last rows, whichever exchange
 * leaves the pair's larger load lowest, as long as it lowers the most loaded device's load by
 * more than tolerance x the mean. Deterministic: every rank of a one-process-per-GPU job that calls it with
 * the same inputs gets the same partition. *moved = rows moved; *predicted_imbalance = max / mean
 * load afterwards (either may be NULL). */
int rt_partition_rebalance(uint32_t n_devices, uint32_t height, uint32_t* rows, uint32_t* counts, double* row_cost,
                           const uint32_t* meas_rows, const uint32_t* meas_counts, const float* meas_ms,
                           double tolerance, uint32_t* moved, double* predicted_imbalance);

/* ---- host-pointer convenience ------------------------------------------------------ */
/*
 * One frame over the full image rci[0].image_size with host buffers. rci_count bands, band i
 * spanning rows [rci[i].offset.y, rci[i+1].offset.y) (last band to image height), band i on
 * device i % device_count, gathered to device 0 by RCCL (rt_multi), then copied to the host. Each
 * band renders and is tonemapped with its own RenderCallInfo (its own samplesPerRenderCall, as the
 * reference fills one per GPU, src/ray_trace.cpp:660-676).
 * accum_rgba32f: W*H*4 floats (read first when opt->accumulate), out_rgba8: W*H*4 bytes.
 */
int rt_render(const Sphere* spheres, uint32_t sphere_count, const RenderCallInfo* rci,
              uint32_t rci_count, float* accum_rgba32f, uint8_t* out_rgba8,
              const rt_options* opt, rt_stats* stats);

/* Writes an rgba8 image as binary PPM (P6, alpha dropped). */
int rt_store_ppm(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height);

/* Build provenance of this library: "sources_sha256=<16 hex of the sources it was compiled
 * from>;arch=<offload arch>;flags=<compiler flags>;variant=<A/B variant flags, empty for the
 * shipped build>". Static string. */
const char* rt_build_info(void);

/* src/ray_trace.h:9-15 — identical symbol and parameter list. Renders the canonical scene once
 * (t = 0) on min(gpu_count, visible) GPUs through rt_multi (row-exact strips, RCCL gather, global
 * seeds, so the image does not depend on gpu_count), prints the frame time, stores `render.ppm`
 * when storeRenderResult, and returns. Random stream: the reference's per-pixel LCG stream, or
 * RT_RNG_SAMPLE_HASH when the environment holds RT_RNG=hash (the signature has no parameter for
 * it; any other RT_RNG value than "stream" / "hash" is reported and nothing renders). */
void ray_trace(uint32_t samples, bool storeRenderResult, uint32_t width, uint32_t height,
               uint32_t gpu_count);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* RT_MI355X_H */
