/*
 * rt_mi355x_debug.h — diagnostic and A/B entry points of librt_mi355x.so.
 *
 * Not part of the drop-in boundary (include/rt_mi355x.h is what replaces src/ray_trace.h): the
 * same library exports these for the test suite, bench.py and the A/B scripts (instrumented
 * counters, per-launch timing, launch-plan tuning, the multi-GPU frame plan). Production callers
 * never need them; none of them changes an image.
 */
#ifndef RT_MI355X_DEBUG_H
#define RT_MI355X_DEBUG_H

#include "rt_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic (tests only): evaluates one arithmetic-contract primitive on `device` for n
 * (x, y) pairs: op 0 sqrt(x), 1 x/y, 2 sin(x), 3 fma(x,y,1), 4 normalize(x,y,0.5).x, 5 pow(x,5),
 * 6 sample_seed_hash(bits(x), bits(y)) as bits, 7 / 8 low / high word of the 8.24 fixed-point
 * value of colour x, as bits, 9 checker decision at (x, y, 0.5 (x - y)) as 1 / 0. */
int rt_debug_math(int device, int op, const float* in_pairs, float* out, uint32_t n);
/* Diagnostic (tests only): the kernels' cheap correctly rounded operations against hipcc's
 * correctly rounded ones on `device`: rcp_cr(x) vs 1.0f / x and sqrt_cr(x) vs sqrtf(x) over all 2^32
 * binary32 inputs (mismatches3[0], [1]; NaN == NaN), and the camera's float(double(x) * (1 /
 * double(b))) vs x / b for every binary32 x in [0, 65536) and eleven image sizes b (mismatches3[2]). */
int rt_debug_exact_exhaustive(int device, uint64_t* mismatches3);
/* Durations (ms) of the trace kernel of ctx's most recent launches (at most 64 are kept), oldest
 * first, from HIP events recorded on the launch stream around the kernel itself (not the resolve):
 * a caller times K launches inside its own timed region and reads them afterwards. *count =
 * min(capacity, launches kept). Synchronises on those events. */
int rt_debug_kernel_times(rt_context* ctx, float* out_ms, uint32_t capacity, uint32_t* count);
/* Diagnostic (tests, A/B timing): sets one launch-plan parameter of ctx (value -1 restores the
 * default). None of them changes an image; the defaults are the measured best. Keys: "grid" (0: no
 * uniform grid), "grid_scale", "grid_coop" (1: wave-cooperative grid walk), "grid_cq" (1: wave-wide
 * candidate queue), "grid_rec" (0: no
 * shading records in LDS), "grid_full_slack", "units_per_lane", "unit_min_samples",
 * "sample_chunks", "head_chunks", "tail_tiles_pm", "schedule" (0 LPT, 1 row-major, 2 LPT by tile
 * sum), "refill_reserve", "isolate_tiles", "sah_knobs". Unknown keys: RT_ERR_INVALID_ARGUMENT.
 * Scene-build keys (grid, grid_scale, sah_knobs) apply from the next rt_set_scene. The library
 * reads no environment variable for any of them. */
int rt_debug_tune(rt_context* ctx, const char* key, double value);
/* Diagnostic: of ctx's last launch, {sample chunks per pixel (low 16 bits: of the LPT order's tail
 * tiles; high 16 bits: of its head tiles, 0 when the launch had no head), the kernel form it ran
 * (low 16 bits: rt_internal.h ACCEL_*, before any launch the scene's default form; bit 16: its
 * grid walk was the one-layer form, the grid one cell thick in y; bit 17: its camera rays started
 * at the camera position itself, the pinhole shortcut), its dynamic LDS bytes, CU count}. */
int rt_debug_launch_info(rt_context* ctx, uint32_t* out4);
/* Diagnostic: per-phase cycle sums of ctx's last launch, filled only by -DRT_STAMPS builds. */
int rt_debug_stamps(rt_context* ctx, uint64_t* out8);
/* Diagnostic: lane utilisation of ctx's last launch per kernel code point k (0..15), filled only by
 * -DRT_UTIL builds: out32[2k] wave passes through the point, out32[2k + 1] active lanes summed. */
int rt_debug_util(rt_context* ctx, uint64_t* out32);
/* Diagnostic: histogram of LBVH box tests per segment of the last instrumented launch
 * (options.reserved[0] & 1), 2 x 64 bins: [0] segments that miss, [1] segments that hit. */
int rt_debug_walk_hist(rt_context* ctx, uint64_t* out128);
/* Diagnostic: walk work (cells + references) of ctx's last instrumented launch per segment pass,
   max over the wave's tracing lanes [0] and over its bounce (depth > 0) lanes [1], summed over
   passes; the primary (depth 0) lanes' summed work [2] and their count [3]. */
int rt_debug_walk_split(rt_context* ctx, uint64_t* out4);
/* Diagnostic: of ctx's last instrumented launch of a grid walk, {cells visited, visited cells that
 * hold no reference}. */
int rt_debug_grid_cells(rt_context* ctx, uint64_t* out2);
/* Diagnostic: segment-loop iterations of the last instrumented launch by the number of lanes
 * (0..64) of the wave tracing in that iteration (the persistent kernel's lane occupancy), then
 * three s_memrealtime stamps (100 MHz): first wave start, pixel queue dry, last wave exit. */
int rt_debug_lane_hist(rt_context* ctx, uint64_t* out68);
/* Diagnostic: tail steals of ctx's last instrumented launch (options.reserved[0] & 1;
 * RT_RNG_SAMPLE_HASH: once the work queue is empty, an idle lane takes half of the samples its
 * wave's busiest lane has not started). */
int rt_debug_steals(rt_context* ctx, uint64_t* out);
/* Diagnostic: per 8x8 tile of ctx's last LBVH launch, the traced segments of its most expensive
 * pixel (the key its next launch over the same band geometry hands tiles out by, longest
 * first); *count = tiles (ceil(W/8) x ceil(H/8), row-major), 0 before the first launch. */
int rt_debug_tile_cost(rt_context* ctx, uint32_t* out, uint64_t capacity, uint64_t* count);

/* Diagnostic (tests): copies one scene array of ctx to host memory. what: 0 geometry records,
 * 1 radii, 2 material records, 3 big-sphere ids, 4 LBVH nodes (padded), 5 LBVH nodes (unpadded),
 * 6 leaf geometry, 7 leaf ids, 8 info {u32 n_spheres, n_big, n_nodes, n_leaf_slots,
 * device_built, 0; f32 small_rmax, scene_radius}, 9 grid {u32 cells in x, y, z, cells, references}
 * (zeros without a grid). *bytes = the array's size; RT_ERR_INVALID_ARGUMENT when it exceeds
 * capacity. */
int rt_debug_scene(rt_context* ctx, uint32_t what, void* out, uint64_t capacity, uint64_t* bytes);

/*
 * The multi-device frame plan rt_multi_render (band_starts NULL: its first frame's row-exact strips,
 * rt_partition_strips) or rt_render (band i = rows [band_starts[i], band_starts[i+1]) on device
 * i % n_devices) executes for a width x height frame, with or without accumulation. Host only (no
 * device needed). Flat u32 form: {n_parts, n_steps}, per part {device, whole, n_rows, rows...},
 * per step {op, device, peer, part, flags, count low, count high}; ops 1 load rows (device 0:
 * caller accumulator -> part buffer), 2 RCCL group start, 3 send, 4 receive, 5 group end,
 * 6 render (flags bit 0: straight into the caller's buffers), 7 store rows (part buffer -> caller
 * accumulator), 8 resolve rgba8 (count texels); send / receive counts are floats. out NULL: size
 * query (*count = words).
 */
int rt_debug_multi_plan(uint32_t n_devices, uint32_t width, uint32_t height, const uint32_t* band_starts,
                        uint32_t n_bands, uint32_t accumulate, uint32_t* out, uint64_t capacity,
                        uint64_t* count);
/* The same plan for an explicit partition (rows / counts as rt_partition_strips writes them: every
 * row of [0, height) exactly once), e.g. one the balancer re-dealt. */
int rt_debug_multi_plan_rows(uint32_t n_devices, uint32_t width, uint32_t height, const uint32_t* rows,
                             const uint32_t* counts, uint32_t accumulate, uint32_t* out, uint64_t capacity,
                             uint64_t* count);
/* Tests on a one-GPU box: an rt_multi of n_devices LOGICAL devices, all on device 0 (one context
 * and one stream each), executing the same frame plans as rt_multi_create's, with every RCCL
 * send / receive pair of a group replaced by one device copy on the receiver's stream, ordered
 * after the sender's earlier work and before its later work (the group boundaries of the plan).
 * No communicator (rt_multi_info reports 0 ranks). */
int rt_debug_multi_create_logical(uint32_t n_devices, rt_multi** out);
/* The same logical devices with the transfers through RCCL itself: one communicator of one rank on
 * device 0 (ncclCommInitAll), every group's sends and receives issued as ncclSend / ncclRecv of
 * rank 0 to itself on logical device 0's stream (fenced by events against every logical device's
 * stream before and after the group), so the one-GPU pool runs rt_multi's RCCL branch: the
 * communicator, the grouped calls and their buffers (rt_multi_info reports 1 rank). */
int rt_debug_multi_create_logical_rccl(uint32_t n_devices, rt_multi** out);
/* The balancer of m's strip frames: "balance" (1 on, 0 off), "tolerance" (re-deal above
 * (1 + tolerance) x the mean device time, by exchanges that gain more than tolerance x the mean;
 * default 0.001), "blend" (weight in (0, 1] of a new measurement in the per-row estimates, above 1
 * taken as 1; default 0.5), "lag" (frames between the measured frame and the one it re-deals, 1 to
 * 8; default 2); -1 restores the default. Other values: RT_ERR_INVALID_ARGUMENT. */
int rt_debug_multi_tune(rt_multi* m, const char* key, double value);
/* Feeds n device times (ms) as if measured on the current partition: the next rt_multi_render
 * re-deals from them instead of its own measurement (tests: forced re-deals). */
int rt_debug_multi_feedback(rt_multi* m, const float* device_ms, uint32_t n);
/* {strip frames rendered since the partition was set up, re-deals, rows moved, predicted max / mean
 * device time after the last re-deal}. */
int rt_debug_multi_balance_info(const rt_multi* m, double* out4);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* RT_MI355X_DEBUG_H */
