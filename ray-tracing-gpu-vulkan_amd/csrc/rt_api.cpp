// rt_api.cpp — host runtime behind the C-ABI (include/rt_mi355x.h), one device context at a time.
//
// Replaces the reference's host orchestration for the hot path (src/ray_trace.cpp:42-972,
// src/vulkan.h): device contexts instead of Vulkan devices, one HBM-resident scene + LBVH per
// context instead of UBO + BLAS/TLAS, one fused persistent kernel launch per band instead of
// clear + vkCmdTraceRaysKHR. The multi-device frame (RCCL) and ray_trace() are in rt_multi.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <random>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rt_abi.h"
#include "../../include/rt_mi355x.h"
#include "../../include/rt_mi355x_debug.h"
#include "rt_build.h"
#include "rt_bvh.h"
#include "rt_grid.h"
#include "rt_host.h"
#include "rt_internal.h"

namespace rt {
hipError_t launch_trace(const TraceParams& P, uint32_t accel, bool count, int mode, int grid, size_t lds_bytes,
                        hipStream_t st);
hipError_t trace_occupancy(uint32_t accel, bool count, int mode, bool flat, size_t lds_bytes, int* blocks_per_cu);
bool flat_grid_form(const TraceParams& P, uint32_t accel, bool count);
hipError_t launch_resolve_fixed(unsigned long long* fixed, uint64_t n_texels, uint32_t accumulate, uint32_t spp,
                                float* accum, uint8_t* out, hipStream_t st);
hipError_t launch_tonemap(const float* accum, uint64_t n_texels, uint32_t spp, uint8_t* out, hipStream_t st);
hipError_t launch_prep(const TraceParams& P, uint32_t work_head, float* tab, uint32_t n_cost, hipStream_t st);
uint32_t block_size(uint32_t accel);
hipError_t launch_scatter_rows(const float* src_acc, const uint8_t* src_px, const uint32_t* rows,
                               uint32_t n_rows, uint32_t width, uint32_t dst_rows, float* dst_acc, uint8_t* dst_px,
                               hipStream_t st);
hipError_t launch_gather_rows(const float* src_acc, const uint32_t* rows, uint32_t n_rows, uint32_t width,
                              uint32_t src_rows, float* dst_acc, hipStream_t st);
hipError_t launch_debug_math(int op, const float* in, float* out, uint32_t n, hipStream_t st);
hipError_t launch_debug_exact(unsigned long long* bad, hipStream_t st);
}  // namespace rt

// Launch-plan parameters that tests and A/B scripts vary through rt_debug_tune() (per context; the
// shipped defaults are the measured best). None changes an image. The library reads
// no environment variable for them: only RT_RNG (ray_trace) and RT_BVH_BUILD are read, both
// documented.
struct Tuning {
    static constexpr double kUnset = -1.0;
    double grid = kUnset;               // 0: no uniform grid (LBVH walks only)
    double grid_scale = kUnset;         // cell size scale (rt_grid.h kGridCellScale)
    double grid_coop = kUnset;          // 1: the wave-cooperative grid walk
    double grid_cq = kUnset;            // 1: the wave-wide candidate queue in the LDS grid walk (§4.9)
    double grid_rec = kUnset;           // 0: no shading records in the LDS grid kernel's LDS
    double grid_full_slack = kUnset;    // 1: the full cull slack in grid walks
    double units_per_lane = kUnset;     // sample-chunk targets (counter-based stream)
    double unit_min_samples = kUnset;
    double sample_chunks = kUnset;      // forced chunk count (tail count when the LPT order is split)
    double head_chunks = kUnset;        // head / tail split of the LPT order
    double tail_tiles_pm = kUnset;
    double schedule = kUnset;           // 0 LPT (longest unit chain), 1 row-major
    double refill_reserve = kUnset;     // units handed out one by one at the end of the queue
    double isolate_tiles = kUnset;      // reference stream: waves on the first LPT blocks take no more
    double sah_knobs = kUnset;          // host SAH builder variants (rt_bvh.h)
    static double get(double v, double def) { return v == kUnset ? def : v; }
};

// One arena of device-built scenes (rt_context::slot; rt_api.cpp device_build_begin).
struct SceneSlot {
    rt::DeviceScene scene;            // its arrays (pointers into mem / grid_mem) and counts
    void* mem = nullptr;              // every per-sphere array of the build, one allocation
    uint32_t cap_n = 0;               // spheres it holds
    void* grid_mem = nullptr;         // cell offsets, fill cursor, references, ids, scan scratch
    size_t grid_cap = 0;              // bytes
    hipEvent_t ev_free = nullptr;     // recorded after every launch that reads this arena
    bool used = false;                // ev_free has been recorded
};

struct rt_context {
    int device = 0;
    Tuning tune;
    int cu_count = 0;
    rt::DeviceScene scene;                       // the current scene (host blob or an arena)
    bool scene_set = false;                      // a set/refit call has succeeded (RT_ERR_NO_SCENE)
    // device-built scenes: two arenas used alternately, built on the context's own stream
    SceneSlot slot[2];
    int slot_cur = -1;                           // arena of the current scene (-1: host-built / none)
    hipStream_t build_stream = nullptr;
    hipEvent_t ev_summary = nullptr;             // the build's summary has reached pinned memory
    hipEvent_t ev_caller = nullptr;              // device spheres: the caller's stream reached the call
    rt::BuildSummary* summary = nullptr;         // pinned
    void* sph_stage = nullptr;                   // pinned staging of host spheres
    size_t sph_stage_cap = 0;
    bool pending = false;                        // a build begun, not yet ended (rt_multi_set_scene)
    int pending_slot = 0;
    uint32_t pending_count = 0;
    rt::Counters* counters = nullptr;            // device
    float* big_tab = nullptr;                    // device, in the counters' allocation (TraceParams::big_tab)
    // Every device operation of a context (scene upload / build, render) is ordered after the
    // previous one, whatever streams they are issued on: an op on a stream other than the last
    // one first waits for `ev_last`, and every op records it when issued. A device build runs on
    // the build stream beside the previous op (it waits only for the launches that read its
    // arena), so it does not cover that op: the op's event moves to `ev_prev`,
    // which the next op waits for as well (order_on) until an op issued after both clears it.
    hipStream_t last_stream = nullptr;
    hipEvent_t ev_last = nullptr;
    bool ev_valid = false;
    hipStream_t prev_stream = nullptr;
    hipEvent_t ev_prev = nullptr;
    bool prev_valid = false;
    // the build workspace (ws) holds the topology of a full build that completed: a refit may
    // reuse it (a full build that failed after overwriting ws leaves it false)
    bool topo_ok = false;
    bool pending_refit = false;
    // occupancy cache per kernel form, count flag and rng mode, valid for occ_lds bytes
    int occ[rt::ACCEL_COUNT][3][2] = {};   // [form][plain, count_tests, one-layer grid walk][mode]
    size_t occ_lds[rt::ACCEL_COUNT][3][2] = {};
    size_t lds1_bytes = 0;                       // one node copy + leaves + big table (0: no fit)
    size_t oct_bytes = 0;                        // 8 octant node copies + leaves + big table (0: no fit)
    size_t grid_bytes = 0;                       // grid references + offsets + big table (0: no grid / no fit)
    bool has_grid = false;                       // the scene has a grid (staged in LDS when grid_bytes)
    float grid_pad_radius = 0.0f;                // camera radius the grid's margin covers
    // unpadded LBVH node boxes (host) and the radius the device copy is padded for
    std::vector<rt::BvhNode> nodes_host;
    float scene_radius = 0.0f;
    float pad_radius = 0.0f;
    float padded_for = 0.0f;                     // pad radius the device node copy currently carries
    bool gpu_tree = false;
    bool treelet_stale = true;                   // ACCEL_LBVH_TOP: the treelet predates the node boxes
    rt::TileSchedule sched;                      // unit hand-out order (LPT from the last launch's costs)
    rt::BuildWorkspace ws;                       // device build scratch, kept for refits
    Sphere* d_spheres = nullptr;                 // staging copy of host-provided spheres (device build)
    uint32_t d_spheres_cap = 0;
    // Host-built scenes: every device array lives in one device blob, rewritten in stream order
    // by one copy from a pinned staging buffer (two, alternating, each guarded by the event of
    // its last copy), so rt_set_scene builds the next frame's tree on the host while the
    // previous frame still renders (no device-wide sync, no per-frame hipMalloc/hipFree).
    void* blob = nullptr;
    size_t blob_cap = 0;
    void* stage[2] = {nullptr, nullptr};
    size_t stage_cap[2] = {0, 0};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    bool stage_used[2] = {false, false};
    int stage_cur = 0;
    // RT_RNG_SAMPLE_HASH: 3 planes of fixed-point sums, zero between launches (the resolve
    // kernel clears what it reads)
    unsigned long long* fixed = nullptr;
    uint64_t fixed_cap = 0;                      // texels
    uint32_t last_chunks = 1;
    uint32_t last_accel = 0;                     // kernel form (rt::ACCEL_*) of the last launch, 0 = none yet
    size_t last_lds = 0;                         // its dynamic LDS bytes
    bool last_flat = false;                      // its grid walk was the one-layer form
    bool last_pinhole = false;                   // its camera rays started at lf (TraceParams::pinhole_lf)
    // every colour the shaders can return lies in [0, 1] (RT_RNG_SAMPLE_HASH's fixed point needs it)
    bool colours_unit = true;
    // HIP events bracketing the trace kernel of the last kKernelEvents launches (ring; timing
    // inside a caller's timed region without a host sync per launch, rt_debug_kernel_times)
    static constexpr uint32_t kKernelEvents = 64;
    hipEvent_t kev[kKernelEvents][2] = {};
    uint64_t kev_count = 0;                      // launches recorded so far
    // Host copies of the last launches' tile-cost records (and the LPT order they ran in), copied
    // after the kernel on the launch stream: the cross-device balancer reads a launch's per-row
    // work from them two frames later without a wait on queued work (rt_launch_row_weights).
    struct CostSnap {
        uint32_t* host = nullptr;                // pinned: cost[n], then order[n] when has_order
        uint32_t cap = 0;                        // tiles it holds
        hipEvent_t ev = nullptr;                 // after the copies
        bool pending = false;
        uint64_t launch = ~0ull;                 // launch index the record belongs to
        uint32_t n = 0, tiles_x = 0, band_h = 0, head_tiles = 0, head_chunks = 1, chunks = 1;
        bool has_order = false;
    };
    static constexpr uint32_t kSnaps = 4;
    CostSnap snap[kSnaps];
    bool keep_snaps = false;   // set by the first rt_launch_row_weights (or rt_multi at N > 1):
                               // a one-device frame loop pays no copies it never reads
};

namespace {
// Node boxes grow by 12u * R (u = 2^-24): the one-fma slab form of the walk differs from the
// exact form of the AABB gate by at most u|o| + 5u(|bound| + |o|) in distance along each axis
// for |o|, |bound| <= R; 1.5x margin.
float pad_for(float R) { return 18.0f * 5.9604645e-8f * R; }

void pad_nodes(const std::vector<rt::BvhNode>& in, std::vector<rt::BvhNode>& out, float pad) {
    out = in;
    for (auto& n : out) {
        n.lox -= pad; n.loy -= pad; n.loz -= pad;
        n.hix += pad; n.hiy += pad; n.hiz += pad;
    }
}

// Eight re-orderings of an escape-link tree, one per ray direction octant (bit k of the octant:
// axis k runs negative): each copy lists the nearer child of every inner node first, "nearer"
// meaning lower along the axis that best separates the two child boxes when the octant runs
// positive on it (higher when negative). The walk of a ray then reaches close spheres early, so
// its cull limit shrinks sooner. Escape links are re-derived per copy; leaves keep their slots.
void make_octant_orders(const std::vector<rt::BvhNode>& n, std::vector<rt::BvhNode>& out) {
    const uint32_t N = uint32_t(n.size());
    out.assign(size_t(8) * N, rt::BvhNode{});
    if (N == 0) return;
    std::vector<uint32_t> size(N, 1);   // nodes in the subtree rooted at i (children follow i)
    for (uint32_t i = N; i-- > 0;)
        if (n[i].first_count == 0) size[i] = 1 + size[i + 1] + size[n[i + 1].escape];
    for (uint32_t o = 0; o < 8; ++o) {
        rt::BvhNode* dst = out.data() + size_t(o) * N;
        uint32_t next = 0;
        // (node, escape in the new order), depth-first
        std::vector<std::pair<uint32_t, uint32_t>> stack{{0u, 0xffffffffu}};
        while (!stack.empty()) {
            const auto [i, esc] = stack.back();
            stack.pop_back();
            const uint32_t at = next++;
            dst[at] = n[i];
            dst[at].escape = esc;
            if (n[i].first_count != 0) continue;
            const uint32_t L = i + 1, R = n[L].escape;
            float best = -1.0f;
            int axis = 0;
            const float cl[3] = {n[L].lox + n[L].hix, n[L].loy + n[L].hiy, n[L].loz + n[L].hiz};
            const float cr[3] = {n[R].lox + n[R].hix, n[R].loy + n[R].hiy, n[R].loz + n[R].hiz};
            for (int k = 0; k < 3; ++k)
                if (std::fabs(cl[k] - cr[k]) > best) { best = std::fabs(cl[k] - cr[k]); axis = k; }
            const bool neg = (o >> axis) & 1u;
            const bool l_first = neg ? cl[axis] >= cr[axis] : cl[axis] <= cr[axis];
            const uint32_t a = l_first ? L : R, b = l_first ? R : L;
            // a is emitted at `at + 1`, b right after a's subtree; b inherits this node's escape
            stack.push_back({b, esc});
            stack.push_back({a, at + 1 + size[a]});
        }
    }
}

// LDS budget of the staged forms: 160 KiB per CU, one 1024-thread block per CU; 4 KiB kept free.
constexpr size_t kMaxLdsBytes = 156 * 1024;
// ... and of a form that must keep two 768-thread blocks per CU (static + dynamic LDS).
constexpr size_t kTwoBlockLdsBytes = 78 * 1024;
// The LDS walk's leaf words hold a leaf index in 10 bits (<= 4096 slots of 4) and an escape node
// of the 8 copies in 19 bits.
constexpr uint32_t kMaxLdsLeafSlots = 4096;
constexpr uint32_t kMaxLdsNodes = 0x7fffeu / 8u;

void size_lds_forms(rt_context* ctx) {
    const rt::DeviceScene& d = ctx->scene;
    const size_t tree = size_t(2 * d.n_nodes + d.n_leaf + (d.n_leaf + 3) / 4) * 16;
    const size_t lds1 = tree;   // shading records stay in HBM (rt_kernels.hip)
    const bool ok = d.n_nodes && d.n_leaf <= kMaxLdsLeafSlots && d.n_nodes <= kMaxLdsNodes;
    ctx->lds1_bytes = (ok && lds1 <= kMaxLdsBytes) ? lds1 : 0;
    const size_t oct = lds1 + size_t(14u) * d.n_nodes * 16u;
    ctx->oct_bytes = (ok && oct <= kMaxLdsBytes) ? oct : 0;
    const rt::GridInfo& g = d.grid;
    const size_t grid = (size_t(g.n_refs) + (g.n_refs + 3) / 4 + (size_t(g.n_cells) + 4) / 4) * 16;
    ctx->grid_bytes = (g.n_refs && grid + rt::kLaneSumLdsBytes <= kMaxLdsBytes) ? grid : 0;
}


// Stream chaining of a context's device operations (rt_context::ev_last).
int order_on(rt_context* ctx, hipStream_t st) {
    if (ctx->ev_valid && ctx->last_stream != st) RT_HIP(hipStreamWaitEvent(st, ctx->ev_last, 0));
    if (ctx->prev_valid && ctx->prev_stream != st) RT_HIP(hipStreamWaitEvent(st, ctx->ev_prev, 0));
    return RT_OK;
}
// After an op issued on `st` behind order_on(ctx, st): it follows everything before it.
int mark_issued(rt_context* ctx, hipStream_t st) {
    if (!ctx->ev_last) RT_HIP(hipEventCreateWithFlags(&ctx->ev_last, hipEventDisableTiming));
    RT_HIP(hipEventRecord(ctx->ev_last, st));
    ctx->ev_valid = true;
    ctx->last_stream = st;
    ctx->prev_valid = false;
    return RT_OK;
}
// After a device build on the build stream, which did not wait for the previous op: the build's
// event becomes ev_last and the previous op's event is kept in ev_prev (unless the previous op
// was itself a build, whose own ev_prev then still stands).
int mark_built(rt_context* ctx) {
    if (ctx->ev_valid && ctx->last_stream != ctx->build_stream) {
        std::swap(ctx->ev_last, ctx->ev_prev);
        ctx->prev_valid = true;
        ctx->prev_stream = ctx->last_stream;
    }
    if (!ctx->ev_last) RT_HIP(hipEventCreateWithFlags(&ctx->ev_last, hipEventDisableTiming));
    RT_HIP(hipEventRecord(ctx->ev_last, ctx->build_stream));
    ctx->ev_valid = true;
    ctx->last_stream = ctx->build_stream;
    return RT_OK;
}
// Host wait for every op issued so far (statistics and diagnostic readers).
int sync_issued(rt_context* ctx) {
    if (ctx->ev_valid) RT_HIP(hipEventSynchronize(ctx->ev_last));
    if (ctx->prev_valid) RT_HIP(hipEventSynchronize(ctx->ev_prev));
    return RT_OK;
}

// One device blob for a host-built scene (rt_context::blob): add() the arrays, then commit()
// packs them into a pinned staging buffer and issues one stream-ordered copy.
class BlobUpload {
  public:
    template <typename T>
    void add(const std::vector<T>& v, T** dst) {
        *dst = nullptr;
        if (v.empty()) return;
        parts_.push_back(Part{v.data(), v.size() * sizeof(T), total_, reinterpret_cast<void**>(dst)});
        total_ += (v.size() * sizeof(T) + 255u) & ~size_t(255);
    }
    int commit(rt_context* ctx, hipStream_t st) {
        if (total_ == 0) return RT_OK;
        const int k = ctx->stage_cur;
        if (ctx->stage_used[k]) RT_HIP(hipEventSynchronize(ctx->stage_ev[k]));   // its last copy is done
        if (ctx->stage_cap[k] < total_) {
            if (ctx->stage[k]) RT_HIP(hipHostFree(ctx->stage[k]));
            ctx->stage[k] = nullptr;
            ctx->stage_cap[k] = 0;
            const size_t cap = total_ + total_ / 4;
            RT_HIP(hipHostMalloc(&ctx->stage[k], cap, hipHostMallocDefault));
            ctx->stage_cap[k] = cap;
        }
        if (!ctx->stage_ev[k]) RT_HIP(hipEventCreateWithFlags(&ctx->stage_ev[k], hipEventDisableTiming));
        uint8_t* h = static_cast<uint8_t*>(ctx->stage[k]);
        for (const Part& p : parts_) std::memcpy(h + p.off, p.src, p.bytes);
        if (ctx->blob_cap < total_) {   // grow: the old blob may still be read by earlier launches
            RT_HIP(hipDeviceSynchronize());
            if (ctx->blob) RT_HIP(hipFree(ctx->blob));
            ctx->blob = nullptr;
            ctx->blob_cap = 0;
            const size_t cap = total_ + total_ / 4;
            RT_HIP(hipMalloc(&ctx->blob, cap));
            ctx->blob_cap = cap;
        }
        uint8_t* d = static_cast<uint8_t*>(ctx->blob);
        RT_HIP(hipMemcpyAsync(d, h, total_, hipMemcpyHostToDevice, st));
        RT_HIP(hipEventRecord(ctx->stage_ev[k], st));
        ctx->stage_used[k] = true;
        ctx->stage_cur = k ^ 1;
        for (const Part& p : parts_) *p.dst = d + p.off;
        return RT_OK;
    }

  private:
    struct Part { const void* src; size_t bytes, off; void** dst; };
    std::vector<Part> parts_;
    size_t total_ = 0;
};

// ---- shader.rgen:29, 48-49, 92-105: camera + viewport, once per launch ------------------
struct F3 { float x, y, z; };
inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
inline F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline float dot3(F3 a, F3 b) { return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x)); }
inline F3 unit(F3 v) {
    float len = std::sqrt(dot3(v, v));
    float inv = 1.0f / len;
    return f3(v.x * inv, v.y * inv, v.z * inv);
}
inline F3 cross3(F3 a, F3 b) {
    return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

void fill_camera(const RenderCallInfo& rci, rt::TraceParams& P) {
    const float fov = 25.0f, aperture = 0.0f, focus = 10.0f;  // shader.rgen:29
    const F3 up = f3(0.0f, 1.0f, 0.0f);
    const F3 from = f3(rci.camera_pos.x, rci.camera_pos.y, rci.camera_pos.z);
    const F3 at = from + f3(rci.camera_dir.x, rci.camera_dir.y, rci.camera_dir.z);
    const float sx = float(rci.image_size.x), sy = float(rci.image_size.y);
    const float aspect = sx / sy;
    const float half = (fov * 0.017453292519943295f) / 2.0f;
    const float vh = float(std::tan(double(half))) * 2.0f;
    const float vw = aspect * vh;
    const F3 fwd = unit(at - from);
    const F3 right = unit(cross3(up, fwd));
    const F3 cup = unit(cross3(fwd, right));
    const F3 hor = f3(vw * right.x * focus, vw * right.y * focus, vw * right.z * focus);
    const F3 ver = f3(vh * cup.x * focus, vh * cup.y * focus, vh * cup.z * focus);
    const F3 ulc = ((from - f3(hor.x / 2.0f, hor.y / 2.0f, hor.z / 2.0f)) +
                    f3(ver.x / 2.0f, ver.y / 2.0f, ver.z / 2.0f)) +
                   f3(fwd.x * focus, fwd.y * focus, fwd.z * focus);
    auto put = [](float* d, F3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; };
    put(P.lf, from); put(P.hor, hor); put(P.ver, ver); put(P.ulc, ulc); put(P.cup, cup); put(P.crt, right);
    P.half_aperture = aperture / 2.0f;
    auto finite3 = [](F3 v) { return std::isfinite(v.x) && std::isfinite(v.y) && std::isfinite(v.z); };
    P.pinhole_lf = (P.half_aperture == 0.0f && from.x != 0.0f && from.y != 0.0f && from.z != 0.0f &&
                    finite3(right) && finite3(cup)) ? 1u : 0u;
    P.size_x = sx;
    P.size_y = sy;
    P.inv_size_x = 1.0 / double(sx);
    P.inv_size_y = 1.0 / double(sy);
}

// ---- scene.h:37-157 -------------------------------------------------------------------------
inline float uniform(std::mt19937& e, float lo, float hi) {
    std::uniform_real_distribution<float> d(lo, hi);
    return d(e);
}
rt_vec4 hsv_color(std::mt19937& e) {
    const float h = std::floor(uniform(e, 0.0f, 360.0f));
    const float s = 0.75f, v = 0.45f, C = s * v;
    const float X = C * (1.0f - std::fabs(std::fmod(h / 60.0f, 2.0f) - 1.0f));
    const float m = v - C;
    float r, g, b;
    if (h >= 0 && h < 60) { r = C; g = X; b = 0; }
    else if (h >= 60 && h < 120) { r = X; g = C; b = 0; }
    else if (h >= 120 && h < 180) { r = 0; g = C; b = X; }
    else if (h >= 180 && h < 240) { r = 0; g = X; b = C; }
    else if (h >= 240 && h < 300) { r = X; g = 0; b = C; }
    else { r = C; g = 0; b = X; }
    return rt_vec4{r + m, g + m, b + m, 1.0f};
}
Sphere make_sphere(rt_vec4 g, uint32_t mat, uint32_t tex, rt_vec4 c0, rt_vec4 c1, float attr) {
    Sphere s;
    std::memset(&s, 0, sizeof(s));
    s.geometry = g;
    s.materialType = mat;
    s.textureType = tex;
    s.colors[0] = c0;
    s.colors[1] = c1;
    s.materialSpecificAttribute = attr;
    return s;
}

}  // namespace

namespace rt {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int current_device_count(int* n) {
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess || *n <= 0) {
        *n = 0;
        return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
    }
    return RT_OK;
}
}  // namespace rt

using rt::fail;
using rt::DeviceGuard;

extern "C" {

uint32_t rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return rt::g_last_error.c_str(); }

int rt_device_count(int* count) {
    if (!count) return fail(RT_ERR_INVALID_ARGUMENT, "count is NULL");
    return rt::current_device_count(count);
}

int rt_generate_scene(float t, uint32_t K, Sphere* out, uint32_t capacity, uint32_t* count) {
    const uint64_t need = 4ull + 4ull * K * K;
    if (count) *count = uint32_t(need);
    if (need > 0xffffffffull) return fail(RT_ERR_INVALID_ARGUMENT, "grid too large");
    if (!out) return count ? RT_OK : fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    if (capacity < need) return fail(RT_ERR_INVALID_ARGUMENT, "capacity too small");
    const rt_vec4 z = {0, 0, 0, 0};
    // scene.h:85-116; cos of the float time argument in double, rounded to float.
    out[0] = make_sphere({0.0f, -1000.0f, 1.0f, 1000.0f}, RT_DIFFUSE, RT_CHECKERED,
                         {0.05f, 0.05f, 0.05f, 1.0f}, {0.95f, 0.95f, 0.95f, 1.0f}, 0.0f);
    out[1] = make_sphere({-4.0f, 1.0f, float(std::cos(double(2 * t))), 1.0f}, RT_DIFFUSE, RT_SOLID,
                         {0.6f, 0.3f, 0.1f, 1.0f}, z, 0.0f);
    out[2] = make_sphere({4.0f, 1.0f, float(std::cos(double(3 * t))), 1.0f}, RT_METAL, RT_SOLID,
                         {0.8f, 0.8f, 0.8f, 1.0f}, z, 0.0f);
    out[3] = make_sphere({0.0f, 1.0f, float(std::cos(double(t))), 1.0f}, RT_REFRACTIVE, RT_SOLID,
                         {1.0f, 1.0f, 1.0f, 1.0f}, z, 1.5f);
    std::mt19937 e{};  // scene.h:120
    uint32_t i = 4;
    const int k = int(K);
    for (int a = -k; a < k; a++) {
        for (int b = -k; b < k; b++) {
            // g++ (the reference's compiler) evaluates the vec4 arguments right to left:
            // the z offset is drawn before the x offset (scene.h:124-125).
            const float dz = uniform(e, 0.0f, 1.0f);
            const float dx = uniform(e, 0.0f, 1.0f);
            const rt_vec4 g = {float(a) + 0.9f * dx, 0.2f, float(b) + 0.9f * dz, 0.2f};
            const float pm = uniform(e, 0.0f, 1.0f);
            if (double(pm) < 0.7) {
                out[i] = make_sphere(g, RT_DIFFUSE, RT_SOLID, hsv_color(e), z, 0.0f);
            } else if (double(pm) < 0.85) {
                const float cb = uniform(e, 0.5f, 1.0f);
                const float cg = uniform(e, 0.5f, 1.0f);
                const float cr = uniform(e, 0.5f, 1.0f);
                out[i] = make_sphere(g, RT_METAL, RT_SOLID, {cr, cg, cb, 1.0f}, z, 0.0f);
            } else {
                out[i] = make_sphere(g, RT_REFRACTIVE, RT_SOLID, {1.0f, 1.0f, 1.0f, 1.0f}, z, 1.5f);
            }
            i++;
        }
    }
    return RT_OK;
}

int rt_canonical_render_call_info(uint32_t spp, uint32_t width, uint32_t height, RenderCallInfo* out) {
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    std::memset(out, 0, sizeof(*out));
    out->number = 0;                                   // src/ray_trace.cpp:665
    out->samplesPerRenderCall = spp;                   // :666
    out->offset = rt_uvec2{0, 0};
    out->image_size = rt_uvec2{width, height};         // :668
    out->camera_pos = rt_vec4{13.0f, 11.0f, -3.0f, 0.0f};   // :669
    out->camera_dir = rt_vec4{-13.0f, -11.0f, 3.0f, 0.0f};  // :670
    return RT_OK;
}

int rt_context_create(int device, rt_context** out) {
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (int rc = rt::current_device_count(&n)) return rc;
    if (device < 0 || device >= n) return fail(RT_ERR_INVALID_ARGUMENT, "device index out of range");
    DeviceGuard g(device);
    std::unique_ptr<rt_context> ctx(new rt_context());
    ctx->device = device;
    RT_HIP(hipDeviceGetAttribute(&ctx->cu_count, hipDeviceAttributeMultiprocessorCount, device));
    void* c = nullptr;
    constexpr size_t kBigOff = (sizeof(rt::Counters) + 255) & ~size_t(255);
    RT_HIP(hipMalloc(&c, kBigOff + rt::kBigMax * 20u));
    RT_HIP(hipMemset(c, 0, kBigOff + rt::kBigMax * 20u));
    ctx->counters = static_cast<rt::Counters*>(c);
    ctx->big_tab = reinterpret_cast<float*>(static_cast<char*>(c) + kBigOff);
    for (auto& a : ctx->occ_lds)
        for (auto& b : a)
            for (auto& v : b) v = ~size_t(0);
    *out = ctx.release();
    return RT_OK;
}

int rt_context_destroy(rt_context* ctx) {
    if (!ctx) return RT_OK;
    DeviceGuard g(ctx->device);
    (void)hipDeviceSynchronize();
    for (SceneSlot& s : ctx->slot) {
        if (s.mem) (void)hipFree(s.mem);
        if (s.grid_mem) (void)hipFree(s.grid_mem);
        if (s.ev_free) (void)hipEventDestroy(s.ev_free);
    }
    if (ctx->build_stream) (void)hipStreamDestroy(ctx->build_stream);
    if (ctx->ev_summary) (void)hipEventDestroy(ctx->ev_summary);
    if (ctx->ev_caller) (void)hipEventDestroy(ctx->ev_caller);
    if (ctx->summary) (void)hipHostFree(ctx->summary);
    if (ctx->sph_stage) (void)hipHostFree(ctx->sph_stage);
    rt::build_release(ctx->ws);
    rt::schedule_release(ctx->sched);
    if (ctx->blob) (void)hipFree(ctx->blob);
    for (int k = 0; k < 2; k++) {
        if (ctx->stage[k]) (void)hipHostFree(ctx->stage[k]);
        if (ctx->stage_ev[k]) (void)hipEventDestroy(ctx->stage_ev[k]);
    }
    if (ctx->ev_last) (void)hipEventDestroy(ctx->ev_last);
    if (ctx->ev_prev) (void)hipEventDestroy(ctx->ev_prev);
    for (auto& pr : ctx->kev)
        for (hipEvent_t e : pr)
            if (e) (void)hipEventDestroy(e);
    for (auto& sn : ctx->snap) {
        if (sn.host) (void)hipHostFree(sn.host);
        if (sn.ev) (void)hipEventDestroy(sn.ev);
    }
    if (ctx->d_spheres) (void)hipFree(ctx->d_spheres);
    if (ctx->fixed) (void)hipFree(ctx->fixed);
    if (ctx->counters) (void)hipFree(ctx->counters);
    delete ctx;
    return RT_OK;
}

}  // extern "C"

namespace {

// ---- host-built scenes ---------------------------------------------------------------------
// Host-built tree (rt_bvh.cpp, binned SAH or Morton split) + host uniform grid: the default for
// scenes whose tree and records fit LDS, and the A/B reference of the device builder. Built once
// into a HostPackage, which any number of contexts upload (rt_multi builds it once for every GPU).
}  // namespace

namespace rt {
struct HostPackage {
    uint32_t count = 0;
    std::vector<GeomRec> geom;
    std::vector<float> radius;
    std::vector<MatRec> mat;
    HostBvh bvh;                        // nodes padded for pad_radius, leaf ids padded to 4
    std::vector<BvhNode> nodes_host;    // unpadded (far-camera re-pad)
    std::vector<BvhNode> oct;           // 8 near-child-first orders of the padded nodes
    HostGrid grid;
    bool has_grid = false;
    bool colours_unit = true;
    float scene_radius = 0.0f, pad_radius = 0.0f;
};
void HostPackageDeleter::operator()(HostPackage* p) const { delete p; }
}  // namespace rt

namespace {

rt::HostPackagePtr build_host_package(const rt_context* ctx, const Sphere* spheres, uint32_t count, bool sah) {
    rt::HostPackagePtr pk(new rt::HostPackage());
    pk->count = count;
    pk->geom.resize(count);
    pk->radius.resize(count);
    pk->mat.resize(count);
    for (uint32_t i = 0; i < count; i++) {
        const Sphere& s = spheres[i];
        if (!rt::colours_in_unit(s)) pk->colours_unit = false;
        const float r = s.geometry.w;
        pk->geom[i] = rt::GeomRec{s.geometry.x, s.geometry.y, s.geometry.z, r * r};
        pk->radius[i] = r;
        pk->mat[i] = rt::make_mat(s.colors[0].x, s.colors[0].y, s.colors[0].z, s.materialSpecificAttribute,
                                  s.colors[1].x, s.colors[1].y, s.colors[1].z, s.materialType, s.textureType);
    }
    // Brute-force padding: whole batches of 8; the pad spheres sit 1e19 away with
    // radius^2 = -1e38, so D = b^2 - a(|oc|^2 + 1e38) < 0 for every ray.
    while (pk->geom.size() % 8) pk->geom.push_back(rt::GeomRec{0.0f, 1e19f, 0.0f, -1e38f});
    rt::build_lbvh_host(spheres, count, pk->bvh, sah, uint32_t(Tuning::get(ctx->tune.sah_knobs, 0)));
    // leaf ids are read as uint4: pad to a multiple of 4
    while (pk->bvh.leaf_ids.size() % 4) pk->bvh.leaf_ids.push_back(0u);
    // pad node boxes for origins within the scene radius (hit points) and a nearby camera
    float R = 0.0f;
    for (uint32_t i = 0; i < count; i++) {
        const rt_vec4& gg = spheres[i].geometry;
        R = std::max(R, std::sqrt(gg.x * gg.x + gg.y * gg.y + gg.z * gg.z) + std::fabs(gg.w));
    }
    pk->scene_radius = R;
    pk->pad_radius = R * 1.01f + 100.0f;
    pk->nodes_host = pk->bvh.nodes;
    pad_nodes(pk->nodes_host, pk->bvh.nodes, pad_for(pk->pad_radius));
    make_octant_orders(pk->bvh.nodes, pk->oct);
    // Uniform grid (rt_grid.h) when the scene suits one: the default walk.
    // Tuning grid = 0 disables it, grid_scale sets the cell size scale (A/B; rt_grid.h).
    const float gscale = float(Tuning::get(ctx->tune.grid_scale, rt::kGridCellScaleHost));
    pk->has_grid = Tuning::get(ctx->tune.grid, 1) != 0 &&
                   rt::build_grid_host(spheres, count, pk->bvh.big_ids, 64.0f * 0x1p-24f * pk->pad_radius, gscale,
                                       1u << 22, pk->grid);
    return pk;
}

// Uploads a host package into ctx's blob (one stream-ordered copy, BlobUpload) and makes it the
// context's scene.
int commit_host_package(rt_context* ctx, const rt::HostPackage& pk, hipStream_t st) {
    ctx->scene = rt::DeviceScene{};
    ctx->slot_cur = -1;
    ctx->gpu_tree = false;
    ctx->colours_unit = pk.colours_unit;
    BlobUpload up;
    rt::DeviceScene& d = ctx->scene;
    d.n_spheres = pk.count;
    up.add(pk.geom, &d.geom);
    up.add(pk.radius, &d.radius);
    up.add(pk.mat, &d.mat);
    d.small_rmax = pk.bvh.small_rmax;
    d.small_rmin = pk.bvh.small_rmin;
    d.n_big = uint32_t(pk.bvh.big_ids.size());
    up.add(pk.bvh.big_ids, &d.big_ids);
    d.n_nodes = uint32_t(pk.bvh.nodes.size());
    d.n_leaf = uint32_t(pk.bvh.leaf_geom.size());
    ctx->scene_radius = pk.scene_radius;
    ctx->pad_radius = pk.pad_radius;
    ctx->padded_for = pk.pad_radius;
    ctx->nodes_host = pk.nodes_host;
    up.add(pk.oct, &d.nodes_oct);
    ctx->has_grid = pk.has_grid;
    if (pk.has_grid) {
        d.grid = pk.grid.info;
        up.add(pk.grid.cell_start, &d.cell_start);
        up.add(pk.grid.rec, &d.grid_rec);
        up.add(pk.grid.ids, &d.grid_ids);
        ctx->grid_pad_radius = pk.pad_radius;
    }
    size_lds_forms(ctx);
    up.add(pk.bvh.nodes, &d.nodes);
    up.add(pk.bvh.leaf_geom, &d.leaf_geom);
    up.add(pk.bvh.leaf_ids, &d.leaf_ids);
    return up.commit(ctx, st);
}

// ---- device-built scenes (rt_build.hip) ------------------------------------------------------
// Two arenas used alternately (rt_context::slot): frame k + 1's build writes the arena frame k
// does not read, on the context's own build stream, so it runs beside frame k (in the CUs its
// tail frees) instead of after it, and no arena is freed or allocated per frame. The build waits
// only for the launches that read its arena two scenes ago (SceneSlot::ev_free). The host reads
// one summary back (counts, radii, root box) to lay out the grid; the next launch of the context
// waits for the build's last kernel (ev_last on the build stream), on whatever stream it runs.
size_t round256(size_t b) { return (b + 255u) & ~size_t(255); }

int ensure_build_stream(rt_context* ctx) {
    if (ctx->build_stream) return RT_OK;
    RT_HIP(hipStreamCreateWithFlags(&ctx->build_stream, hipStreamNonBlocking));
    RT_HIP(hipEventCreateWithFlags(&ctx->ev_summary, hipEventDisableTiming));
    RT_HIP(hipEventCreateWithFlags(&ctx->ev_caller, hipEventDisableTiming));
    for (SceneSlot& s : ctx->slot) RT_HIP(hipEventCreateWithFlags(&s.ev_free, hipEventDisableTiming));
    void* p = nullptr;
    RT_HIP(hipHostMalloc(&p, sizeof(rt::BuildSummary), hipHostMallocDefault));
    ctx->summary = static_cast<rt::BuildSummary*>(p);
    return RT_OK;
}

// Frees memory an arena's queued launches may still read: waits for them and for the build stream.
int retire_slot_memory(rt_context* ctx, SceneSlot& s, void*& mem) {
    if (!mem) return RT_OK;
    if (s.used) RT_HIP(hipEventSynchronize(s.ev_free));
    RT_HIP(hipStreamSynchronize(ctx->build_stream));
    RT_HIP(hipFree(mem));
    mem = nullptr;
    return RT_OK;
}

// Per-sphere arrays of an arena for n spheres, carved out of one allocation (12.5 % headroom).
int slot_reserve(rt_context* ctx, SceneSlot& s, uint32_t n) {
    if (s.mem && s.cap_n >= n) return RT_OK;
    if (int rc = retire_slot_memory(ctx, s, s.mem)) return rc;
    s.cap_n = 0;
    const size_t c = std::max<size_t>(64, size_t(n) + n / 8);
    const size_t sz[] = {((c + 7) & ~size_t(7)) * sizeof(rt::GeomRec), c * 4, c * sizeof(rt::MatRec), 64 * 4,
                         2 * c * sizeof(rt::BvhNode), 2 * c * sizeof(rt::BvhNode), 4 * c * sizeof(rt::GeomRec),
                         4 * c * 4, 8 * size_t(rt::kTreeletCap) * 4, 16};
    size_t off[10], total = 0;
    for (int i = 0; i < 10; i++) { off[i] = total; total += round256(sz[i]); }
    RT_HIP(hipMalloc(&s.mem, total));
    char* b = static_cast<char*>(s.mem);
    rt::DeviceScene& d = s.scene;
    d = rt::DeviceScene{};
    d.geom = reinterpret_cast<rt::GeomRec*>(b + off[0]);
    d.radius = reinterpret_cast<float*>(b + off[1]);
    d.mat = reinterpret_cast<rt::MatRec*>(b + off[2]);
    d.big_ids = reinterpret_cast<uint32_t*>(b + off[3]);
    d.nodes = reinterpret_cast<rt::BvhNode*>(b + off[4]);
    d.nodes_raw = reinterpret_cast<rt::BvhNode*>(b + off[5]);
    d.leaf_geom = reinterpret_cast<rt::GeomRec*>(b + off[6]);
    d.leaf_ids = reinterpret_cast<uint32_t*>(b + off[7]);
    d.treelet = reinterpret_cast<float*>(b + off[8]);
    d.treelet_count = reinterpret_cast<uint32_t*>(b + off[9]);
    s.cap_n = uint32_t(c);
    return RT_OK;
}

int stage_spheres(rt_context* ctx, const Sphere* spheres, uint32_t count, bool device_ptr, hipStream_t st) {
    const size_t bytes = size_t(count) * sizeof(Sphere);
    if (count > ctx->d_spheres_cap) {   // the previous build's kernels may still read it
        if (ctx->d_spheres) {
            RT_HIP(hipStreamSynchronize(ctx->build_stream));
            RT_HIP(hipFree(ctx->d_spheres));
        }
        ctx->d_spheres = nullptr;
        ctx->d_spheres_cap = 0;
        void* p = nullptr;
        RT_HIP(hipMalloc(&p, bytes));
        ctx->d_spheres = static_cast<Sphere*>(p);
        ctx->d_spheres_cap = count;
    }
    if (!count) return RT_OK;
    if (device_ptr) {   // written by the caller's earlier work on st; copied so the build (and
                        // the grid build, which runs after the call returns) never reads it later
        RT_HIP(hipEventRecord(ctx->ev_caller, st));
        RT_HIP(hipStreamWaitEvent(ctx->build_stream, ctx->ev_caller, 0));
        RT_HIP(hipMemcpyAsync(ctx->d_spheres, spheres, bytes, hipMemcpyDeviceToDevice, ctx->build_stream));
        return RT_OK;
    }
    // host spheres through a pinned buffer: an asynchronous copy (a pageable one would block the
    // host until the previous frame's GPU work leaves the copy engine)
    if (ctx->sph_stage_cap < bytes) {
        if (ctx->sph_stage) {
            RT_HIP(hipStreamSynchronize(ctx->build_stream));
            RT_HIP(hipHostFree(ctx->sph_stage));
        }
        ctx->sph_stage = nullptr;
        ctx->sph_stage_cap = 0;
        RT_HIP(hipHostMalloc(&ctx->sph_stage, bytes + bytes / 8, hipHostMallocDefault));
        ctx->sph_stage_cap = bytes + bytes / 8;
    }
    std::memcpy(ctx->sph_stage, spheres, bytes);   // the previous copy from it ended with its build
    RT_HIP(hipMemcpyAsync(ctx->d_spheres, ctx->sph_stage, bytes, hipMemcpyHostToDevice, ctx->build_stream));
    return RT_OK;
}

// Phase 1 of a device build: the spheres to the device and the LBVH build of the free arena, all on
// the build stream, up to the summary's copy to pinned memory (ev_summary). refit: keep the
// topology of the last full build (same count; positions / radii / materials may change).
int device_build_begin(rt_context* ctx, const Sphere* spheres, uint32_t count, bool device_ptr, hipStream_t st,
                       bool refit) {
    if (int rc = ensure_build_stream(ctx)) return rc;
    const int k = ctx->slot_cur == 0 ? 1 : 0;
    SceneSlot& s = ctx->slot[k];
    const hipStream_t bs = ctx->build_stream;
    if (s.used) RT_HIP(hipStreamWaitEvent(bs, s.ev_free, 0));   // its last readers (two scenes ago)
    if (int rc = slot_reserve(ctx, s, count)) return rc;
    if (int rc = stage_spheres(ctx, spheres, count, device_ptr, st)) return rc;
    rt::DeviceScene& d = s.scene;
    if (!refit) ctx->topo_ok = false;   // the build overwrites the workspace's topology
    if (refit)   // the big set is the topology's (a refit does not re-select it)
        RT_HIP(hipMemcpyAsync(d.big_ids, ctx->slot[ctx->slot_cur].scene.big_ids, 64 * 4, hipMemcpyDeviceToDevice, bs));
    const rt::BuildOutputs o{d.geom, d.radius, d.mat, d.big_ids, d.nodes, d.nodes_raw, d.leaf_geom, d.leaf_ids};
    const hipError_t e = rt::build_scene_gpu(ctx->ws, ctx->d_spheres, count, o, refit, bs, ctx->summary);
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_DEVICE,
                    std::string("device LBVH build: ") + hipGetErrorString(e));
    RT_HIP(hipEventRecord(ctx->ev_summary, bs));
    ctx->pending = true;
    ctx->pending_slot = k;
    ctx->pending_count = count;
    ctx->pending_refit = refit;
    return RT_OK;
}

// Phase 2: the summary (host wait for the build only, not for earlier launches), the device grid
// over the small spheres (the default walk) from the tree's root box, and the
// arena becomes the context's scene.
int device_build_end(rt_context* ctx) {
    if (!ctx->pending) return RT_OK;
    ctx->pending = false;
    const int k = ctx->pending_slot;
    SceneSlot& s = ctx->slot[k];
    const hipStream_t bs = ctx->build_stream;
    RT_HIP(hipEventSynchronize(ctx->ev_summary));
    const rt::BuildSummary sm = *ctx->summary;
    rt::DeviceScene& d = s.scene;
    d.n_spheres = ctx->pending_count;
    d.n_big = sm.n_big;
    d.n_nodes = sm.n_nodes;
    d.n_leaf = sm.n_leaf_slots;
    d.small_rmax = rt::summary_float(sm.rmax_o);
    d.small_rmin = rt::summary_float(sm.rmin_o);
    d.grid = rt::GridInfo{};
    d.cell_start = d.grid_ids = nullptr;
    d.grid_rec = nullptr;
    ctx->colours_unit = sm.colour_out_of_range == 0u;
    ctx->scene_radius = rt::summary_float(sm.R_o);
    ctx->pad_radius = ctx->scene_radius * 1.01f + 100.0f;   // the build padded for this radius
    ctx->padded_for = ctx->pad_radius;
    ctx->has_grid = false;
    if (Tuning::get(ctx->tune.grid, 1) != 0 && sm.n_small && d.small_rmax > 0.0f) {
        rt::GridInfo gi;
        uint64_t bound = 0;
        if (rt::grid_layout(sm.root_lo, sm.root_hi, sm.n_small, d.small_rmax, 64.0f * 0x1p-24f * ctx->pad_radius,
                            float(Tuning::get(ctx->tune.grid_scale, rt::kGridCellScale)), gi, &bound) &&
            bound <= (1u << 26)) {
            const size_t nc1 = size_t(gi.n_cells) + 1, tb = rt::grid_scan_bytes(gi.n_cells);
            const size_t off_cur = round256(nc1 * 4), off_rec = off_cur + round256(nc1 * 4),
                         off_ids = off_rec + round256(size_t(bound) * sizeof(rt::GeomRec)),
                         off_tmp = off_ids + round256(size_t(bound) * 4), total = off_tmp + round256(tb);
            if (s.grid_cap < total) {
                if (int rc = retire_slot_memory(ctx, s, s.grid_mem)) return rc;
                s.grid_cap = 0;
                RT_HIP(hipMalloc(&s.grid_mem, total + total / 8));
                s.grid_cap = total + total / 8;
            }
            char* g = static_cast<char*>(s.grid_mem);
            d.cell_start = reinterpret_cast<uint32_t*>(g);
            d.grid_rec = reinterpret_cast<rt::GeomRec*>(g + off_rec);
            d.grid_ids = reinterpret_cast<uint32_t*>(g + off_ids);
            RT_HIP(rt::build_grid_gpu(ctx->ws, ctx->d_spheres, d.n_spheres, gi, reinterpret_cast<uint32_t*>(g + off_cur),
                                      d.cell_start, d.grid_rec, d.grid_ids, g + off_tmp, tb, bs));
            gi.n_refs = 0;   // exact count left on the device: the grid is walked from L2
            d.grid = gi;
            ctx->has_grid = true;
            ctx->grid_pad_radius = ctx->pad_radius;
        }
    }
    ctx->scene = d;
    ctx->slot_cur = k;
    if (!ctx->pending_refit) ctx->topo_ok = true;   // ws now holds the current arena's topology
    ctx->gpu_tree = true;
    ctx->treelet_stale = true;
    ctx->nodes_host.clear();
    size_lds_forms(ctx);
    return RT_OK;
}

// Tree builder (RT_BVH_BUILD): "auto" (default) = host binned SAH for scenes whose tree and
// records fit LDS (best walk cost, build <= ~1 ms), else the device LBVH (LDS treelet over L2);
// "gpu", "sah", "morton" force one (A/B, tests).
constexpr uint32_t kHostSahMaxSpheres = 1024;
enum class Builder { GPU, HOST_SAH, HOST_MORTON };
Builder pick_builder(uint32_t count) {
    const char* b = std::getenv("RT_BVH_BUILD");
    if (b && std::strcmp(b, "gpu") == 0) return Builder::GPU;
    if (b && std::strcmp(b, "sah") == 0) return Builder::HOST_SAH;
    if (b && std::strcmp(b, "morton") == 0) return Builder::HOST_MORTON;
    return count <= kHostSahMaxSpheres ? Builder::HOST_SAH : Builder::GPU;
}

int check_scene_args(rt_context* ctx, const Sphere* spheres, uint32_t count) {
    if (!ctx) return fail(RT_ERR_INVALID_ARGUMENT, "ctx is NULL");
    if (!spheres && count) return fail(RT_ERR_INVALID_ARGUMENT, "spheres is NULL");
    if (count >= (1u << 27)) return fail(RT_ERR_INVALID_ARGUMENT, "too many spheres");
    return RT_OK;
}

// Bookkeeping after a scene call: the scene is usable (or not, RT_ERR_NO_SCENE), launch info
// reports its default form until it renders.
int scene_done(rt_context* ctx, int rc) {
    ctx->scene_set = rc == RT_OK;
    ctx->last_accel = 0;
    return rc;
}

// First half of every scene call. Host-built scenes are built (or taken from *shared, built by an
// earlier context of the same rt_multi frame) and uploaded in order on `st` after the context's
// previous operations; device-built scenes start their build on the context's build stream.
int scene_begin(rt_context* ctx, const Sphere* spheres, uint32_t count, bool device_ptr, hipStream_t st, bool refit,
                rt::HostPackagePtr* shared) {
    DeviceGuard g(ctx->device);
    if (int rc = device_build_end(ctx)) return rc;   // a begin without its end (never in this library)
    const Builder b = device_ptr ? Builder::GPU : pick_builder(count);
    if (b != Builder::GPU) {
        try {
            if (int rc = order_on(ctx, st)) return rc;
            rt::HostPackagePtr own;
            rt::HostPackagePtr& pk = shared ? *shared : own;
            if (!pk || pk->count != count) pk = build_host_package(ctx, spheres, count, b == Builder::HOST_SAH);
            if (int rc = commit_host_package(ctx, *pk, st)) return rc;
            return mark_issued(ctx, st);
        } catch (const std::exception& e) {
            return fail(RT_ERR_OUT_OF_MEMORY, e.what());
        }
    }
    return device_build_begin(ctx, spheres, count, device_ptr, st, refit && ctx->gpu_tree && ctx->slot_cur >= 0 &&
                                                                       ctx->topo_ok && count == ctx->scene.n_spheres &&
                                                                       ctx->ws.topo_n == count);
}

int scene_end(rt_context* ctx) {
    if (!ctx->pending) return RT_OK;
    DeviceGuard g(ctx->device);
    if (int rc = device_build_end(ctx)) return rc;
    return mark_built(ctx);   // the next operation waits for the build and for the op before it
}

}  // namespace

namespace rt {
int set_scene_begin(rt_context* ctx, const Sphere* spheres, uint32_t count, void* stream, HostPackagePtr* shared) {
    if (int rc = check_scene_args(ctx, spheres, count)) return rc;
    const int rc = scene_begin(ctx, spheres, count, false, static_cast<hipStream_t>(stream), false, shared);
    if (rc != RT_OK) {
        ctx->pending = false;
        return scene_done(ctx, rc);
    }
    return RT_OK;
}

int set_scene_end(rt_context* ctx) {
    const int rc = scene_end(ctx);
    ctx->pending = false;
    return scene_done(ctx, rc);
}
}  // namespace rt

namespace {

int scene_call(rt_context* ctx, const Sphere* spheres, uint32_t count, bool device_ptr, void* stream, bool refit) {
    if (int rc = check_scene_args(ctx, spheres, count)) return rc;
    int rc = scene_begin(ctx, spheres, count, device_ptr, static_cast<hipStream_t>(stream), refit, nullptr);
    if (rc == RT_OK) rc = scene_end(ctx);
    ctx->pending = false;
    return scene_done(ctx, rc);
}

// Kernel form of a launch (rt_internal.h ACCEL_*) and its dynamic LDS bytes. form =
// options.reserved[1] (A/B and tests, 0 = automatic): 6 one LDS node copy, 8 octant copies, 10
// every node from L2, 12 the grid, 14 the grid with the wave-cooperative walk; cam_r = the camera's
// distance from the origin (the grid's margin covers cameras within its pad radius).
uint32_t choose_accel(const rt_context* ctx, bool brute, uint32_t form, float cam_r, size_t* lds_out) {
    const rt::DeviceScene& d = ctx->scene;
    const Tuning& tu = ctx->tune;
    uint32_t accel;
    size_t lds = 0;
    if (brute) {
        accel = rt::ACCEL_BRUTE;
    } else if (ctx->has_grid && cam_r <= ctx->grid_pad_radius &&
               (form == 12u || form == 14u || form == 16u || (form == 0u && (ctx->grid_bytes || !ctx->oct_bytes)))) {
        // the grid: staged in LDS when it fits (config 3: 1 % faster than the
        // octant tree), else the octant tree when that fits LDS (a device-built scene of ~1000
        // spheres, whose grid would be read from L2), else the grid from L2
        accel = ctx->grid_bytes ? rt::ACCEL_GRID : rt::ACCEL_GRID_GLOBAL;
        lds = ctx->grid_bytes;   // 0: the grid from L2
        // the wave-cooperative walk: form 14, or tuning grid_coop = 1
        const bool coop = form == 14u || (form == 0u && Tuning::get(tu.grid_coop, 0) == 1);
        if (coop && accel == rt::ACCEL_GRID &&
            ctx->grid_bytes + rt::kLaneSumLdsBytes + rt::kCoopLdsBytes <= kMaxLdsBytes)
            accel = rt::ACCEL_GRID_COOP;
        else if (coop && accel == rt::ACCEL_GRID_GLOBAL)
            accel = rt::ACCEL_GRID_GLOBAL_COOP;
        // the LDS grid kernel also stages the winner's gate and shading records ({c, r} + the
        // material record, 48 B per sphere) when two blocks per CU still fit;
        // tuning grid_rec = 0: not (A/B)
        // (the kernel's static table of kRecStatic records: scenes of at most that many spheres)
        const size_t rec_bytes = d.n_spheres <= rt::kRecStatic ? size_t(rt::kRecStatic) * 48u : kMaxLdsBytes;
        // the wave-wide candidate queue: form 16, or tuning grid_cq = 1
        const bool cq = accel == rt::ACCEL_GRID && (form == 16u || (form == 0u && Tuning::get(tu.grid_cq, 0) == 1));
        const size_t cq_bytes = cq ? rt::kCqLdsBytes : 0u;
        if (accel == rt::ACCEL_GRID && Tuning::get(tu.grid_rec, 1) != 0 &&
            ctx->grid_bytes + rec_bytes + rt::kLaneSumLdsBytes + cq_bytes <= kTwoBlockLdsBytes) {
            accel = cq ? rt::ACCEL_GRID_REC_CQ : rt::ACCEL_GRID_REC;
            lds = ctx->grid_bytes;   // (the records: static LDS of the kernel)
        } else if (cq && ctx->grid_bytes + rt::kLaneSumLdsBytes + cq_bytes <= kMaxLdsBytes) {
            accel = rt::ACCEL_GRID_CQ;
        }
    } else if (ctx->oct_bytes && (form == 0u || form == 8u)) {
        accel = rt::ACCEL_LBVH_OCT;
        lds = ctx->oct_bytes;
    } else if (ctx->lds1_bytes && (form == 0u || form == 6u || form == 8u)) {
        accel = rt::ACCEL_LBVH_LDS;
        lds = ctx->lds1_bytes;
    } else if (ctx->gpu_tree && d.treelet && d.n_nodes && d.n_leaf < (1u << 26) && form != 10u) {
        // (treelet leaf words carry first_count in 30 bits)
        accel = rt::ACCEL_LBVH_TOP;
        lds = size_t(rt::kTreeletCap) * 32u;
    } else {
        accel = rt::ACCEL_LBVH_GLOBAL;
    }
    *lds_out = lds;
    return accel;
}

}  // namespace

extern "C" {

int rt_set_scene(rt_context* ctx, const Sphere* spheres, uint32_t count, void* stream) {
    return scene_call(ctx, spheres, count, false, stream, false);
}

int rt_set_scene_device(rt_context* ctx, const Sphere* d_spheres, uint32_t count, void* stream) {
    return scene_call(ctx, d_spheres, count, true, stream, false);
}

int rt_refit_scene(rt_context* ctx, const Sphere* spheres, uint32_t count, void* stream) {
    // without a device-built tree of this count there is no topology to reuse: a full build
    return scene_call(ctx, spheres, count, false, stream, true);
}

int rt_refit_scene_device(rt_context* ctx, const Sphere* d_spheres, uint32_t count, void* stream) {
    return scene_call(ctx, d_spheres, count, true, stream, true);
}

int rt_render_device(rt_context* ctx, const RenderCallInfo* rci, const uint32_t* rows,
                     uint32_t band_width, uint32_t band_height, float* accum, uint8_t* out,
                     const rt_options* opt, void* stream) {
    if (!ctx || !rci) return fail(RT_ERR_INVALID_ARGUMENT, "ctx or rci is NULL");
    if (ctx->pending) return fail(RT_ERR_INVALID_ARGUMENT, "rt_render_device between the halves of a scene build");
    if (!ctx->scene_set) return fail(RT_ERR_NO_SCENE, "rt_render_device before rt_set_scene");
    if (band_width == 0 || band_height == 0) return RT_OK;
    if (!accum || !out) return fail(RT_ERR_INVALID_ARGUMENT, "accum or out is NULL");
    if (rci->image_size.x == 0 || rci->image_size.y == 0)
        return fail(RT_ERR_INVALID_ARGUMENT, "image_size is zero");
    // the kernel keeps a pixel's band coordinates as 16-bit halves of one word (Path::px)
    if (band_width > 65535u || band_height > 65535u)
        return fail(RT_ERR_INVALID_ARGUMENT, "band width and height must be below 65536");
    rt_options o;
    std::memset(&o, 0, sizeof(o));
    if (opt) o = *opt;
    if (o.accel > RT_ACCEL_LBVH) return fail(RT_ERR_INVALID_ARGUMENT, "unknown accel");
    if (o.seed_mode > RT_SEED_LAUNCH_LOCAL) return fail(RT_ERR_INVALID_ARGUMENT, "unknown seed_mode");
    if (o.rng_mode > RT_RNG_SAMPLE_HASH) return fail(RT_ERR_INVALID_ARGUMENT, "unknown rng_mode");
    const int mode = o.rng_mode == RT_RNG_SAMPLE_HASH ? rt::MODE_HASH : rt::MODE_STREAM;
    const uint32_t spp = rci->samplesPerRenderCall;
    if (mode == rt::MODE_HASH && spp > rt::kHashMaxSpp)
        return fail(RT_ERR_INVALID_ARGUMENT, "RT_RNG_SAMPLE_HASH: samplesPerRenderCall above 2^19");
    // The fixed-point sums of RT_RNG_SAMPLE_HASH hold per-sample colours in [0, 1]: the reference
    // sums unclamped (shader.rgen:55-59), so a scene whose colours can leave [0, 1] is refused
    // rather than silently clipped (use RT_RNG_PIXEL_STREAM for it).
    if (mode == rt::MODE_HASH && !ctx->colours_unit)
        return fail(RT_ERR_INVALID_ARGUMENT,
                    "RT_RNG_SAMPLE_HASH needs every sphere colour channel in [0, 1] (colors[0], and colors[1] of "
                    "checkered spheres); this scene has one outside: render it with RT_RNG_PIXEL_STREAM");
    const uint64_t tiles_x = (band_width + 7u) / 8u, tiles_y = (band_height + 7u) / 8u;
    const uint64_t n_tiles = tiles_x * tiles_y;
    // reserved[1] (internal, A/B only): walk form, 0 = automatic (choose_accel)
    const rt::DeviceScene& d = ctx->scene;
    const float cam_r = std::sqrt(rci->camera_pos.x * rci->camera_pos.x + rci->camera_pos.y * rci->camera_pos.y +
                                  rci->camera_pos.z * rci->camera_pos.z);
    size_t lds = 0;
    const uint32_t accel = choose_accel(ctx, o.accel == RT_ACCEL_BRUTE, o.reserved[1], cam_r, &lds);
    const bool count = (o.reserved[0] & 1u) != 0;  // internal: count box / sphere tests
    DeviceGuard g(ctx->device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (int rc = order_on(ctx, st)) return rc;

    rt::TraceParams P;
    std::memset(&P, 0, sizeof(P));
    fill_camera(*rci, P);
    P.number = rci->number;
    P.spp = spp;
    P.max_depth = o.max_depth ? o.max_depth : 50u;
    P.seed_local = o.seed_mode == RT_SEED_LAUNCH_LOCAL;
    P.force_regate = (o.reserved[0] & 2u) ? 1u : 0u;   // test only: exercise regate_brute everywhere
    P.rng_counter = o.rng_mode == RT_RNG_SAMPLE_COUNTER;
    P.sample_base = o.sample_base;
    P.accumulate = o.accumulate ? 1u : 0u;
    P.off_x = rci->offset.x;
    P.off_y = rci->offset.y;
    P.band_w = band_width;
    P.band_h = band_height;
    P.tiles_x = uint32_t(tiles_x);
    P.rows = rows;
    P.n_spheres = d.n_spheres;
    P.geom = d.geom;
    P.radius = d.radius;
    P.mat = d.mat;
    P.n_big = d.n_big;
    P.big_ids = d.big_ids;
    P.nodes = d.n_nodes ? d.nodes : nullptr;
    P.n_nodes = d.n_nodes;
    P.nodes_oct = d.nodes_oct;
    P.treelet = d.treelet;
    P.treelet_count = d.treelet_count;
    const bool grid_walk = accel == rt::ACCEL_GRID || accel == rt::ACCEL_GRID_GLOBAL || accel == rt::ACCEL_GRID_COOP ||
                           accel == rt::ACCEL_GRID_GLOBAL_COOP || accel == rt::ACCEL_GRID_REC ||
                           accel == rt::ACCEL_GRID_CQ || accel == rt::ACCEL_GRID_REC_CQ;
    if (grid_walk) {   // (cell_start also marks a walk)
        P.grid = d.grid;
        P.cell_start = d.cell_start;
        P.grid_rec = d.grid_rec;
        P.grid_ids = d.grid_ids;
    }
    P.n_leaf = d.n_leaf;
    P.leaf_geom = d.leaf_geom;
    P.leaf_ids = d.leaf_ids;
    // Node-cull slack: a candidate's AABB entry lies at most
    // 2.75 r + 1.15e-3 t beyond its reported t.
    P.cull_abs = 3.0f * d.small_rmax + 1e-3f;
    P.cull_rel = 2e-3f;
    // Grid walks: the r-term of the slack is there for quadratic false positives
    // (computed D >= 0, the line passing eps_d <= 7 u |oc|^2 / r outside the sphere, u = 2^-24)
    // whose AABB entry lies up to ~1.42 r past t. The grid registers a sphere in every cell its AABB
    // widened by 64 u R + 1e-3 cell overlaps; the 1e-3-cell part is spare (64 u R covers the DDA's
    // rounding), so while eps_d <= 1e-3 cell the cell holding the ray's closest approach, reached by
    // best + 1e-3 + 2e-3 best, already references the sphere. eps_d <= 1e-3 cell holds for |oc| <= T
    // = sqrt(1e-3 cs r_min / 7u) (3/4 of that budget below), and t <= 0.95 T - r_max - 1e-3 cs implies
    // |oc| <= T. The reported
    // t lies within 9.1e-4 |oc| (sqrt of D's error, 14 u |oc|^2) of the true or closest-approach t.
    P.cull_near_t = -1.0f;
    P.cull_near_abs = P.cull_abs;
    if (grid_walk && d.small_rmin > 0.0f &&
        std::isfinite(d.small_rmin)) {
        const double m = RT_GRID_SPARE * std::min<double>(d.grid.cs[0], std::min<double>(d.grid.cs[1], d.grid.cs[2]));
        // budget: 3/4 of the spare part for eps_d, 1/4 for a walk that starts (at tmin) up to
        // 9.1e-4 |oc| ~ 9.1e-4 (r + tmin) past a closest approach just behind tmin
        const double T = std::sqrt(0.75 * m * double(d.small_rmin) / (7.0 * 0x1p-24));
        const double tn = 0.95 * T - double(d.small_rmax) - m;
        const bool start_ok = 9.1e-4 * (double(d.small_rmax) + 1e-3) <= 0.25 * m;
        if (tn > 0.0 && start_ok && Tuning::get(ctx->tune.grid_full_slack, 0) == 0) {   // grid_full_slack: A/B only
            P.cull_near_t = float(tn);
            P.cull_near_abs = 1e-3f + 1e-3f * d.small_rmax;   // covers 9.1e-4 (r + eps_d) of |oc| - t
        }
    }
    P.accum = accum;
    P.out = reinterpret_cast<uint32_t*>(out);
    P.counters = ctx->counters;

    {   // a camera outside the padded radius: re-pad the node boxes for it (rare, synchronous)
        const float cx = rci->camera_pos.x, cy = rci->camera_pos.y, cz = rci->camera_pos.z;
        const float cam_r = std::sqrt(cx * cx + cy * cy + cz * cz);
        if (!(cam_r <= ctx->pad_radius) && d.n_nodes) {
            if (!std::isfinite(cam_r)) return fail(RT_ERR_INVALID_ARGUMENT, "camera position is not finite");
            ctx->pad_radius = std::max(ctx->scene_radius, cam_r) * 1.01f + 100.0f;
        }
        if (ctx->gpu_tree && ctx->pad_radius != ctx->padded_for) {
            RT_HIP(rt::repad_nodes_gpu(d.nodes_raw, d.nodes, d.n_nodes, pad_for(ctx->pad_radius), st));
            ctx->treelet_stale = true;
            ctx->padded_for = ctx->pad_radius;
        } else if (!ctx->gpu_tree && ctx->pad_radius != ctx->padded_for) {
            std::vector<rt::BvhNode> n1;
            pad_nodes(ctx->nodes_host, n1, pad_for(ctx->pad_radius));
            RT_HIP(hipStreamSynchronize(st));
            if (!n1.empty()) RT_HIP(hipMemcpy(d.nodes, n1.data(), n1.size() * sizeof(n1[0]), hipMemcpyHostToDevice));
            if (d.nodes_oct) {
                std::vector<rt::BvhNode> oct;
                make_octant_orders(n1, oct);
                RT_HIP(hipMemcpy(d.nodes_oct, oct.data(), oct.size() * sizeof(oct[0]), hipMemcpyHostToDevice));
            }
            ctx->padded_for = ctx->pad_radius;
        }
    }
    // The row map of a banded launch (N > 1 strips) is staged in the walk kernels' dynamic LDS
    // after their own data (band_row, rt_kernels.hip) when that keeps the blocks per CU; else it
    // is read from global memory.
    P.rows_lds = rt::kNoRowsLds;
    const bool flat = rt::flat_grid_form(P, accel, count);   // the kernel launch_trace picks
    if (rows && accel != rt::ACCEL_BRUTE) {
        const size_t off = (lds + 15) & ~size_t(15), with = off + size_t(band_height) * 4u;
        int b0 = 0, b1 = 0;
        if (with <= kMaxLdsBytes && rt::trace_occupancy(accel, count, mode, flat, lds, &b0) == hipSuccess &&
            rt::trace_occupancy(accel, count, mode, flat, with, &b1) == hipSuccess && b1 >= b0 && b1 > 0) {
            P.rows_lds = uint32_t(off);
            lds = with;
        }
    }
    // Grid: one persistent block per CU slot the occupancy allows.
    const int ci = count ? 1 : flat ? 2 : 0;
    if (ctx->occ_lds[accel][ci][mode] != lds) {
        int b = 0;
        RT_HIP(rt::trace_occupancy(accel, count, mode, flat, lds, &b));
        ctx->occ[accel][ci][mode] = std::max(1, b);
        ctx->occ_lds[accel][ci][mode] = lds;
    }
    const uint64_t blk = rt::block_size(accel);
    const uint64_t lanes = uint64_t(ctx->cu_count) * ctx->occ[accel][ci][mode] * blk;
    // Sample chunks per pixel (HASH only: the image does not depend on them):
    // enough units for ~128 per lane, but units of at least 256 samples, so the frame is
    // throughput-bound and its tail (the units running when the queue runs dry, about one unit
    // long) short, without paying a unit's start and flush too often (config 3,
    // 10 000 spp, 4 -> 25 chunks -2.0 %; config 5, 1000 spp 4K: 1 / 3 / 7 / 14 chunks 658.6 /
    // 655.3 / 666.0 / 685.9 ms). Tuning sample_chunks forces a count, units_per_lane /
    // unit_min_samples set the targets. The brute-force walk's samples cost ~n/10 times a grid
    // sample, so its floor scales down with n (488 spheres: 5 samples; config 2, 100 spp: 1 -> 20
    // chunks).
    uint64_t chunks = 1;
    bool chunks_forced = false;
    if (mode == rt::MODE_HASH && spp > 1) {
        // units of >= spp / 32 samples, between 32 and 128 (256 until round 5; 128 for every spp
        // until round 6): a band of the N = 8 frame (135 rows at 10 000 spp) is capped by this
        // floor, not by the lanes, and its 256-sample tail units left a tail after the queue ran
        // dry of 4.9 % of the band; config 5's 270-row band at 1 000 spp had 7
        // chunks of 143 samples under the 128 floor, a 6-7 ms tail of a 68 ms band: 15 chunks
        // (32-sample floor) -1.1 / -2.0 % on two bands, configs 3 / 4 unchanged (10 000 / 32 >
        // 128; profiles/r06d_tune2_*.txt)
        uint64_t per_lane = 128, min_samples = std::min<uint64_t>(128, std::max<uint64_t>(32, spp / 32));
        if (accel == rt::ACCEL_BRUTE) min_samples = std::min<uint64_t>(256, std::max<uint64_t>(4, 2560 / std::max(1u, d.n_spheres)));
        per_lane = std::max<uint64_t>(1, uint64_t(Tuning::get(ctx->tune.units_per_lane, double(per_lane))));
        min_samples = std::max<uint64_t>(1, uint64_t(Tuning::get(ctx->tune.unit_min_samples, double(min_samples))));
        const uint64_t pixels = uint64_t(band_width) * band_height;
        chunks = std::min<uint64_t>((lanes * per_lane + pixels - 1) / pixels, std::max<uint64_t>(1, spp / min_samples));
        if (ctx->tune.sample_chunks != Tuning::kUnset) {
            chunks = uint64_t(ctx->tune.sample_chunks);
            chunks_forced = true;
        }
        chunks = std::max<uint64_t>(1, std::min<uint64_t>({chunks, spp, 4096}));
        while (chunks > 1 && n_tiles * chunks * 64u >= (1ull << 31)) chunks /= 2;   // unit ids in 32 bits
    }
    if (n_tiles * chunks * 64u >= (1ull << 32)) return fail(RT_ERR_INVALID_ARGUMENT, "band too large");
    P.chunks = uint32_t(chunks);
    ctx->last_accel = accel;
    ctx->last_lds = lds;
    ctx->last_flat = flat;
    ctx->last_pinhole = P.pinhole_lf != 0;
    const uint64_t texels = uint64_t(band_width) * band_height;
    if (mode == rt::MODE_HASH) {
        if (ctx->fixed_cap < texels) {
            if (ctx->fixed) {
                RT_HIP(hipStreamSynchronize(st));   // ordered after every earlier op of ctx
                RT_HIP(hipFree(ctx->fixed));
            }
            ctx->fixed = nullptr;
            ctx->fixed_cap = 0;
            void* p = nullptr;
            constexpr size_t kPlanes = 3;   // (texel-major, one 32-B sector per texel: +22 % WRITE_SIZE)
            RT_HIP(hipMalloc(&p, texels * kPlanes * sizeof(unsigned long long)));
            RT_HIP(hipMemsetAsync(p, 0, texels * kPlanes * sizeof(unsigned long long), st));
            ctx->fixed = static_cast<unsigned long long*>(p);
            ctx->fixed_cap = texels;
        }
        P.fixed = ctx->fixed;
    }
    // Longest-processing-time-first hand-out from the last launch of this band geometry: tiles
    // in descending order of their longest unit chain (tuning schedule 1 = row-major; the summed
    // chains instead: an -DRT_TILE_COST_SUM build, A/B only); this launch records the next costs.
    if (accel != rt::ACCEL_BRUTE) {
        rt::TileSchedule& sc = ctx->sched;
        RT_HIP(rt::schedule_reserve(sc, uint32_t(n_tiles), st));
        const double sched = Tuning::get(ctx->tune.schedule, 0);
        const bool lpt = sched != 1;
        if (lpt && sc.valid) {
            RT_HIP(rt::schedule_order(sc, st));
            P.tile_order = sc.order;
        }
        P.tile_cost = sc.cost[sc.cur];   // zeroed by the launch's prep kernel (-DRT_TILE_COST_SUM
                                         // builds record the tile's summed chains instead of the longest)
    }
    // Head and tail of the LPT order (HASH): the frame's tail is made of the units
    // still running when the queue runs dry, so only the last ranks (the shortest fifth of the
    // tiles) need short units, 2/5 of `chunks` (the count that keeps a uniform split
    // throughput-bound); the head ranks run longer ones, about 12 per lane (a head unit ~1/12 of
    // the frame, so it ends while the tail runs), and only when that is fewer chunks than the
    // tail's (not at 1080p / 1000 spp, whose uniform units are already that long). Config 3:
    // 25 -> 3 head / 10 tail chunks, config 5: 3 -> 1 / 3. A sixth of the units at config 3, so
    // fewer unit starts and flushes, and fewer 64-bit fixed-point atomics, whose memory-side requests are most of the
    // kernel's HBM traffic: 6.6 -> 0.98 GB per frame at -0.6 % frame time (10 tail chunks; 25:
    // 1.6 GB at -0.9 %; profiles/r03_tail_chunks_traffic.txt). Tuning head_chunks / tail_tiles_pm
    // (tail tiles per mille) override; sample_chunks sets the tail count itself.
    uint64_t head_tiles = 0, head_chunks = chunks;
    if (mode == rt::MODE_HASH && chunks > 1 && P.tile_order) {
        const uint64_t pixels = uint64_t(band_width) * band_height;
        head_chunks = std::max<uint64_t>(1, (12u * lanes + pixels - 1) / std::max<uint64_t>(1, pixels));
        // tail units: at most 2.5x the uniform ones, and at least 3x shorter than the head's
        const uint64_t tail_chunks =
            chunks_forced ? chunks : std::max<uint64_t>((chunks * 2 + 4) / 5, std::min<uint64_t>(chunks, 3 * head_chunks));
        head_chunks = uint64_t(Tuning::get(ctx->tune.head_chunks, double(head_chunks)));
        // the last 30 % of the tiles (20 % until round 5: the frame's tail after the queue ran
        // dry 25.5 -> 16.4 ms at config 3, -0.7 %; the N = 8 band with 128-sample units -1.8 %)
        const uint64_t tail_pm = uint64_t(Tuning::get(ctx->tune.tail_tiles_pm, 300));
        head_chunks = std::max<uint64_t>(1, std::min<uint64_t>(head_chunks, tail_chunks));
        const uint64_t tail = std::min<uint64_t>(n_tiles, (n_tiles * std::min<uint64_t>(tail_pm, 1000) + 999) / 1000);
        if (head_chunks < tail_chunks) {
            head_tiles = n_tiles - tail;
            P.chunks = uint32_t(tail_chunks);
        }
    }
    chunks = P.chunks;
    P.head_tiles = uint32_t(head_tiles);
    P.head_chunks = uint32_t(head_tiles ? head_chunks : chunks);
    P.n_units = uint32_t((head_tiles * P.head_chunks + (n_tiles - head_tiles) * chunks) * 64u);
    ctx->last_chunks = P.chunks | (head_tiles ? P.head_chunks << 16 : 0u);
    if (P.tile_cost) {   // this launch's chunk split, for the cost normalisation of the next order
        rt::TileSchedule& sc = ctx->sched;
        sc.rec_head_tiles[sc.cur] = P.head_tiles;
        sc.rec_head_chunks[sc.cur] = P.head_chunks;
        sc.rec_chunks[sc.cur] = P.chunks;
    }
    const uint64_t full = uint64_t(ctx->cu_count) * ctx->occ[accel][ci][mode];
    const uint64_t by_work = (uint64_t(P.n_units) + blk - 1) / blk;
    const int grid = int(std::max<uint64_t>(1, std::min(full, by_work)));
    {   // Block hand-out: the last `reserve` units go out one by one. Measured
        // (scripts/refill_ab.py, 1080p): 0 to 32 Ki are within 1 %, one pixel per lane of the
        // grid (262 Ki) is 10-15 % slower at 13-50 spp.
        const uint64_t reserve = uint64_t(Tuning::get(ctx->tune.refill_reserve, 8192));
        P.n_block_units = P.n_units > reserve ? uint32_t((P.n_units - reserve) & ~uint64_t(63)) : 0u;
        P.first_blocks = uint32_t(std::min<uint64_t>(uint64_t(grid) * blk / 64u, P.n_block_units / 64u));
        // A STREAM frame is as long as its longest pixel chain; the waves that
        // start on the longest-chain tiles of the LPT order take no further work, so no refill of
        // their other lanes slows the chain down. 1/512 of the waves (32 on a full MI355X):
        // 12 spp -3.4 %, 50 spp -3 %, 100 spp +-0 (scripts/env_ab.py isolate_tiles). HASH
        // units are short: no isolation.
        const uint64_t iso = uint64_t(Tuning::get(ctx->tune.isolate_tiles, double(uint64_t(grid) * blk / 64u / 512u)));
        P.isolate_blocks = (P.tile_order && mode == rt::MODE_STREAM) ? uint32_t(std::min<uint64_t>(P.first_blocks, iso)) : 0u;
    }
    if (accel == rt::ACCEL_LBVH_TOP && ctx->treelet_stale) {   // after a build, refit or re-pad
        RT_HIP(rt::build_treelet(d.nodes, d.n_nodes, d.treelet, d.treelet_count, st));
        ctx->treelet_stale = false;
    }
    hipEvent_t* kev = ctx->kev[ctx->kev_count % rt_context::kKernelEvents];
    for (int k = 0; k < 2; k++)
        if (!kev[k]) RT_HIP(hipEventCreate(&kev[k]));
    // counters zeroed, work counter past the first blocks, big-sphere table, tile-cost table zeroed
    RT_HIP(rt::launch_prep(P, P.first_blocks * 64u, ctx->big_tab, P.tile_cost ? uint32_t(n_tiles) : 0u, st));
    P.big_tab = ctx->big_tab;
    RT_HIP(hipEventRecord(kev[0], st));
    RT_HIP(rt::launch_trace(P, accel, count, mode, grid, lds, st));
    RT_HIP(hipEventRecord(kev[1], st));
    ctx->kev_count++;
    if (mode == rt::MODE_HASH)
        RT_HIP(rt::launch_resolve_fixed(ctx->fixed, texels, P.accumulate, spp, accum, out, st));
    if (P.tile_cost && ctx->keep_snaps) {   // this launch's record (+ its order) for rt_launch_row_weights
        rt_context::CostSnap& sn = ctx->snap[(ctx->kev_count - 1) % rt_context::kSnaps];
        if (sn.pending) RT_HIP(hipEventSynchronize(sn.ev));   // four launches old
        sn.pending = false;
        sn.launch = ~0ull;
        if (sn.cap < n_tiles) {
            if (sn.host) RT_HIP(hipHostFree(sn.host));
            sn.host = nullptr;
            sn.cap = 0;
            RT_HIP(hipHostMalloc(reinterpret_cast<void**>(&sn.host), size_t(n_tiles) * 8, hipHostMallocDefault));
            sn.cap = uint32_t(n_tiles);
        }
        if (!sn.ev) RT_HIP(hipEventCreateWithFlags(&sn.ev, hipEventDisableTiming));
        RT_HIP(hipMemcpyAsync(sn.host, P.tile_cost, size_t(n_tiles) * 4, hipMemcpyDeviceToHost, st));
        if (P.tile_order)
            RT_HIP(hipMemcpyAsync(sn.host + n_tiles, P.tile_order, size_t(n_tiles) * 4, hipMemcpyDeviceToHost, st));
        RT_HIP(hipEventRecord(sn.ev, st));
        sn.pending = true;
        sn.launch = ctx->kev_count - 1;
        sn.n = uint32_t(n_tiles);
        sn.tiles_x = uint32_t(tiles_x);
        sn.band_h = band_height;
        sn.head_tiles = P.head_tiles;
        sn.head_chunks = P.head_chunks;
        sn.chunks = P.chunks;
        sn.has_order = P.tile_order != nullptr;
    }
    if (P.tile_cost) {
        ctx->sched.cur ^= 1;
        ctx->sched.valid = true;
    }
    if (ctx->slot_cur >= 0) {   // the next build into this arena waits for this launch
        SceneSlot& sl = ctx->slot[ctx->slot_cur];
        RT_HIP(hipEventRecord(sl.ev_free, st));
        sl.used = true;
    }
    return mark_issued(ctx, st);
}

int rt_get_stats(rt_context* ctx, rt_stats* out) {
    if (!ctx || !out) return fail(RT_ERR_INVALID_ARGUMENT, "ctx or out is NULL");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    out->segments = c.segments;
    out->samples = c.samples;
    out->box_tests = c.box_tests;
    out->sphere_tests = c.sphere_tests;
    return RT_OK;
}

int rt_resolve_rgba8(rt_context* ctx, const float* accum, uint64_t n_texels, uint32_t spp, uint8_t* out,
                     void* stream) {
    if (!ctx) return fail(RT_ERR_INVALID_ARGUMENT, "ctx is NULL");
    if (n_texels == 0) return RT_OK;
    if (!accum || !out) return fail(RT_ERR_INVALID_ARGUMENT, "accum or out is NULL");
    // spp 0 is accepted: the same expression as the trace kernel's store of a 0-sample frame, so
    // a multi-device frame resolves to the bytes a one-device render stores
    DeviceGuard g(ctx->device);
    RT_HIP(rt::launch_tonemap(accum, n_texels, spp, out, static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int rt_scatter_rows(rt_context* ctx, const float* src_accum, const uint8_t* src_rgba8,
                    const uint32_t* rows, uint32_t n_rows, uint32_t width, uint32_t dst_rows, float* dst_accum,
                    uint8_t* dst_rgba8, void* stream) {
    if (!ctx || !rows) return fail(RT_ERR_INVALID_ARGUMENT, "ctx or rows is NULL");
    if ((dst_accum && !src_accum) || (dst_rgba8 && !src_rgba8))
        return fail(RT_ERR_INVALID_ARGUMENT, "source missing for a destination");
    DeviceGuard g(ctx->device);
    RT_HIP(rt::launch_scatter_rows(src_accum, src_rgba8, rows, n_rows, width, dst_rows, dst_accum, dst_rgba8,
                                   static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int rt_gather_rows(rt_context* ctx, const float* src_accum, const uint32_t* rows, uint32_t n_rows, uint32_t width,
                   uint32_t src_rows, float* dst_accum, void* stream) {
    if (!ctx || !rows) return fail(RT_ERR_INVALID_ARGUMENT, "ctx or rows is NULL");
    if (n_rows && width && (!src_accum || !dst_accum)) return fail(RT_ERR_INVALID_ARGUMENT, "accum is NULL");
    DeviceGuard g(ctx->device);
    RT_HIP(rt::launch_gather_rows(src_accum, rows, n_rows, width, src_rows, dst_accum,
                                  static_cast<hipStream_t>(stream)));
    return RT_OK;
}

// Diagnostic export: per-code-point lane utilisation of the last launch (RT_UTIL builds; zeros
// otherwise).
int rt_debug_util(rt_context* ctx, uint64_t* out32) {
    if (!ctx || !out32) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int k = 0; k < 32; k++) out32[k] = c.util[k];
    return RT_OK;
}

// Diagnostic export: phase cycle sums of the last launch (RT_STAMPS builds; zeros otherwise).
int rt_debug_stamps(rt_context* ctx, uint64_t* out8) {
    if (!ctx || !out8) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int k = 0; k < 8; k++) out8[k] = c.stamp[k];
    if (!c.stamp[0] && !c.stamp[1]) out8[6] = c.wave_iters;   // non-stamp builds: walk iterations
    return RT_OK;
}

int rt_debug_tile_cost(rt_context* ctx, uint32_t* out, uint64_t capacity, uint64_t* count) {
    if (!ctx || !count) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    const rt::TileSchedule& sc = ctx->sched;
    *count = sc.valid ? sc.n : 0;
    if (!sc.valid || !out) return RT_OK;   // size query
    if (capacity < sc.n) return fail(RT_ERR_INVALID_ARGUMENT, "capacity");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    RT_HIP(hipMemcpy(out, sc.cost[sc.cur ^ 1], size_t(sc.n) * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_lane_hist(rt_context* ctx, uint64_t* out68) {
    if (!ctx || !out68) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    std::memcpy(out68, c.lane_hist, sizeof(c.lane_hist));
    out68[65] = c.t_first;
    out68[66] = c.t_dry;
    out68[67] = c.t_last;
    return RT_OK;
}

int rt_debug_steals(rt_context* ctx, uint64_t* out) {
    if (!ctx || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    *out = c.steals;
    return RT_OK;
}

// Diagnostic export: walk work of the last COUNT launch split by primary / bounce segments
// (rt_internal.h Counters::walk_split).
int rt_debug_walk_split(rt_context* ctx, uint64_t* out4) {
    if (!ctx || !out4) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    std::memcpy(out4, c.walk_split, sizeof(c.walk_split));
    return RT_OK;
}

// Diagnostic export: of the last COUNT launch of a grid walk, {cells visited, visited cells without
// references} (the decision metric of an occupancy bitmap).
int rt_debug_grid_cells(rt_context* ctx, uint64_t* out2) {
    if (!ctx || !out2) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    out2[0] = c.box_tests;
    out2[1] = c.cells_empty;
    return RT_OK;
}

// Diagnostic export: walk-length histogram of the last COUNT launch (2 x 64 bins: miss, hit).
int rt_debug_walk_hist(rt_context* ctx, uint64_t* out128) {
    if (!ctx || !out128) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    if (int rc = sync_issued(ctx)) return rc;
    rt::Counters c;
    RT_HIP(hipMemcpy(&c, ctx->counters, sizeof(c), hipMemcpyDeviceToHost));
    std::memcpy(out128, c.walk_hist, sizeof(c.walk_hist));
    return RT_OK;
}

int rt_debug_kernel_times(rt_context* ctx, float* out_ms, uint32_t capacity, uint32_t* count) {
    if (!ctx || !count || (!out_ms && capacity)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    DeviceGuard g(ctx->device);
    const uint64_t have = std::min<uint64_t>(ctx->kev_count, rt_context::kKernelEvents);
    const uint32_t n = uint32_t(std::min<uint64_t>(have, capacity));
    for (uint32_t i = 0; i < n; i++) {   // the n most recent launches, oldest first
        hipEvent_t* e = ctx->kev[(ctx->kev_count - n + i) % rt_context::kKernelEvents];
        RT_HIP(hipEventSynchronize(e[1]));
        RT_HIP(hipEventElapsedTime(&out_ms[i], e[0], e[1]));
    }
    *count = n;
    return RT_OK;
}

// Per-row work of ctx's launch `back` launches before its most recent one, from its tile-cost
// record (copied to pinned memory after the kernel once a caller has asked for weights): waits for
// that copy only. The cross-device balancer of rt_multi / rtvk.dist splits a band's measured time
// over its rows with it.
int rt_launch_row_weights(rt_context* ctx, uint32_t back, double* weights, uint32_t band_rows) {
    if (!ctx || (!weights && band_rows)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    rt::keep_row_weights(ctx);   // from now on, even when this call finds nothing
    if (back >= ctx->kev_count) return fail(RT_ERR_INVALID_ARGUMENT, "no such launch recorded");
    std::vector<double> w;
    if (int rc = rt::launch_row_weights(ctx, ctx->kev_count - 1 - back, w)) return rc;
    if (w.size() != band_rows) return fail(RT_ERR_INVALID_ARGUMENT, "band_rows differs from the launch's band");
    std::copy(w.begin(), w.end(), weights);
    return RT_OK;
}

// Trace-kernel duration of ctx's launch `back` launches before its most recent one: waits for
// that launch's end event only, so a caller reading a launch two frames old does not drain the
// frames queued behind it.
int rt_launch_ms(rt_context* ctx, uint32_t back, float* ms) {
    if (!ctx || !ms) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (back >= ctx->kev_count || back >= rt_context::kKernelEvents)
        return fail(RT_ERR_INVALID_ARGUMENT, "no such launch recorded");
    return rt::launch_ms_at(ctx, ctx->kev_count - 1 - back, ms);
}

}  // extern "C"

namespace rt {
uint64_t launch_count(const rt_context* ctx) { return ctx ? ctx->kev_count : 0; }
void keep_row_weights(rt_context* ctx) {
    if (ctx) ctx->keep_snaps = true;
}
int launch_row_weights(rt_context* ctx, uint64_t index, std::vector<double>& w) {
    w.clear();
    if (!ctx) return fail(RT_ERR_INVALID_ARGUMENT, "ctx is NULL");
    ctx->keep_snaps = true;   // the launches from now on keep their records
    for (rt_context::CostSnap& sn : ctx->snap) {
        if (sn.launch != index || !sn.pending) continue;
        DeviceGuard g(ctx->device);
        RT_HIP(hipEventSynchronize(sn.ev));
        // a tile's record is its longest unit chain; x the chunk count of the rank it ran at (the
        // LPT head / tail split) it estimates its longest pixel's chain, the key the LPT order uses
        std::vector<uint32_t> rank;
        if (sn.has_order && sn.head_tiles) {
            rank.assign(sn.n, 0u);
            for (uint32_t r = 0; r < sn.n; r++)
                if (sn.host[sn.n + r] < sn.n) rank[sn.host[sn.n + r]] = r;
        }
        const uint32_t tiles_y = sn.tiles_x ? sn.n / sn.tiles_x : 0;
        std::vector<double> tile_row(tiles_y, 0.0);
        for (uint32_t t = 0; t < sn.n && sn.tiles_x; t++) {
            const double mult = rank.empty() ? 1.0 : double(rank[t] < sn.head_tiles ? sn.head_chunks : sn.chunks);
            if (t / sn.tiles_x < tiles_y) tile_row[t / sn.tiles_x] += double(sn.host[t]) * mult;
        }
        w.assign(sn.band_h, 0.0);
        for (uint32_t i = 0; i < sn.band_h; i++) {
            const uint32_t ty = i / 8u;
            const uint32_t rows_in = std::min<uint32_t>(8u, sn.band_h - ty * 8u);
            if (ty < tiles_y) w[i] = tile_row[ty] / double(rows_in);
        }
        return RT_OK;
    }
    return fail(RT_ERR_INVALID_ARGUMENT, "no tile-cost record kept for that launch");
}
int launch_ms_at(rt_context* ctx, uint64_t index, float* ms) {
    if (!ctx || !ms) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (index >= ctx->kev_count || ctx->kev_count - index > rt_context::kKernelEvents)
        return fail(RT_ERR_INVALID_ARGUMENT, "launch not recorded");
    DeviceGuard g(ctx->device);
    hipEvent_t* e = ctx->kev[index % rt_context::kKernelEvents];
    RT_HIP(hipEventSynchronize(e[1]));
    RT_HIP(hipEventElapsedTime(ms, e[0], e[1]));
    return RT_OK;
}
}  // namespace rt

extern "C" {

#ifndef RT_BUILD_ARCH
#define RT_BUILD_ARCH "unknown"
#endif
#ifndef RT_BUILD_FLAGS
#define RT_BUILD_FLAGS "unknown"
#endif
#ifndef RT_BUILD_VARIANT
#define RT_BUILD_VARIANT ""
#endif
// The Makefile passes the real architecture, device flags and the variant flags of an A/B build
// (make variant VFLAGS=...), so a variant never reports itself as the shipped build.
const char* rt_build_info(void) {
    return "sources_sha256=" RT_SOURCES_SHA256 ";arch=" RT_BUILD_ARCH ";flags=" RT_BUILD_FLAGS
           ";variant=" RT_BUILD_VARIANT;
}

int rt_debug_tune(rt_context* ctx, const char* key, double value) {
    if (!ctx || !key) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    static const struct { const char* name; double Tuning::*field; } kKeys[] = {
        {"grid", &Tuning::grid}, {"grid_scale", &Tuning::grid_scale}, {"grid_coop", &Tuning::grid_coop},
        {"grid_cq", &Tuning::grid_cq},
        {"grid_rec", &Tuning::grid_rec}, {"grid_full_slack", &Tuning::grid_full_slack},
        {"units_per_lane", &Tuning::units_per_lane}, {"unit_min_samples", &Tuning::unit_min_samples},
        {"sample_chunks", &Tuning::sample_chunks}, {"head_chunks", &Tuning::head_chunks},
        {"tail_tiles_pm", &Tuning::tail_tiles_pm}, {"schedule", &Tuning::schedule},
        {"refill_reserve", &Tuning::refill_reserve}, {"isolate_tiles", &Tuning::isolate_tiles},
        {"sah_knobs", &Tuning::sah_knobs}};
    if (!(value >= 0.0 || value == Tuning::kUnset))
        return fail(RT_ERR_INVALID_ARGUMENT, "tuning values are >= 0 (-1 restores the default)");
    for (const auto& k : kKeys) {
        if (std::strcmp(k.name, key) == 0) {
            ctx->tune.*(k.field) = value;
            return RT_OK;
        }
    }
    return fail(RT_ERR_INVALID_ARGUMENT, std::string("unknown tuning key ") + key);
}

int rt_debug_launch_info(rt_context* ctx, uint32_t* out4) {
    if (!ctx || !out4) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    out4[0] = ctx->last_chunks;
    if (ctx->last_accel) {   // the kernel form the last launch actually ran
        out4[1] = ctx->last_accel | (ctx->last_flat ? 0x10000u : 0u) | (ctx->last_pinhole ? 0x20000u : 0u);
        out4[2] = uint32_t(ctx->last_lds);
    } else {   // no launch yet: the default form of the current scene (camera within its pad radius)
        size_t lds = 0;
        out4[1] = choose_accel(ctx, false, 0u, 0.0f, &lds);
        out4[2] = uint32_t(lds);
    }
    out4[3] = uint32_t(ctx->cu_count);
    return RT_OK;
}

int rt_debug_scene(rt_context* ctx, uint32_t what, void* out, uint64_t capacity, uint64_t* bytes) {
    if (!ctx || !bytes) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    const rt::DeviceScene& d = ctx->scene;
    DeviceGuard g(ctx->device);
    RT_HIP(hipDeviceSynchronize());
    if (what == 8) {
        struct { uint32_t n_spheres, n_big, n_nodes, n_leaf, gpu, z; float rmax, R; } info{
            d.n_spheres, d.n_big, d.n_nodes, d.n_leaf, ctx->gpu_tree ? 1u : 0u, 0u, d.small_rmax, ctx->scene_radius};
        *bytes = sizeof(info);
        if (!out || capacity < sizeof(info)) return fail(RT_ERR_INVALID_ARGUMENT, "capacity too small");
        std::memcpy(out, &info, sizeof(info));
        return RT_OK;
    }
    if (what == 9) {   // the uniform grid's layout (all 0 without a grid)
        const rt::GridInfo gi = ctx->has_grid ? d.grid : rt::GridInfo{};
        const uint32_t info[5] = {gi.n[0], gi.n[1], gi.n[2], gi.n_cells, gi.n_refs};
        *bytes = sizeof(info);
        if (!out || capacity < sizeof(info)) return fail(RT_ERR_INVALID_ARGUMENT, "capacity too small");
        std::memcpy(out, info, sizeof(info));
        return RT_OK;
    }
    const void* src = nullptr;
    size_t n = 0;
    switch (what) {
        case 0: src = d.geom; n = size_t(d.n_spheres) * sizeof(rt::GeomRec); break;
        case 1: src = d.radius; n = size_t(d.n_spheres) * 4; break;
        case 2: src = d.mat; n = size_t(d.n_spheres) * sizeof(rt::MatRec); break;
        case 3: src = d.big_ids; n = size_t(d.n_big) * 4; break;
        case 4: src = d.nodes; n = size_t(d.n_nodes) * sizeof(rt::BvhNode); break;
        case 5: src = ctx->gpu_tree ? d.nodes_raw : nullptr; n = size_t(d.n_nodes) * sizeof(rt::BvhNode); break;
        case 6: src = d.leaf_geom; n = size_t(d.n_leaf) * sizeof(rt::GeomRec); break;
        case 7: src = d.leaf_ids; n = size_t(d.n_leaf) * 4; break;
        default: return fail(RT_ERR_INVALID_ARGUMENT, "unknown scene array");
    }
    *bytes = n;
    if (n == 0) return RT_OK;
    if (!out || capacity < n) return fail(RT_ERR_INVALID_ARGUMENT, "capacity too small");
    if (what == 5 && !ctx->gpu_tree) {   // host-built: the unpadded boxes live on the host
        std::memcpy(out, ctx->nodes_host.data(), n);
        return RT_OK;
    }
    RT_HIP(hipMemcpy(out, src, n, hipMemcpyDeviceToHost));
    return RT_OK;
}

// Diagnostic export for the parity tests: evaluates a contract primitive on the device.
int rt_debug_math(int device, int op, const float* in_pairs, float* out, uint32_t n) {
    if (!in_pairs || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL buffer");
    int nd = 0;
    if (int rc = rt::current_device_count(&nd)) return rc;
    if (device < 0 || device >= nd) return fail(RT_ERR_INVALID_ARGUMENT, "device index out of range");
    DeviceGuard g(device);
    float *din = nullptr, *dout = nullptr;
    RT_HIP(hipMalloc(&din, size_t(n) * 2 * sizeof(float) + 16));
    RT_HIP(hipMalloc(&dout, size_t(n) * sizeof(float) + 16));
    RT_HIP(hipMemcpy(din, in_pairs, size_t(n) * 2 * sizeof(float), hipMemcpyHostToDevice));
    RT_HIP(rt::launch_debug_math(op, din, dout, n, nullptr));
    RT_HIP(hipMemcpy(out, dout, size_t(n) * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(din);
    (void)hipFree(dout);
    return RT_OK;
}

int rt_debug_exact_exhaustive(int device, uint64_t* mismatches3) {
    if (!mismatches3) return fail(RT_ERR_INVALID_ARGUMENT, "NULL buffer");
    int nd = 0;
    if (int rc = rt::current_device_count(&nd)) return rc;
    if (device < 0 || device >= nd) return fail(RT_ERR_INVALID_ARGUMENT, "device index out of range");
    DeviceGuard g(device);
    unsigned long long* bad = nullptr;
    RT_HIP(hipMalloc(&bad, 3 * sizeof(unsigned long long)));
    RT_HIP(hipMemset(bad, 0, 3 * sizeof(unsigned long long)));
    RT_HIP(rt::launch_debug_exact(bad, nullptr));
    unsigned long long h[3] = {0, 0, 0};
    RT_HIP(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(bad);
    for (int k = 0; k < 3; k++) mismatches3[k] = h[k];
    return RT_OK;
}

int rt_store_ppm(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height) {
    if (!path || !rgba8) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_ERR_IO, std::string("cannot open ") + path);
    std::fprintf(f, "P6\n%u %u\n255\n", width, height);
    std::vector<uint8_t> row(size_t(width) * 3);
    bool ok = true;
    for (uint32_t y = 0; y < height && ok; y++) {
        for (uint32_t x = 0; x < width; x++)
            for (int c = 0; c < 3; c++) row[size_t(x) * 3 + c] = rgba8[(size_t(y) * width + x) * 4 + c];
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_OK : fail(RT_ERR_IO, std::string("write failed: ") + path);
}

}  // extern "C"
