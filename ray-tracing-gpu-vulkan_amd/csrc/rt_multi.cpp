// rt_multi.cpp — one process driving N GPUs: the multi-device frame over RCCL (rt_multi_*),
// the host-buffer frame rt_render(), and the reference's entry point ray_trace().
//
// The reference creates one Vulkan device per GPU (src/ray_trace.cpp:42-105), gives each a
// contiguous row band (:74-93, tuned by src/workload_tuner.hpp) and never moves pixels between
// GPUs (each device presents its own window). Here the image is tiled into 8-row strips dealt
// round robin over the devices (interleaving balances sky-heavy and sphere-heavy rows without a
// tuner), each device renders its strips through a rows map (global pixel seeds, so the image
// does not depend on the device count), one RCCL group moves every other device's float4
// accumulator strips to device 0 over xGMI (ncclSend / ncclRecv; device 0's own strips are not
// sent), one kernel per source puts them in place (rt_scatter_rows) and device 0 tonemaps the
// whole accumulator to rgba8 once (rt_resolve_rgba8: the rgba8 bytes are a function of the float
// sum, shader.rgen:65-66, so they need not travel). A single device holding every row renders
// straight into the caller's buffers. SURVEY.md §8(e).
//
// A frame is a FramePlan: the partition (device + global rows per part) and the ordered list of
// steps (row loads / stores on device 0, grouped sends / receives, renders, the resolve) that
// rt_multi_render executes. The plan is host-only data, so the CPU tests check it for every device
// count and height without a GPU (rt_debug_multi_plan, tests/test_multi_plan.py).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rt_abi.h"
#include "../../include/rt_mi355x.h"
#include "../../include/rt_mi355x_debug.h"
#include "rt_host.h"
#include "rt_internal.h"

using rt::DeviceGuard;
using rt::fail;

#define RT_NCCL(call)                                                                       \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess)                                                              \
            return fail(RT_ERR_DEVICE, std::string(#call) + ": " + ncclGetErrorString(r_));  \
    } while (0)

namespace {

constexpr uint32_t kStrip = 8;   // rows per strip: one 8x8 pixel tile high, the kernel's wave tile

// ---- the frame plan ----------------------------------------------------------------------
// Buffers a step names: the caller's accumulator / rgba8 image on device 0 (W x H), each part's
// band on its device (rows x W), and each remote part's stage on device 0 (rows x W float4).
enum PlanOp : uint32_t {
    OP_LOAD_ROWS = 1,   // device 0: the part's rows of the caller's accumulator -> its band (a part
                        // of device 0) or its stage (accumulating frames: the running sums)
    OP_GROUP_START = 2, // ncclGroupStart
    OP_SEND = 3,        // dev -> peer: `count` floats of the part's band (dev != 0) or stage (dev 0)
    OP_RECV = 4,        // dev <- peer: `count` floats into the part's band (dev != 0) or stage (dev 0)
    OP_GROUP_END = 5,   // ncclGroupEnd
    OP_RENDER = 6,      // dev renders the part; flags bit 0: straight into the caller's buffers
    OP_STORE_ROWS = 7,  // device 0: the part's band (device 0) or stage -> its rows of the accumulator
    OP_RESOLVE = 8,     // device 0: rgba8 of the whole accumulator (`count` texels)
};
constexpr uint32_t kDirect = 1u;

struct PlanPart {
    uint32_t dev = 0;
    std::vector<uint32_t> rows;   // global rows, band order
    bool whole = false;           // device 0, every row in order: renders into the caller's buffers
};
struct PlanStep {
    uint32_t op, dev, peer, part, flags;
    uint64_t count;
};
struct FramePlan {
    std::vector<PlanPart> parts;
    std::vector<PlanStep> steps;
};
using Parts = std::vector<std::pair<uint32_t, std::vector<uint32_t>>>;

// Strips k = 0, 1, ... of kStrip rows, strip k on device k % n (rtvk.dist.strip_rows).
Parts strip_parts(uint32_t n, uint32_t H) {
    Parts parts(n);
    for (uint32_t d = 0; d < n; d++) parts[d].first = d;
    for (uint32_t y = 0; y < H; y++) parts[(y / kStrip) % n].second.push_back(y);
    return parts;
}

// The reference's contiguous bands (src/ray_trace.cpp:74-93): band i = rows [start[i], start[i+1])
// (the last to H), on device i % n. Empty when the starts do not tile [0, H) top to bottom.
Parts band_parts(uint32_t n, uint32_t H, const uint32_t* start, uint32_t n_bands) {
    Parts parts(n_bands);
    for (uint32_t i = 0; i < n_bands; i++) {
        const uint32_t y0 = start[i], y1 = i + 1 < n_bands ? start[i + 1] : H;
        if (y1 < y0 || y1 > H || (i == 0 && y0 != 0)) return Parts{};
        parts[i].first = i % n;
        for (uint32_t y = y0; y < y1; y++) parts[i].second.push_back(y);
    }
    return parts;
}

// The steps of one frame over `parts` (W x H). accumulate: every part starts from its rows of the
// caller's accumulator (rt_render_device's accumulate semantics for the whole image, at any
// device count): device 0 loads them into its own bands and into the stages of the other
// devices' parts, and sends those in one group. Then every part renders; one group brings the
// other devices' accumulator bands to device 0's stages; device 0 stores every band in place and
// tonemaps the whole image. A part of device 0 never goes through RCCL; a `whole` part renders
// into the caller's buffers and needs nothing else (the one-device frame).
FramePlan make_plan(uint32_t W, uint32_t H, Parts&& parts, bool accumulate) {
    FramePlan p;
    for (auto& pr : parts) {
        PlanPart q;
        q.dev = pr.first;
        q.rows = std::move(pr.second);
        q.whole = q.dev == 0 && q.rows.size() == H;
        for (uint32_t y = 0; q.whole && y < H; y++) q.whole = q.rows[y] == y;
        p.parts.push_back(std::move(q));
    }
    const uint32_t np = uint32_t(p.parts.size());
    auto live = [&](uint32_t i) { return !p.parts[i].rows.empty(); };
    auto floats = [&](uint32_t i) { return uint64_t(p.parts[i].rows.size()) * W * 4u; };
    auto add = [&](uint32_t op, uint32_t dev, uint32_t peer, uint32_t part, uint32_t flags, uint64_t count) {
        p.steps.push_back(PlanStep{op, dev, peer, part, flags, count});
    };
    bool whole = false, remote = false;
    for (uint32_t i = 0; i < np; i++) {
        whole |= live(i) && p.parts[i].whole;
        remote |= live(i) && p.parts[i].dev != 0;
    }
    if (accumulate && !whole) {
        for (uint32_t i = 0; i < np; i++)
            if (live(i)) add(OP_LOAD_ROWS, 0, 0, i, 0, floats(i));
        if (remote) {
            add(OP_GROUP_START, 0, 0, 0, 0, 0);
            for (uint32_t i = 0; i < np; i++) {
                if (!live(i) || p.parts[i].dev == 0) continue;
                add(OP_SEND, 0, p.parts[i].dev, i, 0, floats(i));
                add(OP_RECV, p.parts[i].dev, 0, i, 0, floats(i));
            }
            add(OP_GROUP_END, 0, 0, 0, 0, 0);
        }
    }
    for (uint32_t i = 0; i < np; i++)
        if (live(i)) add(OP_RENDER, p.parts[i].dev, p.parts[i].dev, i, p.parts[i].whole ? kDirect : 0u, 0);
    if (whole) return p;
    if (remote) {
        add(OP_GROUP_START, 0, 0, 0, 0, 0);
        for (uint32_t i = 0; i < np; i++) {
            if (!live(i) || p.parts[i].dev == 0) continue;
            add(OP_SEND, p.parts[i].dev, 0, i, 0, floats(i));
            add(OP_RECV, 0, p.parts[i].dev, i, 0, floats(i));
        }
        add(OP_GROUP_END, 0, 0, 0, 0, 0);
    }
    for (uint32_t i = 0; i < np; i++)
        if (live(i)) add(OP_STORE_ROWS, 0, 0, i, 0, floats(i));
    add(OP_RESOLVE, 0, 0, 0, 0, uint64_t(W) * H);
    return p;
}

// One part of a multi-device frame on its device (its own context), with its buffers.
struct Launch {
    uint32_t dev = 0;
    std::vector<uint32_t> rows;          // global rows, band order
    bool whole = false;
    rt_context* ctx = nullptr;           // on dev
    uint32_t* rows_dev = nullptr;        // rows on dev (the kernel's map)
    uint32_t* rows_root = nullptr;       // rows on device 0 (the row loads / stores)
    float* acc = nullptr;                // band on dev: rows x W float4 (not for a whole part)
    uint8_t* out = nullptr;              // band on dev: rows x W rgba8 (the kernel's store; not sent)
    float* stage_acc = nullptr;          // dev != 0: the band's copy on device 0
};

}  // namespace

struct rt_multi {
    uint32_t n = 0;
    std::vector<hipStream_t> stream;     // one per device
    std::vector<ncclComm_t> comm;        // one per device, rank = device index
    hipEvent_t ev_in = nullptr, ev_out = nullptr;   // device 0: caller stream <-> stream[0]
    std::vector<Sphere> spheres;         // the scene, for contexts created later
    bool scene_set = false;
    // cached partition (geometry + kind): strips of W x H, or explicit bands
    uint32_t W = 0, H = 0;
    std::string key;
    std::vector<Launch> launches;        // one per plan part, same index
    FramePlan plan[2];                   // steps without / with accumulation
};

namespace {

void free_launches(rt_multi* m) {
    for (Launch& l : m->launches) {
        {
            DeviceGuard g(static_cast<int>(l.dev));
            (void)hipDeviceSynchronize();
            if (l.rows_dev) (void)hipFree(l.rows_dev);
            if (l.acc) (void)hipFree(l.acc);
            if (l.out) (void)hipFree(l.out);
            rt_context_destroy(l.ctx);
        }
        DeviceGuard g0(0);
        (void)hipDeviceSynchronize();
        if (l.rows_root) (void)hipFree(l.rows_root);
        if (l.stage_acc) (void)hipFree(l.stage_acc);
    }
    m->launches.clear();
    m->plan[0] = m->plan[1] = FramePlan{};
    m->key.clear();
}

// The scene on every device: each device's build is issued before any is waited for (device-built
// scenes build on every GPU at once, each beside its previous frame), and a host-built scene is
// built once and uploaded to every device (rt_api.cpp set_scene_begin / set_scene_end).
int set_scene_all(rt_multi* m) {
    rt::HostPackagePtr shared;
    const uint32_t count = uint32_t(m->spheres.size());
    int rc = RT_OK;
    size_t begun = 0;
    for (; begun < m->launches.size(); begun++) {
        Launch& l = m->launches[begun];
        rc = rt::set_scene_begin(l.ctx, m->spheres.data(), count, m->stream[l.dev], &shared);
        if (rc != RT_OK) break;
    }
    for (size_t i = 0; i < begun; i++) {   // every begun build is ended, even after a failure
        const int e = rt::set_scene_end(m->launches[i].ctx);
        if (rc == RT_OK) rc = e;
    }
    return rc;
}

// (Re)builds the launches for `key` from the partition: one per part (device + global rows), its
// context and buffers, and the frame's plans with and without accumulation.
int set_partition(rt_multi* m, const std::string& key, uint32_t W, uint32_t H, Parts&& parts) {
    if (m->key == key && m->W == W && m->H == H) return RT_OK;
    free_launches(m);
    m->W = W;
    m->H = H;
    Parts copy = parts;
    m->plan[0] = make_plan(W, H, std::move(copy), false);
    m->plan[1] = make_plan(W, H, std::move(parts), true);
    for (const PlanPart& q : m->plan[0].parts) {
        Launch l;
        l.dev = q.dev;
        l.rows = q.rows;
        l.whole = q.whole;
        m->launches.push_back(std::move(l));
    }
    for (Launch& l : m->launches) {
        const size_t nr = l.rows.size(), texels = nr * W;
        if (int rc = rt_context_create(int(l.dev), &l.ctx)) return rc;
        if (!nr || l.whole) continue;
        {
            DeviceGuard g(static_cast<int>(l.dev));
            RT_HIP(hipMalloc(&l.rows_dev, nr * 4));
            RT_HIP(hipMemcpy(l.rows_dev, l.rows.data(), nr * 4, hipMemcpyHostToDevice));
            RT_HIP(hipMalloc(&l.acc, texels * 16));
            RT_HIP(hipMalloc(&l.out, texels * 4));
        }
        DeviceGuard g0(0);
        RT_HIP(hipMalloc(&l.rows_root, nr * 4));
        RT_HIP(hipMemcpy(l.rows_root, l.rows.data(), nr * 4, hipMemcpyHostToDevice));
        if (l.dev != 0) RT_HIP(hipMalloc(&l.stage_acc, texels * 16));
    }
    m->key = key;
    return m->scene_set ? set_scene_all(m) : RT_OK;
}

// A context on device 0 (the row loads / stores and the resolve run on stream[0]).
rt_context* root_ctx(rt_multi* m) {
    for (Launch& l : m->launches)
        if (l.dev == 0) return l.ctx;
    return nullptr;
}

// Executes a frame plan: rcis[i] for part i (n_rci == 1: rcis[0] for every part; offsets replaced
// by the rows maps), into the caller's acc / out (device 0, W x H). Every step is queued on its
// device's stream; the stream order of each device and the RCCL groups order them across devices.
int run_plan(rt_multi* m, const FramePlan& p, const RenderCallInfo* rcis, size_t n_rci, const rt_options* opt,
             float* acc, uint8_t* out) {
    const uint32_t W = m->W, H = m->H;
    rt_context* c0 = root_ctx(m);
    bool in_group = false;
    auto body = [&]() -> int {
        for (const PlanStep& s : p.steps) {
            Launch& l = m->launches[s.part];
            float* dev_buf = s.dev == 0 ? l.stage_acc : l.acc;   // a SEND / RECV's buffer on s.dev
            float* root_buf = l.dev == 0 ? l.acc : l.stage_acc;  // the part's accumulator on device 0
            const uint32_t nr = uint32_t(l.rows.size());
            switch (s.op) {
                case OP_GROUP_START:
                    RT_NCCL(ncclGroupStart());
                    in_group = true;
                    break;
                case OP_GROUP_END:
                    in_group = false;
                    RT_NCCL(ncclGroupEnd());
                    break;
                case OP_SEND:
                case OP_RECV: {
                    DeviceGuard g(static_cast<int>(s.dev));
                    const ncclResult_t e =
                        s.op == OP_SEND
                            ? ncclSend(dev_buf, s.count, ncclFloat32, int(s.peer), m->comm[s.dev], m->stream[s.dev])
                            : ncclRecv(dev_buf, s.count, ncclFloat32, int(s.peer), m->comm[s.dev], m->stream[s.dev]);
                    if (e != ncclSuccess) return fail(RT_ERR_DEVICE, std::string("RCCL: ") + ncclGetErrorString(e));
                    break;
                }
                case OP_LOAD_ROWS:
                    if (int rc = rt_gather_rows(c0, acc, l.rows_root, nr, W, H, root_buf, m->stream[0])) return rc;
                    break;
                case OP_STORE_ROWS:
                    if (int rc = rt_scatter_rows(c0, root_buf, nullptr, l.rows_root, nr, W, H, acc, nullptr,
                                                 m->stream[0]))
                        return rc;
                    break;
                case OP_RENDER: {
                    RenderCallInfo r = rcis[n_rci == 1 ? 0 : s.part];
                    r.offset = rt_uvec2{0, 0};   // the rows map carries the global rows
                    const bool d = (s.flags & kDirect) != 0;
                    if (int rc = rt_render_device(l.ctx, &r, d ? nullptr : l.rows_dev, W, nr, d ? acc : l.acc,
                                                  d ? out : l.out, opt, m->stream[l.dev]))
                        return rc;
                    break;
                }
                case OP_RESOLVE:
                    if (int rc = rt_resolve_rgba8(c0, acc, s.count, rcis[0].samplesPerRenderCall, out, m->stream[0]))
                        return rc;
                    break;
                default:
                    return fail(RT_ERR_INVALID_ARGUMENT, "bad plan step");
            }
        }
        return RT_OK;
    };
    const int rc = body();
    if (in_group) (void)ncclGroupEnd();   // a failure inside a group still closes it
    return rc;
}

// Flat form of a plan (rt_debug_multi_plan): {n_parts, n_steps}, then per part {dev, whole,
// n_rows, rows...}, then per step {op, dev, peer, part, flags, count low, count high}.
std::vector<uint32_t> serialize(const FramePlan& p) {
    std::vector<uint32_t> v{uint32_t(p.parts.size()), uint32_t(p.steps.size())};
    for (const PlanPart& q : p.parts) {
        v.push_back(q.dev);
        v.push_back(q.whole ? 1u : 0u);
        v.push_back(uint32_t(q.rows.size()));
        v.insert(v.end(), q.rows.begin(), q.rows.end());
    }
    for (const PlanStep& s : p.steps) {
        const uint32_t w[7] = {s.op, s.dev, s.peer, s.part, s.flags, uint32_t(s.count), uint32_t(s.count >> 32)};
        v.insert(v.end(), w, w + 7);
    }
    return v;
}

}  // namespace

extern "C" {

int rt_multi_create(uint32_t gpu_count, rt_multi** out) {
    if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = nullptr;
    int nd = 0;
    if (int rc = rt::current_device_count(&nd)) return rc;
    rt_multi* m = nullptr;
    try {
        m = new rt_multi();
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    // every failure below releases what was created so far (streams, events, comms)
    auto body = [&]() -> int {
        m->n = std::max(1u, std::min(gpu_count, uint32_t(nd)));
        m->stream.assign(m->n, nullptr);
        m->comm.assign(m->n, nullptr);
        for (uint32_t d = 0; d < m->n; d++) {
            DeviceGuard g(static_cast<int>(d));
            RT_HIP(hipStreamCreateWithFlags(&m->stream[d], hipStreamNonBlocking));
        }
        {
            DeviceGuard g(0);
            RT_HIP(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
            RT_HIP(hipEventCreateWithFlags(&m->ev_out, hipEventDisableTiming));
        }
        // A single device's frame plan holds no send or receive (tests/test_multi_plan.py), so
        // one device needs no communicator: the drop-in ray_trace(..., 1) does not pay RCCL's
        // initialisation on its cold call.
        if (m->n > 1) {
            std::vector<int> devs(m->n);
            for (uint32_t d = 0; d < m->n; d++) devs[d] = int(d);
            RT_NCCL(ncclCommInitAll(m->comm.data(), int(m->n), devs.data()));
        }
        return RT_OK;
    };
    int rc;
    try {
        rc = body();
    } catch (const std::exception& e) {
        rc = fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    if (rc != RT_OK) {
        const std::string msg = rt::g_last_error;   // destroy must not overwrite the cause
        rt_multi_destroy(m);
        rt::g_last_error = msg;
        return rc;
    }
    *out = m;
    return RT_OK;
}

int rt_multi_destroy(rt_multi* m) {
    if (!m) return RT_OK;
    free_launches(m);
    for (uint32_t d = 0; d < m->n; d++) {
        DeviceGuard g(static_cast<int>(d));
        (void)hipDeviceSynchronize();
        if (d < m->comm.size() && m->comm[d]) (void)ncclCommDestroy(m->comm[d]);
        if (d < m->stream.size() && m->stream[d]) (void)hipStreamDestroy(m->stream[d]);
    }
    {
        DeviceGuard g(0);
        if (m->ev_in) (void)hipEventDestroy(m->ev_in);
        if (m->ev_out) (void)hipEventDestroy(m->ev_out);
    }
    delete m;
    return RT_OK;
}

int rt_multi_device_count(const rt_multi* m, uint32_t* n) {
    if (!m || !n) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    *n = m->n;
    return RT_OK;
}

int rt_multi_set_scene(rt_multi* m, const Sphere* spheres, uint32_t count) {
    if (!m) return fail(RT_ERR_INVALID_ARGUMENT, "m is NULL");
    if (!spheres && count) return fail(RT_ERR_INVALID_ARGUMENT, "spheres is NULL");
    try {
        m->spheres.assign(spheres, spheres + count);
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    if (int rc = set_scene_all(m)) return rc;
    m->scene_set = true;
    return RT_OK;
}

int rt_multi_render(rt_multi* m, const RenderCallInfo* rci, const rt_options* opt, float* accum,
                    uint8_t* out, void* stream) {
    if (!m || !rci) return fail(RT_ERR_INVALID_ARGUMENT, "m or rci is NULL");
    if (!m->scene_set) return fail(RT_ERR_NO_SCENE, "rt_multi_render before rt_multi_set_scene");
    const uint32_t W = rci->image_size.x, H = rci->image_size.y;
    if (W == 0 || H == 0) return fail(RT_ERR_INVALID_ARGUMENT, "image_size is zero");
    if (!accum || !out) return fail(RT_ERR_INVALID_ARGUMENT, "accum or out is NULL");
    try {
        if (int rc = set_partition(m, "strips", W, H, strip_parts(m->n, H))) return rc;
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    {   // the frame starts after the caller's earlier work on `stream` (device 0)
        DeviceGuard g0(0);
        RT_HIP(hipEventRecord(m->ev_in, st));
        for (uint32_t d = 0; d < m->n; d++) RT_HIP(hipStreamWaitEvent(m->stream[d], m->ev_in, 0));
    }
    const bool acc_mode = opt && opt->accumulate;
    if (int rc = run_plan(m, m->plan[acc_mode ? 1 : 0], rci, 1, opt, accum, out)) return rc;
    DeviceGuard g0(0);
    RT_HIP(hipEventRecord(m->ev_out, m->stream[0]));   // the caller's later work waits for it
    RT_HIP(hipStreamWaitEvent(st, m->ev_out, 0));
    return RT_OK;
}

int rt_debug_multi_plan(uint32_t n_devices, uint32_t width, uint32_t height, const uint32_t* band_starts,
                        uint32_t n_bands, uint32_t accumulate, uint32_t* out, uint64_t capacity, uint64_t* count) {
    if (!count) return fail(RT_ERR_INVALID_ARGUMENT, "count is NULL");
    *count = 0;
    if (n_devices == 0 || width == 0 || height == 0) return fail(RT_ERR_INVALID_ARGUMENT, "zero size");
    if (band_starts && n_bands == 0) return fail(RT_ERR_INVALID_ARGUMENT, "no bands");
    std::vector<uint32_t> v;
    try {
        Parts parts = band_starts ? band_parts(n_devices, height, band_starts, n_bands) : strip_parts(n_devices, height);
        if (parts.empty()) return fail(RT_ERR_INVALID_ARGUMENT, "bands must tile the image top to bottom");
        v = serialize(make_plan(width, height, std::move(parts), accumulate != 0));
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    *count = v.size();
    if (!out) return RT_OK;   // size query
    if (capacity < v.size()) return fail(RT_ERR_INVALID_ARGUMENT, "capacity");
    std::memcpy(out, v.data(), v.size() * 4);
    return RT_OK;
}

int rt_multi_info(const rt_multi* m, uint32_t* out4) {
    if (!m || !out4) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    int ranks = 0;   // 0: one device, no communicator
    if (m->comm[0]) RT_NCCL(ncclCommCount(m->comm[0], &ranks));
    uint32_t launches = 0;
    for (const Launch& l : m->launches) launches += l.rows.empty() ? 0u : 1u;
    out4[0] = m->n;
    out4[1] = uint32_t(ranks);
    out4[2] = kStrip;
    out4[3] = launches;
    return RT_OK;
}

int rt_multi_kernel_times(rt_multi* m, float* out_ms, uint32_t capacity, uint32_t* count) {
    if (!m || !count || (!out_ms && capacity)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    uint32_t k = 0;
    for (Launch& l : m->launches) {
        if (l.rows.empty()) continue;
        if (k >= capacity) break;
        uint32_t got = 0;
        if (int rc = rt_debug_kernel_times(l.ctx, out_ms + k, 1, &got)) return rc;
        if (got == 0) out_ms[k] = 0.0f;
        k++;
    }
    *count = k;
    return RT_OK;
}

int rt_multi_kernel_times_frames(rt_multi* m, uint32_t frames, float* out_ms, uint32_t capacity, uint32_t* count) {
    if (!m || !count || (!out_ms && capacity)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    std::vector<Launch*> ls;
    for (Launch& l : m->launches)
        if (!l.rows.empty()) ls.push_back(&l);
    const uint32_t n = uint32_t(ls.size());
    if (uint64_t(frames) * n > capacity) return fail(RT_ERR_INVALID_ARGUMENT, "capacity below frames x devices");
    std::vector<float> t(frames);
    for (uint32_t d = 0; d < n; d++) {
        uint32_t got = 0;
        if (int rc = rt_debug_kernel_times(ls[d]->ctx, t.data(), frames, &got)) return rc;
        if (got < frames) return fail(RT_ERR_INVALID_ARGUMENT, "fewer launches recorded than frames asked");
        for (uint32_t f = 0; f < frames; f++) out_ms[size_t(f) * n + d] = t[f];
    }
    *count = frames * n;
    return RT_OK;
}

int rt_multi_stats(rt_multi* m, rt_stats* out) {
    if (!m || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    for (Launch& l : m->launches) {
        if (l.rows.empty()) continue;
        rt_stats s;
        if (int rc = rt_get_stats(l.ctx, &s)) return rc;
        out->segments += s.segments;
        out->samples += s.samples;
        out->box_tests += s.box_tests;
        out->sphere_tests += s.sphere_tests;
    }
    return RT_OK;
}

// Host-buffer frame: the reference's contiguous bands (one per RenderCallInfo, band i on device
// i % n), gathered to device 0 by the same RCCL path, then copied to the host.
int rt_render(const Sphere* spheres, uint32_t sphere_count, const RenderCallInfo* rci, uint32_t rci_count,
              float* accum, uint8_t* out, const rt_options* opt, rt_stats* stats) {
    if (!rci || rci_count == 0) return fail(RT_ERR_INVALID_ARGUMENT, "no RenderCallInfo");
    if (!accum || !out) return fail(RT_ERR_INVALID_ARGUMENT, "accum or out is NULL");
    const uint32_t W = rci[0].image_size.x, H = rci[0].image_size.y;
    if (W == 0 || H == 0) return fail(RT_ERR_INVALID_ARGUMENT, "image_size is zero");
    for (uint32_t i = 0; i < rci_count; i++) {
        const uint32_t y0 = rci[i].offset.y;
        const uint32_t y1 = (i + 1 < rci_count) ? rci[i + 1].offset.y : H;
        if (rci[i].image_size.x != W || rci[i].image_size.y != H || rci[i].offset.x != 0 || y1 < y0 || y1 > H ||
            (i == 0 && y0 != 0))
            return fail(RT_ERR_INVALID_ARGUMENT, "bands must tile the image top to bottom");
        // device 0 tonemaps the gathered image once (rt_resolve_rgba8), with one spp
        if (rci[i].samplesPerRenderCall != rci[0].samplesPerRenderCall)
            return fail(RT_ERR_INVALID_ARGUMENT, "every band must have the same samplesPerRenderCall");
    }
    rt_multi* m = nullptr;
    if (int rc = rt_multi_create(rci_count, &m)) return rc;
    std::unique_ptr<rt_multi, int (*)(rt_multi*)> guard(m, rt_multi_destroy);
    float* dacc = nullptr;
    uint8_t* dout = nullptr;
    auto run = [&]() -> int {
        if (int rc = rt_multi_set_scene(m, spheres, sphere_count)) return rc;
        std::vector<uint32_t> starts(rci_count);
        for (uint32_t i = 0; i < rci_count; i++) starts[i] = rci[i].offset.y;
        if (int rc = set_partition(m, "bands", W, H, band_parts(m->n, H, starts.data(), rci_count))) return rc;
        DeviceGuard g0(0);
        RT_HIP(hipMalloc(&dacc, size_t(W) * H * 16));
        RT_HIP(hipMalloc(&dout, size_t(W) * H * 4));
        const bool acc_mode = opt && opt->accumulate;
        if (acc_mode)   // every band starts from its rows of the host accumulator
            RT_HIP(hipMemcpyAsync(dacc, accum, size_t(W) * H * 16, hipMemcpyHostToDevice, m->stream[0]));
        // each band its own RenderCallInfo
        if (int rc = run_plan(m, m->plan[acc_mode ? 1 : 0], rci, rci_count, opt, dacc, dout)) return rc;
        RT_HIP(hipStreamSynchronize(m->stream[0]));
        RT_HIP(hipMemcpy(accum, dacc, size_t(W) * H * 16, hipMemcpyDeviceToHost));
        RT_HIP(hipMemcpy(out, dout, size_t(W) * H * 4, hipMemcpyDeviceToHost));
        if (stats) {
            std::memset(stats, 0, sizeof(*stats));
            for (Launch& l : m->launches) {
                if (l.rows.empty()) continue;
                rt_stats s;
                if (int rc = rt_get_stats(l.ctx, &s)) return rc;
                stats->segments += s.segments;
                stats->samples += s.samples;
                stats->box_tests += s.box_tests;
                stats->sphere_tests += s.sphere_tests;
            }
        }
        return RT_OK;
    };
    int rc;
    try {
        rc = run();
    } catch (const std::exception& e) {
        rc = fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    DeviceGuard g0(0);
    if (dacc) (void)hipFree(dacc);
    if (dout) (void)hipFree(dout);
    return rc;
}

// src/ray_trace.h:9-15. Headless: one frame of the canonical scene (t = 0) tiled over
// min(gpu_count, visible) GPUs (rt_multi). Random stream: the reference's per-pixel LCG stream, or
// with RT_RNG=hash in the environment the counter-based RT_RNG_SAMPLE_HASH stream, whose samples
// split into chunks so that every GPU stays throughput-bound (the reference signature has no
// parameter for it, so the selection travels out of band).
void ray_trace(uint32_t samples, bool storeRenderResult, uint32_t width, uint32_t height, uint32_t gpu_count) {
    auto report = [](const char* what) { std::fprintf(stderr, "ray_trace: %s: %s\n", what, rt::g_last_error.c_str()); };
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    try {
        const auto t_c = clk::now();
        rt_multi* m = nullptr;
        if (rt_multi_create(gpu_count, &m)) return report("rt_multi_create");
        std::unique_ptr<rt_multi, int (*)(rt_multi*)> guard(m, rt_multi_destroy);
        const double create_ms = ms_since(t_c);
        const auto t_s = clk::now();
        std::vector<Sphere> scene(488);
        uint32_t cnt = 0;
        rt_generate_scene(0.0f, 11, scene.data(), uint32_t(scene.size()), &cnt);
        if (rt_multi_set_scene(m, scene.data(), cnt)) return report("rt_multi_set_scene");
        const double scene_ms = ms_since(t_s);
        RenderCallInfo rci;
        rt_canonical_render_call_info(samples, width, height, &rci);
        rt_options opt;
        std::memset(&opt, 0, sizeof(opt));
        opt.rng_mode = RT_RNG_PIXEL_STREAM;
        if (const char* e = std::getenv("RT_RNG")) {
            if (std::strcmp(e, "hash") == 0) opt.rng_mode = RT_RNG_SAMPLE_HASH;
            else if (std::strcmp(e, "stream") != 0) {
                std::fprintf(stderr, "ray_trace: RT_RNG must be 'stream' or 'hash', got '%s'\n", e);
                return;
            }
        }
        DeviceGuard g0(0);
        float* dacc = nullptr;
        uint8_t* dout = nullptr;
        if (hipMalloc(&dacc, size_t(width) * height * 16) != hipSuccess ||
            hipMalloc(&dout, size_t(width) * height * 4) != hipSuccess) {
            std::fprintf(stderr, "ray_trace: out of device memory\n");
            if (dacc) (void)hipFree(dacc);
            return;
        }
        (void)hipDeviceSynchronize();
        const auto t0 = std::chrono::steady_clock::now();
        int rc = rt_multi_render(m, &rci, &opt, dacc, dout, nullptr);
        if (rc == RT_OK) rc = hipDeviceSynchronize() == hipSuccess ? RT_OK : RT_ERR_DEVICE;
        const auto t1 = std::chrono::steady_clock::now();
        rt_stats st;
        std::memset(&st, 0, sizeof(st));
        if (rc == RT_OK) rc = rt_multi_stats(m, &st);
        std::vector<uint8_t> img(size_t(width) * height * 4);
        if (rc == RT_OK && storeRenderResult)
            rc = hipMemcpy(img.data(), dout, img.size(), hipMemcpyDeviceToHost) == hipSuccess ? RT_OK : RT_ERR_DEVICE;
        (void)hipFree(dacc);
        (void)hipFree(dout);
        if (rc != RT_OK) return report("render");
        const double sec = std::chrono::duration<double>(t1 - t0).count();
        std::printf("duration_per_frame: %.3f ms (%u GPU, %s stream, %llu samples, %.1f Msamples/s incl. first-launch setup)\n",
                    sec * 1e3, m->n, opt.rng_mode == RT_RNG_SAMPLE_HASH ? "hash" : "reference",
                    (unsigned long long)st.samples, double(st.samples) / sec / 1e6);
        std::printf("setup: devices + streams%s %.1f ms, scene build + upload %.1f ms\n",
                    m->n > 1 ? " + RCCL communicator" : "", create_ms, scene_ms);
        if (storeRenderResult && rt_store_ppm("render.ppm", img.data(), width, height)) report("store");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ray_trace: %s\n", e.what());
    }
}

}  // extern "C"
