// rt_multi.cpp — one process driving N GPUs: the multi-device frame over RCCL (rt_multi_*),
// the host-buffer frame rt_render(), and the reference's entry point ray_trace().
//
// The reference creates one Vulkan device per GPU (src/ray_trace.cpp:42-105), gives each a
// contiguous row band (:74-93) and moves rows between GPUs from their measured frame times
// (src/workload_tuner.hpp:38-104, hooked at src/ray_trace.cpp:750-775), tearing down and
// rebuilding every Vulkan object on each move (:774, :778-916); it never moves pixels between
// GPUs (each device presents its own window). Here the image starts as row-exact interleaved
// 8-row strips (rt_plan.h strip_parts: every device within one row of H / N), each device renders
// its rows through a rows map (global pixel seeds, so the image does not depend on the partition),
// one RCCL group moves every other device's float4 accumulator rows to device 0 over xGMI
// (ncclSend / ncclRecv; device 0's own rows are not sent), one kernel per source puts them in
// place (rt_scatter_rows) and device 0 tonemaps the whole accumulator to rgba8 once
// (rt_resolve_rgba8: the rgba8 bytes are a function of the float sum, shader.rgen:65-66, so they
// need not travel). A single device holding every row renders straight into the caller's buffers.
// SURVEY.md §8(e).
//
// Balancing: every frame reads each device's trace-kernel time of the frame
// two before it (its end event has long passed: no host wait on queued work), rescales per-row
// cost estimates to those times and moves band-end rows from the slowest device to the fastest
// (rt_plan.h rebalance). A move rewrites rows maps only: the contexts, scenes, buffers (grown when
// needed) and each band's LPT tile costs stay (rows leave and join at a band's end, so its other
// tiles keep their index).
//
// A frame is a FramePlan (rt_plan.h): the partition and the ordered steps rt_multi_render executes.
// The plan is host-only data, so the CPU tests check it for every device count and height without
// a GPU (rt_debug_multi_plan*, tests/test_multi_plan.py). rt_debug_multi_create_logical runs the
// same executor over N logical devices on GPU 0, with each send / receive pair a device copy
// ordered by the same group boundaries, so the one-GPU pool executes every step of the N > 1 plan.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
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
#include "rt_plan.h"

using rt::DeviceGuard;
using rt::fail;
using namespace rt::plan;

#define RT_NCCL(call)                                                                       \
    do {                                                                                    \
        ncclResult_t r_ = (call);                                                           \
        if (r_ != ncclSuccess)                                                              \
            return fail(RT_ERR_DEVICE, std::string(#call) + ": " + ncclGetErrorString(r_));  \
    } while (0)

namespace {

// One part of a multi-device frame on its device (its own context), with its buffers.
struct Launch {
    uint32_t dev = 0;                    // logical device
    std::vector<uint32_t> rows;          // global rows, band order
    bool whole = false;
    rt_context* ctx = nullptr;           // on dev
    uint32_t cap = 0;                    // rows the buffers below hold
    uint32_t* rows_dev = nullptr;        // rows on dev (the kernel's map)
    uint32_t* rows_root = nullptr;       // rows on device 0 (the row loads / stores)
    float* acc = nullptr;                // band on dev: rows x W float4 (not for a whole part)
    uint8_t* out = nullptr;              // band on dev: rows x W rgba8 (the kernel's store; not sent)
    float* stage_acc = nullptr;          // dev != 0: the band's copy on device 0
};

constexpr uint32_t kMaxLag = 8;   // strip frames the balancer keeps (its largest lag)

// A rendered strip frame, for the balancer: its partition and each part's launch index on its
// context (UINT64_MAX: the part rendered nothing).
struct FrameRecord {
    Parts parts;
    std::vector<uint64_t> launch;
};

}  // namespace

struct rt_multi {
    uint32_t n = 0;
    std::vector<int> phys;               // HIP device of each logical device
    bool logical = false;                // N logical devices on GPU 0 (tests on a one-GPU box)
    bool self_rccl = false;              // logical: the transfers through a one-rank communicator
                                         // (ncclSend / ncclRecv to itself on stream[0]); else copies
    std::vector<hipStream_t> stream;     // one per logical device
    std::vector<ncclComm_t> comm;        // one per device, rank = device index
    hipEvent_t ev_in = nullptr, ev_out = nullptr;   // device 0: caller stream <-> stream[0]
    std::vector<hipEvent_t> xev;         // logical transport: two per transfer of a group
    std::vector<Sphere> spheres;         // the scene, for contexts created later
    bool scene_set = false;
    // cached partition (geometry + kind): strips of W x H, or explicit bands
    uint32_t W = 0, H = 0;
    std::string key;
    std::vector<Launch> launches;        // one per plan part, same index
    FramePlan plan[2];                   // steps without / with accumulation
    struct Balancer {
        bool enabled = true;
        double tolerance = 0.001;        // re-deal when the slowest device is above (1 + tol) x mean
        double blend = 0.5;              // weight of a new measurement in the per-row estimates
        uint32_t lag = 2;                // frames between a measured frame and the frame it re-deals
        std::vector<double> cost;        // per global row, ms
        std::deque<FrameRecord> history; // strip frames rendered since the partition was set up
        std::vector<float> injected;     // rt_debug_multi_feedback: times of the current partition
        uint64_t frames = 0, rebalances = 0, moved = 0;
        double predicted = 1.0;          // predicted max / mean after the last re-deal
    } bal;
};

namespace {

int phys_of(const rt_multi* m, uint32_t dev) { return m->phys[dev]; }

void free_buffers(rt_multi* m, Launch& l) {
    {
        DeviceGuard g(phys_of(m, l.dev));
        (void)hipDeviceSynchronize();
        if (l.rows_dev) (void)hipFree(l.rows_dev);
        if (l.acc) (void)hipFree(l.acc);
        if (l.out) (void)hipFree(l.out);
    }
    DeviceGuard g0(phys_of(m, 0));
    (void)hipDeviceSynchronize();
    if (l.rows_root) (void)hipFree(l.rows_root);
    if (l.stage_acc) (void)hipFree(l.stage_acc);
    l.rows_dev = l.rows_root = nullptr;
    l.acc = l.stage_acc = nullptr;
    l.out = nullptr;
    l.cap = 0;
}

void free_launches(rt_multi* m) {
    for (Launch& l : m->launches) {
        free_buffers(m, l);
        DeviceGuard g(phys_of(m, l.dev));
        rt_context_destroy(l.ctx);
    }
    m->launches.clear();
    m->plan[0] = m->plan[1] = FramePlan{};
    m->key.clear();
    m->bal.history.clear();
    m->bal.cost.clear();
    m->bal.injected.clear();
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

// The part's buffers for its rows (grown, never shrunk; a move of a few rows reuses them), and its
// rows maps on its device and on device 0. Callers have drained the streams that read them.
int fit_buffers(rt_multi* m, Launch& l) {
    const uint32_t nr = uint32_t(l.rows.size()), W = m->W;
    if (!nr || l.whole) return RT_OK;
    if (l.cap < nr) {
        free_buffers(m, l);
        // room for the rows a balancer moves in (a few percent of a band) without reallocating
        const uint32_t cap = std::min<uint32_t>(m->H, nr + std::max<uint32_t>(kStrip, nr / 16));
        const size_t texels = size_t(cap) * W;
        {
            DeviceGuard g(phys_of(m, l.dev));
            RT_HIP(hipMalloc(&l.rows_dev, size_t(cap) * 4));
            RT_HIP(hipMalloc(&l.acc, texels * 16));
            RT_HIP(hipMalloc(&l.out, texels * 4));
        }
        DeviceGuard g0(phys_of(m, 0));
        RT_HIP(hipMalloc(&l.rows_root, size_t(cap) * 4));
        if (l.dev != 0) RT_HIP(hipMalloc(&l.stage_acc, texels * 16));
        l.cap = cap;
    }
    {
        DeviceGuard g(phys_of(m, l.dev));
        RT_HIP(hipMemcpy(l.rows_dev, l.rows.data(), size_t(nr) * 4, hipMemcpyHostToDevice));
    }
    DeviceGuard g0(phys_of(m, 0));
    RT_HIP(hipMemcpy(l.rows_root, l.rows.data(), size_t(nr) * 4, hipMemcpyHostToDevice));
    return RT_OK;
}

// (Re)builds the launches for `key` from the partition: one per part (device + global rows), its
// context and buffers, and the frame's plans with and without accumulation. Same key and size:
// nothing to do.
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
        if (int rc = rt_context_create(phys_of(m, l.dev), &l.ctx)) return rc;
        if (m->launches.size() > 1) rt::keep_row_weights(l.ctx);   // the balancer reads them
        if (int rc = fit_buffers(m, l)) return rc;
    }
    m->key = key;
    return m->scene_set ? set_scene_all(m) : RT_OK;
}

// A new partition of the same parts (devices unchanged): rows maps and plans only. Waits for every
// device's queued work first (the maps are read by queued launches); a re-deal happens a few times
// while a run's balance settles, not per frame.
int repartition(rt_multi* m, const Parts& parts) {
    for (uint32_t d = 0; d < m->n; d++) {
        DeviceGuard g(phys_of(m, d));
        RT_HIP(hipStreamSynchronize(m->stream[d]));
    }
    Parts copy = parts, copy2 = parts;
    m->plan[0] = make_plan(m->W, m->H, std::move(copy), false);
    m->plan[1] = make_plan(m->W, m->H, std::move(copy2), true);
    for (size_t i = 0; i < m->launches.size(); i++) {
        Launch& l = m->launches[i];
        l.rows = m->plan[0].parts[i].rows;
        l.whole = m->plan[0].parts[i].whole;
        if (int rc = fit_buffers(m, l)) return rc;
    }
    return RT_OK;
}

Parts current_parts(const rt_multi* m) {
    Parts p;
    for (const Launch& l : m->launches) p.emplace_back(l.dev, l.rows);
    return p;
}

// The balancer step before a strip frame: feedback from the frame `lag` frames back (or injected
// times of the current partition), then a re-deal of the current partition.
int balance_step(rt_multi* m) {
    auto& b = m->bal;
    if (!b.enabled || m->n < 2 || m->launches.size() < 2) return RT_OK;
    if (b.cost.size() != m->H) b.cost.assign(m->H, 0.0);
    std::vector<float> ms;
    Parts measured;
    std::vector<std::vector<double>> weights;
    if (!b.injected.empty()) {
        measured = current_parts(m);
        ms = b.injected;
        ms.resize(measured.size(), 0.0f);
        b.injected.clear();
    } else {
        if (b.history.size() < std::max<uint32_t>(1, b.lag)) return RT_OK;
        const FrameRecord& r = b.history[b.history.size() - std::max<uint32_t>(1, b.lag)];
        measured = r.parts;
        ms.assign(measured.size(), 0.0f);
        weights.resize(measured.size());
        for (size_t i = 0; i < measured.size(); i++) {
            if (r.launch[i] == UINT64_MAX) continue;
            if (rt::launch_ms_at(m->launches[i].ctx, r.launch[i], &ms[i]) != RT_OK) {
                rt::g_last_error.clear();   // a reading lost is no frame error: keep the partition
                return RT_OK;
            }
            // the launch's per-row work from its tile costs (none kept, e.g. brute force: the
            // device time alone rescales the rows' estimates)
            const std::string keep = rt::g_last_error;
            if (rt::launch_row_weights(m->launches[i].ctx, r.launch[i], weights[i]) != RT_OK) weights[i].clear();
            rt::g_last_error = keep;
        }
    }
    update_costs(measured, ms.data(), b.cost, weights.empty() ? nullptr : &weights, b.blend);
    Parts next = current_parts(m);
    std::vector<double> loads;
    const uint32_t moved = rebalance(next, b.cost, b.tolerance, &loads);
    if (!moved) return RT_OK;
    b.rebalances++;
    b.moved += moved;
    b.predicted = imbalance(next, b.cost);
    return repartition(m, next);
}

// A send / receive pair of the logical transport (one GPU): a device copy on the receiver's stream
// after the sender's earlier work, and the sender's later work after the copy.
int logical_transfers(rt_multi* m, const std::vector<PlanStep>& group) {
    size_t ev = 0;
    for (const PlanStep& r : group) {
        if (r.op != OP_RECV) continue;
        const PlanStep* s = nullptr;
        for (const PlanStep& c : group)
            if (c.op == OP_SEND && c.dev == r.peer && c.peer == r.dev && c.part == r.part) s = &c;
        if (!s || s->count != r.count) return fail(RT_ERR_INVALID_ARGUMENT, "unpaired receive in the plan");
        Launch& l = m->launches[r.part];
        const float* src = s->dev == 0 ? l.stage_acc : l.acc;
        float* dst = r.dev == 0 ? l.stage_acc : l.acc;
        while (m->xev.size() < ev + 2) {
            hipEvent_t e = nullptr;
            DeviceGuard g(phys_of(m, 0));
            RT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            m->xev.push_back(e);
        }
        DeviceGuard g(phys_of(m, r.dev));
        RT_HIP(hipEventRecord(m->xev[ev], m->stream[s->dev]));
        RT_HIP(hipStreamWaitEvent(m->stream[r.dev], m->xev[ev], 0));
        RT_HIP(hipMemcpyAsync(dst, src, r.count * 4, hipMemcpyDeviceToDevice, m->stream[r.dev]));
        RT_HIP(hipEventRecord(m->xev[ev + 1], m->stream[r.dev]));
        RT_HIP(hipStreamWaitEvent(m->stream[s->dev], m->xev[ev + 1], 0));
        ev += 2;
    }
    return RT_OK;
}

// The rgba8 resolve of the whole accumulator: one launch when every part shares one spp, else each
// part's contiguous row runs with its own RenderCallInfo's spp (rt_render's bands).
int resolve_all(rt_multi* m, rt_context* c0, const RenderCallInfo* rcis, size_t n_rci, float* acc, uint8_t* out) {
    const uint32_t W = m->W;
    bool same = true;
    for (size_t i = 1; i < n_rci; i++) same &= rcis[i].samplesPerRenderCall == rcis[0].samplesPerRenderCall;
    if (same) return rt_resolve_rgba8(c0, acc, uint64_t(W) * m->H, rcis[0].samplesPerRenderCall, out, m->stream[0]);
    for (size_t p = 0; p < m->launches.size(); p++) {
        const std::vector<uint32_t>& rows = m->launches[p].rows;
        const uint32_t spp = rcis[n_rci == 1 ? 0 : p].samplesPerRenderCall;
        for (size_t k = 0; k < rows.size();) {
            size_t e = k + 1;
            while (e < rows.size() && rows[e] == rows[e - 1] + 1) e++;
            const size_t off = size_t(rows[k]) * W;
            if (int rc = rt_resolve_rgba8(c0, acc + off * 4, uint64_t(e - k) * W, spp, out + off * 4, m->stream[0]))
                return rc;
            k = e;
        }
    }
    return RT_OK;
}

// self_rccl groups run on stream[0]: before a group it waits for every logical device's stream,
// after it every stream waits for it (what the per-device streams of real ranks get from RCCL).
int self_group_fence(rt_multi* m, bool before) {
    while (m->xev.size() < m->n) {
        hipEvent_t e = nullptr;
        DeviceGuard g(phys_of(m, 0));
        RT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        m->xev.push_back(e);
    }
    DeviceGuard g(phys_of(m, 0));
    if (before) {
        for (uint32_t d = 1; d < m->n; d++) {
            RT_HIP(hipEventRecord(m->xev[d], m->stream[d]));
            RT_HIP(hipStreamWaitEvent(m->stream[0], m->xev[d], 0));
        }
    } else {
        RT_HIP(hipEventRecord(m->xev[0], m->stream[0]));
        for (uint32_t d = 1; d < m->n; d++) RT_HIP(hipStreamWaitEvent(m->stream[d], m->xev[0], 0));
    }
    return RT_OK;
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
    std::vector<PlanStep> group;   // logical transport: the group's sends / receives
    auto body = [&]() -> int {
        for (const PlanStep& s : p.steps) {
            Launch& l = m->launches[s.part];
            float* dev_buf = s.dev == 0 ? l.stage_acc : l.acc;   // a SEND / RECV's buffer on s.dev
            float* root_buf = l.dev == 0 ? l.acc : l.stage_acc;  // the part's accumulator on device 0
            const uint32_t nr = uint32_t(l.rows.size());
            switch (s.op) {
                case OP_GROUP_START:
                    if (m->self_rccl) {   // stream[0] carries the group: after every device's work so far
                        if (int rc = self_group_fence(m, true)) return rc;
                    }
                    if (!m->logical || m->self_rccl) RT_NCCL(ncclGroupStart());
                    group.clear();
                    in_group = true;
                    break;
                case OP_GROUP_END:
                    in_group = false;
                    if (m->logical && !m->self_rccl) {
                        if (int rc = logical_transfers(m, group)) return rc;
                    } else {
                        RT_NCCL(ncclGroupEnd());
                        if (m->self_rccl) {   // every device's later work after the group
                            if (int rc = self_group_fence(m, false)) return rc;
                        }
                    }
                    break;
                case OP_SEND:
                case OP_RECV: {
                    if (m->logical && !m->self_rccl) {
                        group.push_back(s);
                        break;
                    }
                    // a one-rank communicator (self_rccl): every transfer is rank 0 to itself on
                    // stream[0]; the k-th send and the k-th receive of a group pair up, as the plan
                    // orders them (each send beside its receive)
                    const uint32_t rank_dev = m->self_rccl ? 0u : s.dev;
                    const int peer = m->self_rccl ? 0 : int(s.peer);
                    DeviceGuard g(phys_of(m, rank_dev));
                    const ncclResult_t e =
                        s.op == OP_SEND
                            ? ncclSend(dev_buf, s.count, ncclFloat32, peer, m->comm[rank_dev], m->stream[rank_dev])
                            : ncclRecv(dev_buf, s.count, ncclFloat32, peer, m->comm[rank_dev], m->stream[rank_dev]);
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
                    if (int rc = resolve_all(m, c0, rcis, n_rci, acc, out)) return rc;
                    break;
                default:
                    return fail(RT_ERR_INVALID_ARGUMENT, "bad plan step");
            }
        }
        return RT_OK;
    };
    const int rc = body();
    if (in_group && (!m->logical || m->self_rccl)) (void)ncclGroupEnd();   // a failure inside a group still closes it
    return rc;
}

int copy_plan(std::vector<uint32_t>&& v, uint32_t* out, uint64_t capacity, uint64_t* count) {
    *count = v.size();
    if (!out) return RT_OK;   // size query
    if (capacity < v.size()) return fail(RT_ERR_INVALID_ARGUMENT, "capacity");
    std::memcpy(out, v.data(), v.size() * 4);
    return RT_OK;
}

int create(uint32_t gpu_count, bool logical, bool self_rccl, rt_multi** out) {
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
        m->logical = logical;
        m->self_rccl = logical && self_rccl;
        m->n = logical ? std::max(1u, gpu_count) : std::max(1u, std::min(gpu_count, uint32_t(nd)));
        m->phys.assign(m->n, 0);
        for (uint32_t d = 0; d < m->n; d++) m->phys[d] = logical ? 0 : int(d);
        m->stream.assign(m->n, nullptr);
        m->comm.assign(m->n, nullptr);
        for (uint32_t d = 0; d < m->n; d++) {
            DeviceGuard g(phys_of(m, d));
            RT_HIP(hipStreamCreateWithFlags(&m->stream[d], hipStreamNonBlocking));
        }
        {
            DeviceGuard g(phys_of(m, 0));
            RT_HIP(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
            RT_HIP(hipEventCreateWithFlags(&m->ev_out, hipEventDisableTiming));
        }
        // A single device's frame plan holds no send or receive (tests/test_multi_plan.py), so
        // one device needs no communicator: the drop-in ray_trace(..., 1) does not pay RCCL's
        // initialisation on its cold call. Logical devices share GPU 0 and copy instead.
        if (m->n > 1 && !logical) {
            std::vector<int> devs(m->n);
            for (uint32_t d = 0; d < m->n; d++) devs[d] = int(d);
            RT_NCCL(ncclCommInitAll(m->comm.data(), int(m->n), devs.data()));
        } else if (m->self_rccl) {   // one rank on GPU 0 (rank 0 = logical device 0)
            int dev0 = 0;
            RT_NCCL(ncclCommInitAll(m->comm.data(), 1, &dev0));
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

}  // namespace

extern "C" {

int rt_multi_create(uint32_t gpu_count, rt_multi** out) { return create(gpu_count, false, false, out); }

int rt_debug_multi_create_logical(uint32_t n_devices, rt_multi** out) {
    if (n_devices == 0 || n_devices > 64) return fail(RT_ERR_INVALID_ARGUMENT, "n_devices must be 1..64");
    return create(n_devices, true, false, out);
}

int rt_debug_multi_create_logical_rccl(uint32_t n_devices, rt_multi** out) {
    if (n_devices == 0 || n_devices > 64) return fail(RT_ERR_INVALID_ARGUMENT, "n_devices must be 1..64");
    return create(n_devices, true, true, out);
}

int rt_multi_destroy(rt_multi* m) {
    if (!m) return RT_OK;
    if (!m->phys.empty()) free_launches(m);
    for (uint32_t d = 0; d < m->n && d < m->phys.size(); d++) {
        DeviceGuard g(phys_of(m, d));
        (void)hipDeviceSynchronize();
        if (d < m->comm.size() && m->comm[d]) (void)ncclCommDestroy(m->comm[d]);
        if (d < m->stream.size() && m->stream[d]) (void)hipStreamDestroy(m->stream[d]);
    }
    if (!m->phys.empty()) {
        DeviceGuard g(phys_of(m, 0));
        if (m->ev_in) (void)hipEventDestroy(m->ev_in);
        if (m->ev_out) (void)hipEventDestroy(m->ev_out);
        for (hipEvent_t e : m->xev) (void)hipEventDestroy(e);
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
        if (int rc = balance_step(m)) return rc;
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    {   // the frame starts after the caller's earlier work on `stream` (device 0)
        DeviceGuard g0(phys_of(m, 0));
        RT_HIP(hipEventRecord(m->ev_in, st));
        for (uint32_t d = 0; d < m->n; d++) RT_HIP(hipStreamWaitEvent(m->stream[d], m->ev_in, 0));
    }
    const bool acc_mode = opt && opt->accumulate;
    if (int rc = run_plan(m, m->plan[acc_mode ? 1 : 0], rci, 1, opt, accum, out)) return rc;
    try {   // the balancer's record of this frame
        FrameRecord r;
        r.parts = current_parts(m);
        for (const Launch& l : m->launches)
            r.launch.push_back(l.rows.empty() ? UINT64_MAX : rt::launch_count(l.ctx) - 1);
        m->bal.history.push_back(std::move(r));
        while (m->bal.history.size() > kMaxLag) m->bal.history.pop_front();
        m->bal.frames++;
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    DeviceGuard g0(phys_of(m, 0));
    RT_HIP(hipEventRecord(m->ev_out, m->stream[0]));   // the caller's later work waits for it
    RT_HIP(hipStreamWaitEvent(st, m->ev_out, 0));
    return RT_OK;
}

int rt_multi_partition(const rt_multi* m, uint32_t* rows, uint32_t* counts, uint32_t capacity) {
    if (!m || !counts) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    uint64_t total = 0;
    for (uint32_t d = 0; d < m->n; d++) counts[d] = 0;
    for (const Launch& l : m->launches) total += l.rows.size();
    if (rows && capacity < total) return fail(RT_ERR_INVALID_ARGUMENT, "capacity below the image height");
    uint64_t at = 0;
    for (const Launch& l : m->launches) {
        if (l.dev < m->n) counts[l.dev] += uint32_t(l.rows.size());
        if (rows) std::memcpy(rows + at, l.rows.data(), l.rows.size() * 4);
        at += l.rows.size();
    }
    return RT_OK;
}

int rt_debug_multi_tune(rt_multi* m, const char* key, double value) {
    if (!m || !key) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    const std::string k = key;
    if (k == "balance") m->bal.enabled = value < 0 ? true : value != 0.0;
    else if (k == "tolerance") m->bal.tolerance = value < 0 ? 0.001 : value;
    else if (k == "blend") {
        if (value == 0.0 || !(value == value)) return fail(RT_ERR_INVALID_ARGUMENT, "blend must be in (0, 1]");
        m->bal.blend = value < 0 ? 0.5 : std::min(1.0, value);
    } else if (k == "lag") {
        if (value >= 0 && value > double(kMaxLag)) return fail(RT_ERR_INVALID_ARGUMENT, "lag above the kept frames");
        m->bal.lag = value < 0 ? 2u : std::max<uint32_t>(1, uint32_t(value));
    }
    else return fail(RT_ERR_INVALID_ARGUMENT, "unknown key " + k);
    return RT_OK;
}

int rt_debug_multi_feedback(rt_multi* m, const float* device_ms, uint32_t n) {
    if (!m || (!device_ms && n)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    m->bal.injected.assign(device_ms, device_ms + n);
    return RT_OK;
}

int rt_debug_multi_balance_info(const rt_multi* m, double* out4) {
    if (!m || !out4) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    out4[0] = double(m->bal.frames);
    out4[1] = double(m->bal.rebalances);
    out4[2] = double(m->bal.moved);
    out4[3] = m->bal.predicted;
    return RT_OK;
}

int rt_debug_multi_plan(uint32_t n_devices, uint32_t width, uint32_t height, const uint32_t* band_starts,
                        uint32_t n_bands, uint32_t accumulate, uint32_t* out, uint64_t capacity, uint64_t* count) {
    if (!count) return fail(RT_ERR_INVALID_ARGUMENT, "count is NULL");
    *count = 0;
    if (n_devices == 0 || width == 0 || height == 0) return fail(RT_ERR_INVALID_ARGUMENT, "zero size");
    if (band_starts && n_bands == 0) return fail(RT_ERR_INVALID_ARGUMENT, "no bands");
    try {
        Parts parts = band_starts ? band_parts(n_devices, height, band_starts, n_bands) : strip_parts(n_devices, height);
        if (parts.empty()) return fail(RT_ERR_INVALID_ARGUMENT, "bands must tile the image top to bottom");
        return copy_plan(serialize(make_plan(width, height, std::move(parts), accumulate != 0)), out, capacity, count);
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
}

int rt_debug_multi_plan_rows(uint32_t n_devices, uint32_t width, uint32_t height, const uint32_t* rows,
                             const uint32_t* counts, uint32_t accumulate, uint32_t* out, uint64_t capacity,
                             uint64_t* count) {
    if (!count) return fail(RT_ERR_INVALID_ARGUMENT, "count is NULL");
    *count = 0;
    if (n_devices == 0 || width == 0 || height == 0 || !rows || !counts)
        return fail(RT_ERR_INVALID_ARGUMENT, "zero size or NULL partition");
    try {
        Parts parts = row_parts(n_devices, height, rows, counts);
        if (parts.empty()) return fail(RT_ERR_INVALID_ARGUMENT, "the partition must hold every row exactly once");
        return copy_plan(serialize(make_plan(width, height, std::move(parts), accumulate != 0)), out, capacity, count);
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
}

int rt_partition_strips(uint32_t n_devices, uint32_t height, uint32_t* rows, uint32_t* counts) {
    if (n_devices == 0 || !rows || !counts) return fail(RT_ERR_INVALID_ARGUMENT, "zero devices or NULL output");
    try {
        const Parts parts = strip_parts(n_devices, height);
        uint64_t at = 0;
        for (uint32_t d = 0; d < n_devices; d++) {
            counts[d] = uint32_t(parts[d].second.size());
            std::memcpy(rows + at, parts[d].second.data(), parts[d].second.size() * 4);
            at += parts[d].second.size();
        }
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    return RT_OK;
}

int rt_partition_rebalance(uint32_t n_devices, uint32_t height, uint32_t* rows, uint32_t* counts, double* row_cost,
                           const uint32_t* meas_rows, const uint32_t* meas_counts, const float* meas_ms,
                           double tolerance, uint32_t* moved, double* predicted_imbalance) {
    if (n_devices == 0 || !rows || !counts || !row_cost) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if ((meas_rows || meas_counts || meas_ms) && !(meas_rows && meas_counts && meas_ms))
        return fail(RT_ERR_INVALID_ARGUMENT, "a measurement needs its rows, counts and times");
    try {
        Parts cur = row_parts(n_devices, height, rows, counts);
        if (cur.empty() && height) return fail(RT_ERR_INVALID_ARGUMENT, "the partition must hold every row exactly once");
        std::vector<double> cost(row_cost, row_cost + height);
        if (meas_rows) {
            Parts meas = row_parts(n_devices, height, meas_rows, meas_counts);
            if (meas.empty() && height)
                return fail(RT_ERR_INVALID_ARGUMENT, "the measured partition must hold every row exactly once");
            update_costs(meas, meas_ms, cost);
        }
        const uint32_t k = rebalance(cur, cost, tolerance, nullptr);
        if (moved) *moved = k;
        if (predicted_imbalance) *predicted_imbalance = imbalance(cur, cost);
        std::memcpy(row_cost, cost.data(), size_t(height) * sizeof(double));
        uint64_t at = 0;
        for (uint32_t d = 0; d < n_devices; d++) {
            counts[d] = uint32_t(cur[d].second.size());
            std::memcpy(rows + at, cur[d].second.data(), cur[d].second.size() * 4);
            at += cur[d].second.size();
        }
    } catch (const std::exception& e) {
        return fail(RT_ERR_OUT_OF_MEMORY, e.what());
    }
    return RT_OK;
}

int rt_multi_info(const rt_multi* m, uint32_t* out4) {
    if (!m || !out4) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    int ranks = 0;   // 0: one device or logical devices with copies, no communicator
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
// i % n), gathered to device 0 by the same RCCL path, then copied to the host. Each band is
// tonemapped with its own samplesPerRenderCall (the reference's per-band RenderCallInfo).
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
        DeviceGuard g0(phys_of(m, 0));
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
    DeviceGuard g0(phys_of(m, 0));
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
