// rt_multi.cpp — one process driving N GPUs: the multi-device frame over RCCL (rt_multi_*),
// the host-buffer frame rt_render(), and the reference's entry point ray_trace().
//
// The reference creates one Vulkan device per GPU (src/ray_trace.cpp:42-105), gives each a
// contiguous row band (:74-93, tuned by src/workload_tuner.hpp) and never moves pixels between
// GPUs (each device presents its own window). Here the image is tiled into 8-row strips dealt
// round robin over the devices (interleaving balances sky-heavy and sphere-heavy rows without a
// tuner), each device renders its strips through a rows map (global pixel seeds, so the image
// does not depend on the device count), and one RCCL group moves every device's float4 + rgba8
// strips to device 0 over xGMI (ncclSend / ncclRecv; device 0's own strips are not sent), where
// one kernel per source puts them in place (rt_scatter_rows); a single device holding every row
// renders straight into the caller's buffers. SURVEY.md §8(e).
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
#include <vector>

#include "../../include/rt_abi.h"
#include "../../include/rt_mi355x.h"
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

// One launch of a multi-device frame: a list of global rows rendered by one device (its own
// context), gathered into a staging band on device 0.
struct Launch {
    uint32_t dev = 0;
    std::vector<uint32_t> rows;          // global rows, band order
    bool whole = false;                  // device 0, every row in order (one device): may render
                                         // straight into the caller's buffers
    float* sum_at = nullptr;             // whole: the caller's accum buffer holding the running sum
                                         // (last frame rendered straight into it), else the band
    rt_context* ctx = nullptr;           // on dev
    uint32_t* rows_dev = nullptr;        // rows on dev (the kernel's map)
    uint32_t* rows_root = nullptr;       // rows on device 0 (the scatter's map)
    float* acc = nullptr;                // band on dev: rows x W float4
    uint8_t* out = nullptr;              // band on dev: rows x W rgba8
    float* stage_acc = nullptr;          // band copy on device 0
    uint8_t* stage_out = nullptr;
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
    std::vector<Launch> launches;
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
        if (l.stage_out) (void)hipFree(l.stage_out);
    }
    m->launches.clear();
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

// (Re)builds the launch list for `key` (one entry per launch: device + global rows). Buffers of
// a launch are zeroed (accumulate adds to the previous frame of the same partition).
int set_partition(rt_multi* m, const std::string& key, uint32_t W, uint32_t H,
                  std::vector<std::pair<uint32_t, std::vector<uint32_t>>>&& parts) {
    if (m->key == key && m->W == W && m->H == H) return RT_OK;
    free_launches(m);
    m->W = W;
    m->H = H;
    for (auto& p : parts) {
        Launch l;
        l.dev = p.first;
        l.rows = std::move(p.second);
        l.whole = l.dev == 0 && l.rows.size() == H;
        for (uint32_t y = 0; l.whole && y < H; y++) l.whole = l.rows[y] == y;
        m->launches.push_back(std::move(l));
    }
    for (Launch& l : m->launches) {
        const size_t nr = l.rows.size(), texels = nr * W;
        if (int rc = rt_context_create(int(l.dev), &l.ctx)) return rc;
        DeviceGuard g(static_cast<int>(l.dev));
        if (nr) {
            RT_HIP(hipMalloc(&l.rows_dev, nr * 4));
            RT_HIP(hipMemcpy(l.rows_dev, l.rows.data(), nr * 4, hipMemcpyHostToDevice));
            RT_HIP(hipMalloc(&l.acc, texels * 16));
            RT_HIP(hipMalloc(&l.out, texels * 4));
            RT_HIP(hipMemset(l.acc, 0, texels * 16));
            RT_HIP(hipMemset(l.out, 0, texels * 4));
        }
        DeviceGuard g0(0);
        if (nr) {
            RT_HIP(hipMalloc(&l.rows_root, nr * 4));
            RT_HIP(hipMemcpy(l.rows_root, l.rows.data(), nr * 4, hipMemcpyHostToDevice));
            if (l.dev != 0) {   // device 0's own bands are scattered in place (gather_to_root)
                RT_HIP(hipMalloc(&l.stage_acc, texels * 16));
                RT_HIP(hipMalloc(&l.stage_out, texels * 4));
            }
        }
    }
    m->key = key;
    return m->scene_set ? set_scene_all(m) : RT_OK;
}

// Strips k = 0, 1, ... of kStrip rows, strip k on device k % n.
std::vector<std::pair<uint32_t, std::vector<uint32_t>>> strip_parts(uint32_t n, uint32_t H) {
    std::vector<std::pair<uint32_t, std::vector<uint32_t>>> parts(n);
    for (uint32_t d = 0; d < n; d++) parts[d].first = d;
    for (uint32_t y = 0; y < H; y++) parts[(y / kStrip) % n].second.push_back(y);
    return parts;
}

// One RCCL group moves every other device's bands (float4 accumulator, then rgba8 image) to
// device 0, then one kernel per band puts its rows in place in dst (device 0 pointers, W x H);
// device 0's own bands go straight from its render buffers (no send to itself: at N = 1 the frame
// moves no byte through RCCL), and a band rendered into dst itself (`direct`) not at all.
// Everything on stream[0] after the group.
int gather_to_root(rt_multi* m, float* dst_acc, uint8_t* dst_out, bool direct) {
    const uint32_t W = m->W;
    RT_NCCL(ncclGroupStart());
    for (Launch& l : m->launches) {
        const size_t texels = l.rows.size() * size_t(W);
        if (!texels || l.dev == 0) continue;
        ncclResult_t e;
        {
            DeviceGuard g(static_cast<int>(l.dev));
            e = ncclSend(l.acc, texels * 4, ncclFloat32, 0, m->comm[l.dev], m->stream[l.dev]);
            if (e == ncclSuccess) e = ncclSend(l.out, texels * 4, ncclUint8, 0, m->comm[l.dev], m->stream[l.dev]);
        }
        if (e == ncclSuccess) {
            DeviceGuard g0(0);
            e = ncclRecv(l.stage_acc, texels * 4, ncclFloat32, int(l.dev), m->comm[0], m->stream[0]);
            if (e == ncclSuccess) e = ncclRecv(l.stage_out, texels * 4, ncclUint8, int(l.dev), m->comm[0], m->stream[0]);
        }
        if (e != ncclSuccess) {
            (void)ncclGroupEnd();
            return fail(RT_ERR_DEVICE, std::string("RCCL gather: ") + ncclGetErrorString(e));
        }
    }
    RT_NCCL(ncclGroupEnd());
    for (Launch& l : m->launches) {
        if (l.rows.empty() || (direct && l.whole)) continue;
        const bool own = l.dev == 0;   // rendered on stream[0] itself
        if (int rc = rt_scatter_rows(m->launches[0].ctx, own ? l.acc : l.stage_acc, own ? l.out : l.stage_out,
                                     l.rows_root, uint32_t(l.rows.size()), W, m->H, dst_acc, dst_out, m->stream[0]))
            return rc;
    }
    return RT_OK;
}

// Launch i renders its rows with rcis[i] (offset replaced by the rows map) on its device's stream.
// direct (dst_acc / dst_out on device 0, W x H): a `whole` launch renders into them, no map.
int render_bands(rt_multi* m, const RenderCallInfo* rcis, size_t n_rci, const rt_options* opt, bool direct,
                 float* dst_acc, uint8_t* dst_out) {
    for (size_t i = 0; i < m->launches.size(); i++) {
        Launch& l = m->launches[i];
        if (l.rows.empty()) continue;
        RenderCallInfo r = rcis[n_rci == 1 ? 0 : i];
        r.offset = rt_uvec2{0, 0};   // the rows map carries the global rows
        const bool d = direct && l.whole;
        if (int rc = rt_render_device(l.ctx, &r, d ? nullptr : l.rows_dev, m->W, uint32_t(l.rows.size()),
                                      d ? dst_acc : l.acc, d ? dst_out : l.out, opt, m->stream[l.dev]))
            return rc;
    }
    return RT_OK;
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
        std::vector<int> devs(m->n);
        for (uint32_t d = 0; d < m->n; d++) devs[d] = int(d);
        RT_NCCL(ncclCommInitAll(m->comm.data(), int(m->n), devs.data()));
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
    // One device holding every row renders straight into the caller's buffers (no band, no
    // reorder). Its running sum then lives in that accum buffer: an accumulating frame into the
    // same buffer adds to it there; into another buffer, the sum is copied into the band first.
    Launch* w = m->launches.size() == 1 && m->launches[0].whole ? &m->launches[0] : nullptr;
    const bool acc_mode = opt && opt->accumulate;
    const bool direct = w && (!acc_mode || w->sum_at == accum);
    if (w && !direct && w->sum_at) {
        DeviceGuard g0(0);
        RT_HIP(hipMemcpyAsync(w->acc, w->sum_at, w->rows.size() * size_t(W) * 16, hipMemcpyDeviceToDevice,
                              m->stream[0]));
    }
    if (int rc = render_bands(m, rci, 1, opt, direct, accum, out)) return rc;
    if (int rc = gather_to_root(m, accum, out, direct)) return rc;
    if (w) w->sum_at = direct ? accum : nullptr;
    DeviceGuard g0(0);
    RT_HIP(hipEventRecord(m->ev_out, m->stream[0]));   // the caller's later work waits for it
    RT_HIP(hipStreamWaitEvent(st, m->ev_out, 0));
    return RT_OK;
}

int rt_multi_info(const rt_multi* m, uint32_t* out4) {
    if (!m || !out4) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    int ranks = 0;
    RT_NCCL(ncclCommCount(m->comm[0], &ranks));
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
        if (rci[i].image_size.x != W || rci[i].image_size.y != H || rci[i].offset.x != 0 || y1 < y0 || y1 > H)
            return fail(RT_ERR_INVALID_ARGUMENT, "bands must tile the image top to bottom");
    }
    rt_multi* m = nullptr;
    if (int rc = rt_multi_create(rci_count, &m)) return rc;
    std::unique_ptr<rt_multi, int (*)(rt_multi*)> guard(m, rt_multi_destroy);
    float* dacc = nullptr;
    uint8_t* dout = nullptr;
    auto run = [&]() -> int {
        if (int rc = rt_multi_set_scene(m, spheres, sphere_count)) return rc;
        std::vector<std::pair<uint32_t, std::vector<uint32_t>>> parts(rci_count);
        for (uint32_t i = 0; i < rci_count; i++) {
            const uint32_t y0 = rci[i].offset.y, y1 = (i + 1 < rci_count) ? rci[i + 1].offset.y : H;
            parts[i].first = i % m->n;
            for (uint32_t y = y0; y < y1; y++) parts[i].second.push_back(y);
        }
        if (int rc = set_partition(m, "bands", W, H, std::move(parts))) return rc;
        if (opt && opt->accumulate) {   // the bands start from the host accumulator
            for (Launch& l : m->launches) {
                if (l.rows.empty()) continue;
                DeviceGuard g(static_cast<int>(l.dev));
                RT_HIP(hipMemcpy(l.acc, accum + size_t(l.rows[0]) * W * 4, l.rows.size() * size_t(W) * 16,
                                 hipMemcpyHostToDevice));
            }
        }
        DeviceGuard g0(0);
        RT_HIP(hipMalloc(&dacc, size_t(W) * H * 16));
        RT_HIP(hipMalloc(&dout, size_t(W) * H * 4));
        if (int rc = render_bands(m, rci, rci_count, opt, false, nullptr, nullptr)) return rc;   // each band its own RenderCallInfo
        if (int rc = gather_to_root(m, dacc, dout, false)) return rc;
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
    try {
        rt_multi* m = nullptr;
        if (rt_multi_create(gpu_count, &m)) return report("rt_multi_create");
        std::unique_ptr<rt_multi, int (*)(rt_multi*)> guard(m, rt_multi_destroy);
        std::vector<Sphere> scene(488);
        uint32_t cnt = 0;
        rt_generate_scene(0.0f, 11, scene.data(), uint32_t(scene.size()), &cnt);
        if (rt_multi_set_scene(m, scene.data(), cnt)) return report("rt_multi_set_scene");
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
        if (storeRenderResult && rt_store_ppm("render.ppm", img.data(), width, height)) report("store");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ray_trace: %s\n", e.what());
    }
}

}  // extern "C"
