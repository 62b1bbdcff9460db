// rt_main.cpp — command-line front end, the counterpart of the reference's src/main.cpp:10-64
// (target RayTracingGPUVulkan, CMakeLists.txt:47-51). Same flags and defaults, same call into the
// library's ray_trace(); unknown flags are reported and ignored as in the reference (:48-50),
// but a flag missing its value is an error here (the reference reads past argv, :33-46).
//
//   --help  --store  --samples <spp>  --width <w>  --height <h>  --gpus <n>
//   --frames <n> [--animate]: the reference's benchmark frame loop (src/ray_trace.cpp:567-748):
//   n frames back to back, each rebuilding the scene (generateRandomScene(t), t = seconds since
//   start with --animate, else 0) and rendering the image tiled over the GPUs with an RCCL gather
//   to GPU 0 (rt_multi); prints duration_per_frame like the reference (:740-744). Frames are
//   queued asynchronously on ONE rt_multi (one communicator, its streams keep the gathers of
//   successive frames in one order on every device), so the host builds frame k+1's scene while
//   frame k renders.
//   --rng stream|hash: the reference's per-pixel LCG stream (default) or the counter-based
//   RT_RNG_SAMPLE_HASH stream, for --frames and for the single ray_trace() frame alike.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_mi355x.h"

static bool parse_u32(const char* s, uint32_t& out) {
    const char* end = s + std::strlen(s);
    auto r = std::from_chars(s, end, out);
    return r.ec == std::errc() && r.ptr == end;
}

#define CLI_HIP(x)                                                                      \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                                   \
        }                                                                               \
    } while (0)
#define CLI_RT(x)                                                                       \
    do {                                                                                \
        if ((x) != RT_OK) {                                                             \
            std::fprintf(stderr, "%s: %s\n", #x, rt_last_error());                     \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

namespace {

int run_frames(uint32_t samples, uint32_t width, uint32_t height, uint32_t gpu_count, uint32_t frames,
               bool animate, bool store, uint32_t rng_mode) {
    // One multi-device renderer: two rt_multi over the same devices would be two RCCL
    // communicators whose grouped gathers could run in different orders on different devices.
    rt_multi* m = nullptr;
    hipStream_t stream = nullptr;   // device 0
    float* accum = nullptr;
    uint8_t* rgba8 = nullptr;
    uint32_t n = 1;
    CLI_HIP(hipSetDevice(0));
    CLI_RT(rt_multi_create(gpu_count, &m));
    CLI_RT(rt_multi_device_count(m, &n));
    CLI_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    CLI_HIP(hipMalloc(&accum, size_t(width) * height * 16));
    CLI_HIP(hipMalloc(&rgba8, size_t(width) * height * 4));
    rt_options opt;
    std::memset(&opt, 0, sizeof(opt));
    opt.rng_mode = rng_mode;
    std::vector<Sphere> scene(488);
    uint32_t cnt = 0;
    const auto t_start = std::chrono::steady_clock::now();
    auto frame = [&]() -> int {
        const float t = animate ? std::chrono::duration<float>(std::chrono::steady_clock::now() - t_start).count() : 0.0f;
        CLI_RT(rt_generate_scene(t, 11, scene.data(), uint32_t(scene.size()), &cnt));   // scene.h:79
        RenderCallInfo rci;
        CLI_RT(rt_canonical_render_call_info(samples, width, height, &rci));
        CLI_RT(rt_multi_set_scene(m, scene.data(), cnt));
        CLI_RT(rt_multi_render(m, &rci, &opt, accum, rgba8, stream));
        return 0;
    };
    auto sync_all = [&]() -> int {
        for (uint32_t g = 0; g < n; g++) {
            CLI_HIP(hipSetDevice(int(g)));
            CLI_HIP(hipDeviceSynchronize());
        }
        CLI_HIP(hipSetDevice(0));
        return 0;
    };
    if (int rc = frame()) return rc;   // warm-up: every context has its LPT order
    if (int rc = sync_all()) return rc;
    // Report about once a second, like the reference's ~4 s benchmark windows (:740-748).
    uint32_t done = 0;
    while (done < frames) {
        const auto b = std::chrono::steady_clock::now();
        uint32_t k = 0;
        for (;;) {
            if (int rc = frame()) return rc;
            ++k;
            if (done + k >= frames) break;
            if (std::chrono::steady_clock::now() - b > std::chrono::milliseconds(1000)) break;
        }
        if (int rc = sync_all()) return rc;
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - b).count();
        done += k;
        std::printf("duration_per_frame: %.3f ms (%u frames, %u GPU, %.1f Msamples/s)\n", sec / k * 1e3, k, n,
                    double(width) * height * samples * k / sec / 1e6);
    }
    if (store) {   // the last frame
        std::vector<uint8_t> img(size_t(width) * height * 4);
        CLI_HIP(hipMemcpy(img.data(), rgba8, img.size(), hipMemcpyDeviceToHost));
        CLI_RT(rt_store_ppm("render.ppm", img.data(), width, height));
    }
    rt_multi_destroy(m);
    (void)hipStreamDestroy(stream);
    (void)hipFree(accum);
    (void)hipFree(rgba8);
    return 0;
}

}  // namespace

int main(int argc, const char** argv) {
    uint32_t samples = 10, width = 1920, height = 1080, gpu_count = 1, frames = 0, rng_mode = RT_RNG_PIXEL_STREAM;
    bool rng_explicit = false;
    bool store = false, animate = false;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--help") {
            std::puts("--help                            # Show this help information");
            std::puts("--store                           # Store rendered image to render.ppm");
            std::puts("--samples <count>                 # Samples per pixel of the frame");
            std::puts("--width <width>                   # Image width");
            std::puts("--height <height>                 # Image height");
            std::puts("--gpus <count>                    # Max used GPUs count");
            std::puts("--frames <count>                  # Benchmark loop: render count frames, print duration_per_frame");
            std::puts("--animate                         # With --frames: scene time t = seconds since start");
            std::puts("--rng <stream|hash>               # Reference per-pixel LCG stream (default) or counter-based stream");
            return 0;
        } else if (a == "--store") {
            store = true;
        } else if (a == "--animate") {
            animate = true;
        } else if (a == "--rng") {
            if (i + 1 >= argc || (std::strcmp(argv[i + 1], "stream") != 0 && std::strcmp(argv[i + 1], "hash") != 0)) {
                std::fprintf(stderr, "--rng needs stream or hash\n");
                return 2;
            }
            rng_mode = std::strcmp(argv[++i], "hash") == 0 ? RT_RNG_SAMPLE_HASH : RT_RNG_PIXEL_STREAM;
            rng_explicit = true;
        } else if (a == "--samples" || a == "--width" || a == "--height" || a == "--gpus" || a == "--frames") {
            uint32_t v = 0;
            if (i + 1 >= argc || !parse_u32(argv[i + 1], v)) {
                std::fprintf(stderr, "%s needs an unsigned integer value\n", a.c_str());
                return 2;
            }
            ++i;
            if (a == "--samples") samples = v;
            else if (a == "--width") width = v;
            else if (a == "--height") height = v;
            else if (a == "--frames") frames = v;
            else gpu_count = v;
        } else {
            std::fprintf(stderr, "unknown argument: %s\n", argv[i]);
        }
    }
    int n = 0;
    if (rt_device_count(&n) != RT_OK) {
        std::fprintf(stderr, "%s\n", rt_last_error());
        return 1;
    }
    if (frames > 0) return run_frames(samples, width, height, gpu_count, frames, animate, store, rng_mode);
    // ray_trace() keeps the reference's signature; its stream is selected through RT_RNG. An
    // explicit --rng wins over the caller's environment; without it RT_RNG passes through.
    if (rng_explicit) setenv("RT_RNG", rng_mode == RT_RNG_SAMPLE_HASH ? "hash" : "stream", 1);
    ray_trace(samples, store, width, height, gpu_count);
    return 0;
}
