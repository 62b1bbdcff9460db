// rt_main.cpp — command-line front end, the counterpart of the reference's src/main.cpp:10-64
// (target RayTracingGPUVulkan, CMakeLists.txt:47-51). Same flags and defaults, same call into the
// library's ray_trace(); unknown flags are reported and ignored as in the reference (:48-50),
// but a flag missing its value is an error here (the reference reads past argv, :33-46).
//
//   --help  --store  --samples <spp>  --width <w>  --height <h>  --gpus <n>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/rt_mi355x.h"

static bool parse_u32(const char* s, uint32_t& out) {
    const char* end = s + std::strlen(s);
    auto r = std::from_chars(s, end, out);
    return r.ec == std::errc() && r.ptr == end;
}

int main(int argc, const char** argv) {
    uint32_t samples = 10, width = 1920, height = 1080, gpu_count = 1;
    bool store = false;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--help") {
            std::puts("--help                            # Show this help information");
            std::puts("--store                           # Store rendered image to render.ppm");
            std::puts("--samples <count>                 # Samples per pixel of the frame");
            std::puts("--width <width>                   # Image width");
            std::puts("--height <height>                 # Image height");
            std::puts("--gpus <count>                    # Max used GPUs count");
            return 0;
        } else if (a == "--store") {
            store = true;
        } else if (a == "--samples" || a == "--width" || a == "--height" || a == "--gpus") {
            uint32_t v = 0;
            if (i + 1 >= argc || !parse_u32(argv[i + 1], v)) {
                std::fprintf(stderr, "%s needs an unsigned integer value\n", a.c_str());
                return 2;
            }
            ++i;
            if (a == "--samples") samples = v;
            else if (a == "--width") width = v;
            else if (a == "--height") height = v;
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
    ray_trace(samples, store, width, height, gpu_count);
    return 0;
}
