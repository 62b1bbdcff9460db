// rt_host.h — error plumbing and device selection shared by the host runtime files
// (rt_api.cpp, rt_multi.cpp). Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/rt_mi355x.h"

namespace rt {

// A host-built scene (tree, grid, records; rt_api.cpp), built once and uploadable to any context:
// rt_multi_set_scene builds it for the first device and uploads the same package to the others.
struct HostPackage;
struct HostPackageDeleter { void operator()(HostPackage* p) const; };
using HostPackagePtr = std::unique_ptr<HostPackage, HostPackageDeleter>;

// rt_set_scene in two halves, so that rt_multi_set_scene issues every device's build before it
// waits for any: begin builds a host scene (or takes *shared) and uploads it, or starts a device
// build on the context's build stream; end waits for the device build's summary and builds its
// grid. Every begin that succeeds must be followed by end on the same context.
int set_scene_begin(rt_context* ctx, const Sphere* spheres, uint32_t count, void* stream, HostPackagePtr* shared);
int set_scene_end(rt_context* ctx);

// Trace launches recorded on ctx so far, and the trace-kernel duration of launch `index` (0 = the
// context's first; only the last 64 are kept), waiting for that launch's end event only.
uint64_t launch_count(const rt_context* ctx);
int launch_ms_at(rt_context* ctx, uint64_t index, float* ms);
// Per band row of launch `index` (one of the last 4), its share of the launch's work as the
// tile-cost record estimates it (rt_launch_row_weights); waits for that launch's copy only.
// Launches keep the record copies only once asked for (keep_row_weights, or the first call).
int launch_row_weights(rt_context* ctx, uint64_t index, std::vector<double>& w);
void keep_row_weights(rt_context* ctx);

// Message of the calling thread's last failure (rt_last_error()).
extern thread_local std::string g_last_error;
int fail(int code, const std::string& msg);
int current_device_count(int* n);

// RAII device selection: restores the caller's current device.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace rt

#define RT_HIP(call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::rt::fail(e_ == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_DEVICE, \
                              std::string(#call) + ": " + hipGetErrorString(e_));          \
    } while (0)
