// rt_host.h — error plumbing and device selection shared by the host runtime files
// (rt_api.cpp, rt_multi.cpp). Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace rt {

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
