// Exhaustive check of the cheap correctly rounded helpers of rt_device_math.h against hipcc's own
// correctly rounded operations, over all 2^32 binary32 inputs, on the GPU:
//   rcp_cr(x)  vs 1.0f / x
//   sqrt_cr(x) vs __builtin_sqrtf(x)
// Bits are compared, except that any NaN equals any NaN. Build + run (GPU box):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I ray-tracing-gpu-vulkan_amd/csrc \
//       scripts/exact_math_exhaustive.hip -o /tmp/exact_math && /tmp/exact_math
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "rt_device_math.h"

using namespace rtd;

__device__ __forceinline__ bool same(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__global__ void check(uint64_t base, unsigned long long* bad, uint32_t* first) {
    const uint64_t i = base + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(uint32_t(i));
    if (!same(rcp_cr(x), 1.0f / x)) {
        if (atomicAdd(&bad[0], 1ull) == 0) first[0] = uint32_t(i);
    }
    if (!same(sqrt_cr(x), __builtin_sqrtf(x))) {
        if (atomicAdd(&bad[1], 1ull) == 0) first[1] = uint32_t(i);
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    hipMemset(bad, 0, 16);
    hipMemset(first, 0xff, 8);
    const uint32_t block = 256, grid = 1u << 22;   // 2^30 inputs per launch
    for (uint64_t base = 0; base < (1ull << 32); base += uint64_t(block) * grid)
        hipLaunchKernelGGL(check, dim3(grid), dim3(block), 0, 0, base, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long hb[2];
    uint32_t hf[2];
    hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(hf, first, 8, hipMemcpyDeviceToHost);
    std::printf("rcp_cr  vs 1.0f/x      : %llu mismatches of 2^32 inputs (first 0x%08x)\n", hb[0], hf[0]);
    std::printf("sqrt_cr vs sqrtf(x)    : %llu mismatches of 2^32 inputs (first 0x%08x)\n", hb[1], hf[1]);
    return (hb[0] || hb[1]) ? 1 : 0;
}
