// rt_device_math.h — device side of the arithmetic contract.
//
// Every operation here is an IEEE binary32 operation with one rounding (the library is built
// with -ffp-contract=off; fmas are written out where the contract names them), so results are
// bit-identical to the CPU oracle (oracle/rt_oracle.cpp), which implements the same contract
// independently. Correctly rounded divide and sqrt are hipcc's defaults for f32 on gfx950
// (-fhip-fp32-correctly-rounded-divide-sqrt); this file must never be built with -ffast-math.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {

struct V3 { float x, y, z; };

__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 scale(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }

// Correctly rounded 1 / x, cheaper than hipcc's general division (11 VALU with v_div_scale /
// v_div_fmas / v_div_fixup): for |x| in [2^-125, 2^125] (x and 1/x normal with room to spare) the
// hardware reciprocal (v_rcp_f32, within 1 ulp) is corrected by one Newton step whose residual
// e = 1 - x r is exact in an fma; the result is the correctly rounded quotient. Other inputs (0,
// inf, NaN, denormal and huge x) take the division. Bit-identical to 1.0f / x for all 2^32 inputs
// (scripts/exact_math_exhaustive.hip, run on the GPU; profiles/r02_exact_math_exhaustive.log).
// Both compute the fast form for every lane and redo only the out-of-range lanes in a rarely
// entered branch: one exec-mask region per call instead of an if / else pair (config 3 -2.0 %,
// config 5 -1.9 % against the if / else form).
__device__ __forceinline__ float rcp_cr(float x) {
    const uint32_t ax = __float_as_uint(x) & 0x7fffffffu;
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    float q = __builtin_fmaf(e, r, r);
    if (__builtin_expect(ax - 0x01000000u > 0x7e000000u - 0x01000000u, 0)) q = 1.0f / x;   // outside [2^-125, 2^125]
    return q;
}

// Correctly rounded sqrt(x), cheaper than hipcc's general sequence: for x in [2^-100, 2^100] the
// hardware square root (v_sqrt_f32, within 1 ulp) is corrected by the exact fma residuals of its
// two neighbours (the same correction hipcc emits, without the denormal scaling and the 0 / inf
// class fix-up, which this range never needs). Other inputs take __builtin_sqrtf. Bit-identical
// to it for all 2^32 inputs (scripts/exact_math_exhaustive.hip).
__device__ __forceinline__ float sqrt_cr(float x) {
    const uint32_t ux = __float_as_uint(x);
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float t = rm <= 0.0f ? sm : s;
    t = rp > 0.0f ? sp : t;
    if (__builtin_expect(ux - 0x0d800000u > 0x71800000u - 0x0d800000u, 0)) t = __builtin_sqrtf(x);   // outside [2^-100, 2^100]
    return t;
}

// dot(a,b) = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
__device__ __forceinline__ float dot(V3 a, V3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
// normalize(v) = v * (1 / sqrt(dot(v,v)))   (both correctly rounded)
__device__ __forceinline__ V3 normalize(V3 v) {
    float len = sqrt_cr(dot(v, v));
    float inv = rcp_cr(len);
    return v3(v.x * inv, v.y * inv, v.z * inv);
}
// GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N
__device__ __forceinline__ V3 reflect(V3 i, V3 n) {
    float k = 2.0f * dot(n, i);
    return sub(i, scale(k, n));
}
// GLSL refract(I, N, eta)
__device__ __forceinline__ V3 refract(V3 i, V3 n, float eta) {
    float d = dot(n, i);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return v3(0.0f, 0.0f, 0.0f);
    float s = eta * d + sqrt_cr(k);
    return sub(scale(eta, i), scale(s, n));
}

// random.glsl:1-13 — 16-round TEA.
__device__ __forceinline__ uint32_t tea(uint32_t v0, uint32_t v1) {
    uint32_t s0 = 0;
#pragma unroll
    for (uint32_t n = 0; n < 16; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
// random.glsl:15-22 — LCG step and 24-bit float (exact: integer * 2^-24).
__device__ __forceinline__ float rnd(uint32_t& seed) {
    seed = 1664525u * seed + 1013904223u;
    return float(seed & 0x00FFFFFFu) * (1.0f / 16777216.0f);
}
// random.glsl:24-34 with [min,max] = [-1,1]: r*2 - 1 (exact in binary32 for 24-bit r).
__device__ __forceinline__ float rnd_pm1(uint32_t& seed) {
    float r = rnd(seed);
    return r * 2.0f + -1.0f;
}
__device__ __forceinline__ V3 random_unit_vector(uint32_t& seed) {
    float x = rnd_pm1(seed);
    float y = rnd_pm1(seed);
    float z = rnd_pm1(seed);
    return normalize(v3(x, y, z));
}

// sin for the checker texture (shader.rchit:59): 3-part Cody-Waite + fdlibm float kernels.
__device__ __forceinline__ float sinf_det(float x) {
    float k = __builtin_rintf(x * 0.636619772f);
    float r = __builtin_fmaf(-k, 1.5707962513e+00f, x);
    r = __builtin_fmaf(-k, 7.5497894159e-08f, r);
    r = __builtin_fmaf(-k, 5.3903029534e-15f, r);
    int q = int(k) & 3;
    float r2 = r * r;
    float ps = __builtin_fmaf(r2, -1.9515295891e-04f, 8.3321608736e-03f);
    ps = __builtin_fmaf(r2, ps, -1.6666654611e-01f);
    float s = __builtin_fmaf(r * r2, ps, r);
    float pc = __builtin_fmaf(r2, 2.4433157118e-05f, -1.3887316255e-03f);
    pc = __builtin_fmaf(r2, pc, 4.1666645683e-02f);
    float r4 = r2 * r2;
    float c = __builtin_fmaf(r4, pc, __builtin_fmaf(-0.5f, r2, 1.0f));
    float v = (q & 1) ? c : s;
    return (q & 2) ? -v : v;
}

// Sign class of sinf_det(x): 0 when the value is +-0 (or x is NaN), else +1 / -1. Same reduction as
// sinf_det; for |r| <= pi/4 (+ rounding) the sine polynomial keeps the sign of r and is zero only
// for r = 0, and the cosine polynomial is > 0.7, so the polynomials need not be evaluated.
__device__ __forceinline__ int sin_sign(float x) {
    float k = __builtin_rintf(x * 0.636619772f);
    float r = __builtin_fmaf(-k, 1.5707962513e+00f, x);
    r = __builtin_fmaf(-k, 7.5497894159e-08f, r);
    r = __builtin_fmaf(-k, 5.3903029534e-15f, r);
    const int q = int(k) & 3;
    if (!(q & 1) && !(__builtin_fabsf(r) > 0.0f)) return 0;   // +-0 (or NaN): the product is not > 0
    const bool neg = (!(q & 1) && __builtin_signbit(r)) != bool(q & 2);
    return neg ? -1 : 1;
}

// sin_sign as two bits, without control flow: `zero` (the value is +-0 or x is NaN) and `neg`.
// Same reduction and the same cases as sin_sign, so the same decision bit for bit.
__device__ __forceinline__ uint32_t sin_class(float x) {   // bit 0: zero, bit 1: negative
    float k = __builtin_rintf(x * 0.636619772f);
    float r = __builtin_fmaf(-k, 1.5707962513e+00f, x);
    r = __builtin_fmaf(-k, 7.5497894159e-08f, r);
    r = __builtin_fmaf(-k, 5.3903029534e-15f, r);
    const uint32_t q = uint32_t(int(k));
    const uint32_t even = ~q & 1u;
    const uint32_t zero = even & (__builtin_fabsf(r) > 0.0f ? 0u : 1u);
    const uint32_t neg = (even & (__float_as_uint(r) >> 31)) ^ ((q >> 1) & 1u);
    return zero | (neg << 1);
}

// shader.rchit:58-60 checker decision, sin(6x) * sin(6y) * sin(6z) > 0, from the signs of the three
// sines: a product of three nonzero finite binary32 values of magnitude >= 1e-15 (hit points are
// fma results of O(1) operands) neither underflows nor changes sign in rounding, so
// it is > 0 exactly when no factor is zero and an even number is negative. Bit-identical decision
// to the oracle's full product (tests: every ground hit of the GPU parity suite). Branch-free (the
// three sign classes combined by xor / or): one exec-mask region fewer per axis in shading.
__device__ __forceinline__ bool checker_positive(float x, float y, float z) {
    const uint32_t a = sin_class(6.0f * x), b = sin_class(6.0f * y), c = sin_class(6.0f * z);
    return (((a | b | c) & 1u) | ((a ^ b ^ c) & 2u)) == 0u;   // no zero factor, even negatives
}

// pow(x, 5.0) with GLSL's undefined negative base mapped to NaN.
__device__ __forceinline__ float pow5(float x) {
    float x2 = x * x;
    float p = x2 * x2 * x;
    return (x < 0.0f) ? __builtin_nanf("") : p;
}

// Vulkan UNORM8 store: clamp to [0,1] (NaN -> 0), round to nearest.
__device__ __forceinline__ uint32_t unorm8(float x) {
    float v = (x > 0.0f) ? ((x < 1.0f) ? x : 1.0f) : 0.0f;
    return uint32_t(__builtin_fmaf(v, 255.0f, 0.5f));
}

}  // namespace rtd
