// rt_kernels.hip — the MI355X path-tracing hot path (hand-written HIP for gfx950).
//
// One fused persistent kernel replaces the reference's whole ray-tracing pipeline:
//   shaders/shader.rgen   per-pixel seed, sample loop, camera ray, depth-50 bounce loop,
//                         double accumulation, accumulator store and rgba8 tonemap
//   shaders/shader.rint   ray-sphere quadratic, t1-else-t2 report inside [tmin, tmax]
//   driver traversal      closest hit: brute force (sphere list through the scalar cache) or a
//                         stackless LBVH walk
//   shaders/shader.rchit  normal, texture, diffuse / metal / dielectric scatter
//   shaders/shader.rmiss  constant sky
//
// Execution model: a lane owns one pixel and runs that pixel's whole sample
// stream (the reference's per-pixel LCG stream, random.glsl, is sequential), flattened into one
// `segment` loop: every iteration traces one segment for every active lane; a lane whose sample
// ends starts the next sample of its pixel, a lane whose pixel ends takes a new pixel from a
// device-wide work counter (wave-batched: one atomic per refill event, ranks from the ballot),
// so lanes stay busy under divergent bounce depth until the image runs out of pixels.
#include <hip/hip_runtime.h>

#include "rt_device_math.h"
#include "rt_internal.h"

using namespace rtd;

namespace {

constexpr float T_MIN = 0.001f;               // shader.rgen:75
constexpr float T_MAX_SUCC = 0x1.388002p+13f; // successor of 10000.0f (shader.rgen:26): a report
                                              // at exactly tMax is accepted, so compare with '<'.

enum : uint32_t { ST_NEED_PIXEL = 0, ST_NEED_SAMPLE = 1, ST_TRACING = 2, ST_RETIRED = 3 };

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Driver traversal test for one sphere's AABB (src/ray_trace.cpp:586-596: center -/+ radius)
// over [T_MIN, T_MAX]; identical arithmetic to the oracle's aabb_hit.
__device__ __forceinline__ bool aabb_hit(float cx, float cy, float cz, float r, V3 o, V3 inv) {
    const float x0 = ((cx - r) - o.x) * inv.x, x1 = ((cx + r) - o.x) * inv.x;
    const float y0 = ((cy - r) - o.y) * inv.y, y1 = ((cy + r) - o.y) * inv.y;
    const float z0 = ((cz - r) - o.z) * inv.z, z1 = ((cz + r) - o.z) * inv.z;
    const float tnear = fmaxf(fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1)), T_MIN);
    const float tfar = fminf(fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)), 10000.0f);
    return tnear <= tfar;
}

// shader.rint:44-60 + the closest-hit rule for one sphere: a candidate when the quadratic
// reports t (t1 if t1 >= tmin else t2) in [tmin, best) and the ray overlaps the sphere's AABB.
// TB (tie-break): searches that do not visit spheres in index order also accept t == best from
// a lower index, so every order yields the first minimum by index.
template <bool TB>
__device__ __forceinline__ void test_sphere(float cx, float cy, float cz, float rr,
                                            const float* __restrict__ radius, V3 o, V3 d, V3 inv,
                                            float a, uint32_t id, float& best, uint32_t& bi) {
    const float ocx = o.x - cx, ocy = o.y - cy, ocz = o.z - cz;
    const float b = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
    const float D = __builtin_fmaf(b, b, -(a * c));
    if (D >= 0.0f) {
        const float sq = __builtin_sqrtf(D);
        const float t1 = (-b - sq) / a;
        const float t2 = (-b + sq) / a;
        const float t = (t1 >= T_MIN) ? t1 : t2;
        const bool better = TB ? (t < best || (t == best && id < bi)) : (t < best);
        if (t >= T_MIN && better && aabb_hit(cx, cy, cz, radius[id], o, inv)) {
            best = t;
            bi = id;
        }
    }
}

// Brute force: every lane tests every sphere. The sphere index is wave-uniform, so the geometry
// comes through the scalar cache: 8 spheres (128 B) per iteration as two s_load_dwordx16 issued
// before any of the 8 tests, feeding the VALU as SGPR operands (13 VALU per sphere, no VGPR
// loads, no LDS). The host pads geom to a multiple of 8 with spheres that can never report.
__device__ __forceinline__ void closest_brute(const rt::TraceParams& P, V3 o, V3 d, V3 inv, float a,
                                              float& best, uint32_t& bi) {
    // Constant address space: wave-uniform loads through it are emitted as s_load (the 32
    // floats of one batch merge into two s_load_dwordx16).
    typedef const __attribute__((address_space(4))) float* ConstF;
    const ConstF g = (ConstF)(P.geom);
    const uint32_t nb = (P.n_spheres + 7u) >> 3;
    for (uint32_t ib = 0; ib < nb; ++ib) {
        float b[32];
#pragma unroll
        for (uint32_t k = 0; k < 32; ++k) b[k] = g[ib * 32u + k];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k)
            test_sphere<false>(b[4 * k], b[4 * k + 1], b[4 * k + 2], b[4 * k + 3], P.radius, o, d, inv,
                               a, ib * 8u + k, best, bi);
    }
}

// LBVH: big spheres exhaustively, then the stackless escape-link walk over the small spheres.
// Node test: slab test over [T_MIN, min(T_MAX, best + cull)], evaluated with one fma per plane
// and widened by `tol` (the fma form's rounding relative to the exact slab form).
// cull = cull_abs + cull_rel * best bounds how far a candidate's AABB entry can lie beyond its
// reported t (quadratic rounding + box-vs-sphere geometry), so no node holding a candidate that
// could still win is ever skipped: the result is identical to brute force.
template <bool COUNT>
__device__ __forceinline__ void closest_lbvh(const rt::TraceParams& P, V3 o, V3 d, V3 inv, float a,
                                             float& best, uint32_t& bi, uint32_t& n_box,
                                             uint32_t& n_sph) {
    for (uint32_t k = 0; k < P.n_big; ++k) {
        const uint32_t id = P.big_ids[k];
        const rt::GeomRec s = P.geom[id];
        test_sphere<true>(s.cx, s.cy, s.cz, s.rr, P.radius, o, d, inv, a, id, best, bi);
    }
    if (COUNT) n_sph += P.n_big;
    const rt::BvhNode* __restrict__ nodes = P.nodes;
    if (nodes == nullptr) return;
    const float ox = o.x * inv.x, oy = o.y * inv.y, oz = o.z * inv.z;
    const float tol = 4.8e-7f * fmaxf(fmaxf(fabsf(ox), fabsf(oy)), fabsf(oz));
    uint32_t ni = 0;
    while (ni != 0xffffffffu) {
        const float4 n0 = *reinterpret_cast<const float4*>(&nodes[ni]);
        const float4 n1 = *(reinterpret_cast<const float4*>(&nodes[ni]) + 1);
        if (COUNT) n_box++;
        const float tx0 = __builtin_fmaf(n0.x, inv.x, -ox), tx1 = __builtin_fmaf(n1.x, inv.x, -ox);
        const float ty0 = __builtin_fmaf(n0.y, inv.y, -oy), ty1 = __builtin_fmaf(n1.y, inv.y, -oy);
        const float tz0 = __builtin_fmaf(n0.z, inv.z, -oz), tz1 = __builtin_fmaf(n1.z, inv.z, -oz);
        const float tnear = fmaxf(fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1)), T_MIN);
        const float limit = fminf(__builtin_fmaf(best, P.cull_rel, best + P.cull_abs), 10000.0f);
        const float tfar = fminf(fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1)), limit);
        const bool hit = tnear <= __builtin_fmaf(fabsf(tfar), 4.8e-7f, tfar + tol);
        const uint32_t fc = __float_as_uint(n1.w);
        if (hit && fc != 0u) {
            const uint32_t first = fc >> 4, cnt = fc & 15u;
            for (uint32_t j = 0; j < cnt; ++j) {
                const rt::GeomRec s = P.leaf_geom[first + j];
                test_sphere<true>(s.cx, s.cy, s.cz, s.rr, P.radius, o, d, inv, a,
                                  P.leaf_ids[first + j], best, bi);
            }
            if (COUNT) n_sph += cnt;
            ni = __float_as_uint(n0.w);
        } else {
            ni = hit ? ni + 1 : __float_as_uint(n0.w);
        }
    }
}

template <uint32_t ACCEL, bool COUNT>
__global__ __launch_bounds__(256) void rt_trace_kernel(const rt::TraceParams P) {
    const uint32_t lane = lane_id();
    uint32_t state = ST_NEED_PIXEL;
    uint32_t lx = 0, ly = 0, gx = 0, gy = 0, pixel_seed = 0, seed = 0, s = 0, depth = 0;
    V3 o = v3(0, 0, 0), d = v3(0, 0, 1), thr = v3(1, 1, 1);
    float a = 1.0f;
    double sum_x = 0.0, sum_y = 0.0, sum_z = 0.0;
    uint32_t n_seg = 0, n_smp = 0, n_box = 0, n_sph = 0;

    const V3 lf = v3(P.lf[0], P.lf[1], P.lf[2]);
    const V3 hor = v3(P.hor[0], P.hor[1], P.hor[2]);
    const V3 ver = v3(P.ver[0], P.ver[1], P.ver[2]);
    const V3 ulc = v3(P.ulc[0], P.ulc[1], P.ulc[2]);
    const V3 cup = v3(P.cup[0], P.cup[1], P.cup[2]);
    const V3 crt = v3(P.crt[0], P.crt[1], P.crt[2]);

    for (;;) {
        // ---- refill: lanes without a pixel take the next units of the work counter ----------
        const unsigned long long need = __ballot(state == ST_NEED_PIXEL);
        if (need) {
            const uint32_t cnt = __popcll(need);
            const int leader = __ffsll(need) - 1;
            uint32_t base = 0;
            if (int(lane) == leader) base = atomicAdd(&P.counters->work_head, cnt);
            base = __shfl(base, leader);
            if (state == ST_NEED_PIXEL) {
                const uint32_t rank = __popcll(need & ((1ull << lane) - 1ull));
                const uint32_t u = base + rank;
                if (u >= P.n_units) {
                    state = ST_RETIRED;
                } else {
                    const uint32_t t = u >> 6, w = u & 63u;
                    lx = (t % P.tiles_x) * 8u + (w & 7u);
                    ly = (t / P.tiles_x) * 8u + (w >> 3);
                    if (lx < P.band_w && ly < P.band_h) {
                        // shader.rgen:40-45
                        gx = P.off_x + lx;
                        gy = P.rows ? P.rows[ly] : P.off_y + ly;
                        const uint32_t sx = P.seed_local ? lx : gx;
                        const uint32_t sy = P.seed_local ? ly : gy;
                        pixel_seed = tea(tea(sx, sy), P.number);
                        seed = pixel_seed;
                        s = 0;
                        if (P.accumulate) {  // shader.rgen:53-55
                            const float4 acc = reinterpret_cast<const float4*>(P.accum)[size_t(ly) * P.band_w + lx];
                            sum_x = acc.x; sum_y = acc.y; sum_z = acc.z;
                        } else {
                            sum_x = sum_y = sum_z = 0.0;
                        }
                        state = ST_NEED_SAMPLE;
                    }
                }
            }
        }
        // ---- sample start (shader.rgen:56-58, 107-115) or pixel end (:61-66) --------------
        if (state == ST_NEED_SAMPLE) {
            if (s < P.spp) {
                if (P.rng_counter) seed = tea(pixel_seed, P.sample_base + s);
                float ux = float(gx) + rnd(seed);
                float uy = float(gy) + rnd(seed);
                ux = ux / P.size_x;
                uy = uy / P.size_y;
                const float lxr = rnd_pm1(seed);
                const float lyr = rnd_pm1(seed);
                const float l2 = __builtin_sqrtf(__builtin_fmaf(lyr, lyr, lxr * lxr));
                const float il = 1.0f / l2;
                const float rx = P.half_aperture * (lxr * il);
                const float ry = P.half_aperture * (lyr * il);
                const V3 from = add(lf, add(scale(rx, crt), scale(ry, cup)));
                const V3 to = sub(add(ulc, scale(ux, hor)), scale(uy, ver));
                o = from;
                d = normalize(sub(to, from));
                a = dot(d, d);
                thr = v3(1.0f, 1.0f, 1.0f);
                depth = 0;
                n_smp++;
                state = ST_TRACING;
            } else {
                const float s0 = float(sum_x), s1 = float(sum_y), s2 = float(sum_z);
                const size_t texel = size_t(ly) * P.band_w + lx;
                reinterpret_cast<float4*>(P.accum)[texel] = make_float4(s0, s1, s2, 1.0f);
                const float spp = float(P.spp);
                const uint32_t r8 = unorm8(__builtin_sqrtf(s0 / spp));
                const uint32_t g8 = unorm8(__builtin_sqrtf(s1 / spp));
                const uint32_t b8 = unorm8(__builtin_sqrtf(s2 / spp));
                P.out[texel] = r8 | (g8 << 8) | (b8 << 16) | (255u << 24);
                state = ST_NEED_PIXEL;
            }
        }
        if (__ballot(state == ST_NEED_PIXEL)) continue;   // refill before the next trace
        if (!__ballot(state == ST_TRACING)) break;         // every lane retired

        if (state == ST_TRACING) {
            // ---- one traceRayEXT (shader.rgen:75) ------------------------------------------
            float best = T_MAX_SUCC;
            uint32_t bi = 0xffffffffu;
            const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
            if (ACCEL == rt::ACCEL_BRUTE) {
                closest_brute(P, o, d, inv, a, best, bi);
                if (COUNT) n_sph += P.n_spheres;
            } else {
                closest_lbvh<COUNT>(P, o, d, inv, a, best, bi, n_box, n_sph);
            }
            n_seg++;
            V3 att;
            bool scatter = false;
            V3 sd = v3(0.0f, 0.0f, 0.0f);
            V3 p = o;
            if (bi == 0xffffffffu) {
                att = v3(0.7f, 0.8f, 1.0f);  // shader.rmiss:15
            } else {
                // shader.rint:33/37 hit attribute; shader.rchit:38-49
                p = v3(__builtin_fmaf(best, d.x, o.x), __builtin_fmaf(best, d.y, o.y),
                       __builtin_fmaf(best, d.z, o.z));
                const rt::GeomRec gc = P.geom[bi];
                const float4 m0 = reinterpret_cast<const float4*>(P.mat)[2 * bi];
                const float4 m1 = reinterpret_cast<const float4*>(P.mat)[2 * bi + 1];
                const uint32_t tt = __float_as_uint(m1.w);
                const uint32_t mtype = tt & 0xffu, ttype = tt >> 8;
                const V3 outward = normalize(sub(p, v3(gc.cx, gc.cy, gc.cz)));
                const bool front = dot(d, outward) < 0.0f;
                const V3 n = front ? outward : neg(outward);
                // shader.rchit:53-64
                att = v3(m0.x, m0.y, m0.z);
                if (ttype == 1u) {
                    const float sines = sinf_det(6.0f * p.x) * sinf_det(6.0f * p.y) * sinf_det(6.0f * p.z);
                    if (!(sines > 0.0f)) att = v3(m1.x, m1.y, m1.z);
                }
                if (mtype == 0u) {                       // diffuse, shader.rchit:68-76
                    sd = add(n, random_unit_vector(seed));
                    if (fabsf(sd.x) < 1e-8f && fabsf(sd.y) < 1e-8f && fabsf(sd.z) < 1e-8f) sd = n;
                } else if (mtype == 1u) {                // metal, shader.rchit:78-89
                    const V3 refl = reflect(d, n);
                    const V3 fuzz = scale(m0.w, random_unit_vector(seed));
                    const V3 sc = normalize(add(refl, fuzz));
                    if (dot(sc, n) > 0.0f) sd = sc;
                } else if (mtype == 2u) {                // dielectric, shader.rchit:91-100,125-133
                    const float eta = front ? (1.0f / m0.w) : m0.w;
                    const float cos_t = dot(neg(d), n);
                    bool refracts = false;
                    if (eta * __builtin_sqrtf(1.0f - cos_t * cos_t) <= 1.0f) {
                        const float q = (1.0f - eta) / (1.0f + eta);
                        const float r = q * q;
                        const float refl = r + (1.0f - r) * pow5(1.0f - cos_t);
                        refracts = refl < rnd(seed);
                    }
                    sd = refracts ? refract(d, n, eta) : reflect(d, n);
                }
                scatter = !(sd.x == 0.0f && sd.y == 0.0f && sd.z == 0.0f);  // shader.rchit:48
            }
            // ---- shader.rgen:77-88 ---------------------------------------------------------
            bool done;
            V3 col;
            if (scatter) {
                thr = mul(thr, att);
                o = p;
                d = normalize(sd);
                a = dot(d, d);
                depth++;
                done = depth >= P.max_depth;
                col = mul(thr, v3(0.0f, 0.0f, 0.0f));   // depth exhausted: light stays 0 (Q6)
            } else {
                done = true;
                col = mul(thr, att);
            }
            if (done) {
                sum_x += double(col.x);
                sum_y += double(col.y);
                sum_z += double(col.z);
                s++;
                state = ST_NEED_SAMPLE;
            }
        }
    }
    // ---- statistics: the atomic optimizer folds these into one add per wave ----------------
    atomicAdd(&P.counters->segments, (unsigned long long)n_seg);
    atomicAdd(&P.counters->samples, (unsigned long long)n_smp);
    if (COUNT) {
        atomicAdd(&P.counters->box_tests, (unsigned long long)n_box);
        atomicAdd(&P.counters->sphere_tests, (unsigned long long)n_sph);
    }
}

// Band rows -> full image rows (the reorder after the multi-GPU gather).
__global__ __launch_bounds__(256) void rt_scatter_rows_kernel(const float4* __restrict__ src_acc,
                                                              const uint32_t* __restrict__ src_px,
                                                              const uint32_t* __restrict__ rows,
                                                              uint32_t n_rows, uint32_t width,
                                                              float4* __restrict__ dst_acc,
                                                              uint32_t* __restrict__ dst_px) {
    const uint32_t r = blockIdx.y;
    if (r >= n_rows) return;
    const uint32_t dr = rows[r];
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < width; x += gridDim.x * blockDim.x) {
        if (dst_acc) dst_acc[size_t(dr) * width + x] = src_acc[size_t(r) * width + x];
        if (dst_px) dst_px[size_t(dr) * width + x] = src_px[size_t(r) * width + x];
    }
}

// Diagnostic: device evaluation of contract primitives (tests/test_gpu_parity.py).
__global__ void rt_debug_math_kernel(int op, const float* __restrict__ in, float* __restrict__ out,
                                     uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = in[2 * i], y = in[2 * i + 1];
    float r = 0.0f;
    switch (op) {
        case 0: r = __builtin_sqrtf(x); break;
        case 1: r = x / y; break;
        case 2: r = sinf_det(x); break;
        case 3: r = __builtin_fmaf(x, y, 1.0f); break;
        case 4: { V3 v = normalize(v3(x, y, 0.5f)); r = v.x; break; }
        case 5: r = pow5(x); break;
        default: r = 0.0f;
    }
    out[i] = r;
}

}  // namespace

// ---- host-callable launchers (rt_api.cpp) ---------------------------------------------------
namespace rt {

hipError_t launch_trace(const TraceParams& P, uint32_t accel, bool count, int grid, hipStream_t st) {
    dim3 g(grid), b(256);
    if (accel == ACCEL_BRUTE) {
        if (count) hipLaunchKernelGGL((rt_trace_kernel<ACCEL_BRUTE, true>), g, b, 0, st, P);
        else hipLaunchKernelGGL((rt_trace_kernel<ACCEL_BRUTE, false>), g, b, 0, st, P);
    } else {
        if (count) hipLaunchKernelGGL((rt_trace_kernel<ACCEL_LBVH, true>), g, b, 0, st, P);
        else hipLaunchKernelGGL((rt_trace_kernel<ACCEL_LBVH, false>), g, b, 0, st, P);
    }
    return hipGetLastError();
}

hipError_t trace_occupancy(uint32_t accel, bool count, int* blocks_per_cu) {
    const void* f;
    if (accel == ACCEL_BRUTE) f = count ? (const void*)rt_trace_kernel<ACCEL_BRUTE, true> : (const void*)rt_trace_kernel<ACCEL_BRUTE, false>;
    else f = count ? (const void*)rt_trace_kernel<ACCEL_LBVH, true> : (const void*)rt_trace_kernel<ACCEL_LBVH, false>;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, f, 256, 0);
}

hipError_t launch_scatter_rows(const float* src_acc, const uint8_t* src_px, const uint32_t* rows,
                               uint32_t n_rows, uint32_t width, float* dst_acc, uint8_t* dst_px,
                               hipStream_t st) {
    if (n_rows == 0 || width == 0) return hipSuccess;
    dim3 g((width + 255) / 256, n_rows), b(256);
    hipLaunchKernelGGL(rt_scatter_rows_kernel, g, b, 0, st,
                       reinterpret_cast<const float4*>(src_acc), reinterpret_cast<const uint32_t*>(src_px),
                       rows, n_rows, width, reinterpret_cast<float4*>(dst_acc),
                       reinterpret_cast<uint32_t*>(dst_px));
    return hipGetLastError();
}

hipError_t launch_debug_math(int op, const float* in, float* out, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(rt_debug_math_kernel, dim3((n + 255) / 256), dim3(256), 0, st, op, in, out, n);
    return hipGetLastError();
}

}  // namespace rt
