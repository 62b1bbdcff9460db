// rt_kernels.hip — the MI355X path-tracing hot path (hand-written HIP for gfx950).
//
// One fused persistent kernel replaces the reference's whole ray-tracing pipeline:
//   shaders/shader.rgen   per-pixel seed, sample loop, camera ray, depth-50 bounce loop,
//                         sample accumulation, accumulator store and rgba8 tonemap
//   shaders/shader.rint   ray-sphere quadratic, t1-else-t2 report inside [tmin, tmax]
//   driver traversal      closest hit: brute force (sphere list through the scalar cache) or a
//                         stackless LBVH walk (node copies in LDS, or an LDS treelet over L2)
//   shaders/shader.rchit  normal, texture, diffuse / metal / dielectric scatter
//   shaders/shader.rmiss  constant sky
//
// Execution model: a lane owns one work unit — a chunk of one pixel's samples
// (the whole pixel in the reference's per-pixel LCG stream mode, whose samples are one sequential
// chain) — flattened into one `segment` loop: every iteration traces one segment for every active
// lane; a lane whose sample ends starts the next sample of its unit, a lane whose unit ends takes
// a new one. A wave takes units 64 at a time (one chunk of one 8x8 tile) from a device-wide
// counter, longest tiles first, and hands them to its lanes as they free (ranks from the ballot),
// so lanes stay busy under divergent bounce depth until the image runs out of work.
#include <hip/hip_runtime.h>

#include "rt_device_math.h"
#include "rt_internal.h"

using namespace rtd;

namespace {

constexpr float T_MIN = 0.001f;               // shader.rgen:75
constexpr float T_MAX_SUCC = 0x1.388002p+13f; // successor of 10000.0f (shader.rgen:26): a report
                                              // at exactly tMax is accepted, so compare with '<'.

enum : uint32_t { ST_NEED_UNIT = 0, ST_NEED_SAMPLE = 1, ST_TRACING = 2, ST_RETIRED = 3 };

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Diagnostic build only (-DRT_STAMPS): wave-level s_memtime phase stamps, summed per wave and
// added to Counters::stamp[] at exit (cdna_hip_programming.md §7, In-kernel stamps). The shipped
// build compiles every STAMP() to nothing.
struct Stamps { unsigned long long acc[8], t; uint32_t cur; };
#ifdef RT_STAMPS
#define STAMP(k)                                                                               \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        unsigned long long t_;                                                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        stamps.acc[stamps.cur] += t_ - stamps.t;                                               \
        stamps.t = t_;                                                                         \
        stamps.cur = (k);                                                                      \
    } while (0)
#define STAMP_DECL                                                                             \
    Stamps stamps = {{0, 0, 0, 0, 0, 0, 0, 0}, 0, 7};                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamps.t)::"memory")
#define STAMP_FLUSH                                                                            \
    do {                                                                                       \
        STAMP(7);                                                                              \
        if (lane_id() == 0)                                                                    \
            for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&P.counters->stamp[k_], stamps.acc[k_]);  \
    } while (0)
#elif defined(RT_ASM_MARKS)   // ISA listing only: phase boundaries as comments (scripts/isa_phases.py)
#define STAMP(k) asm volatile("; RT_PHASE " #k)
#define STAMP_DECL [[maybe_unused]] Stamps stamps
#define STAMP_FLUSH do {} while (0)
#else
#define STAMP(k) do {} while (0)
#define STAMP_DECL [[maybe_unused]] Stamps stamps
#define STAMP_FLUSH do {} while (0)
#endif

// Diagnostic build only (-DRT_UTIL): lane utilisation per code point. UTIL(k, pred) counts one
// wave pass through the point and the lanes executing it with `pred` true (block totals in LDS,
// added to Counters::util at exit; rt_debug_util). Points: 0 node visit, 1 leaf test, 2 sphere
// candidate (test4 loop), 3 shade, 4 diffuse, 5 metal, 6 dielectric, 7 sample start, 8 segment
// (tracing lanes of 64), 9 unit vector draw, 10 shade of a hit, 11 node visit from L2, 12 / 13 / 14
// node visits (LDS) of passes with at most 8 / 16 / 32 active lanes.
#ifdef RT_UTIL
__shared__ unsigned long long s_util[32];
#define UTIL(k, pred)                                                                          \
    do {                                                                                       \
        const unsigned long long b_ = __ballot(pred), a_ = __ballot(true);                     \
        if (lane_id() == uint32_t(__ffsll(a_) - 1)) {                                          \
            atomicAdd(&s_util[2 * (k)], 1ull);                                                 \
            atomicAdd(&s_util[2 * (k) + 1], (unsigned long long)__popcll(b_));               \
        }                                                                                      \
    } while (0)
#define UTIL_INIT do { if (threadIdx.x < 32) s_util[threadIdx.x] = 0ull; } while (0)
#define UTIL_FLUSH                                                                             \
    do {                                                                                       \
        __syncthreads();                                                                       \
        if (threadIdx.x < 32) atomicAdd(&P.counters->util[threadIdx.x], s_util[threadIdx.x]);  \
    } while (0)
#else
#define UTIL(k, pred) do {} while (0)
#define UTIL_INIT do {} while (0)
#define UTIL_FLUSH do {} while (0)
#endif

// Diagnostic build only (-DRT_PLACEMENT): where the trace kernel's waves land. Counters::util[k]
// (k = 0..3) = waves on SIMD k over the chip; util[8 + m] = blocks whose busiest SIMD holds m of
// their waves (from the HW_ID register).
#ifdef RT_PLACEMENT
__shared__ uint32_t s_simd[4];
#define PLACEMENT_RECORD(P)                                                                    \
    do {                                                                                       \
        if (threadIdx.x < 4) s_simd[threadIdx.x] = 0u;                                         \
        __syncthreads();                                                                       \
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);                         \
        const uint32_t simd = (hw >> 4) & 3u;                                                  \
        if (lane_id() == 0) {                                                                  \
            atomicAdd(&s_simd[simd], 1u);                                                      \
            atomicAdd(&(P).counters->util[simd], 1ull);                                        \
        }                                                                                      \
        __syncthreads();                                                                       \
        if (threadIdx.x == 0) {                                                                \
            const uint32_t m = max(max(s_simd[0], s_simd[1]), max(s_simd[2], s_simd[3]));      \
            atomicAdd(&(P).counters->util[8 + min(m, 23u)], 1ull);                             \
        }                                                                                      \
    } while (0)
#else
#define PLACEMENT_RECORD(P) do {} while (0)
#endif

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

// shader.rint:44-60 + the closest-hit rule for one sphere, spheres visited in index order: a
// candidate when the quadratic reports t (t1 if t1 >= tmin else t2) in [tmin, best) and the ray
// overlaps the sphere's AABB. The roots divide by a through its reciprocal ia = 1/a, computed
// once per segment (GLSL's division is 2.5-ulp, and AMD's Vulkan compilers emit
// x * rcp(y) for it too).
template <bool GATE = true>
__device__ __forceinline__ void test_sphere(float cx, float cy, float cz, float rr,
                                            const float* __restrict__ radius, V3 o, V3 d, V3 inv,
                                            float a, float ia, uint32_t id, float& best, uint32_t& bi) {
    const float ocx = o.x - cx, ocy = o.y - cy, ocz = o.z - cz;
    const float b = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
    const float D = __builtin_fmaf(b, b, -(a * c));
    if (D >= 0.0f) {
        const float sq = sqrt_cr(D);
        const float t1 = (-b - sq) * ia;
        const float t2 = (-b + sq) * ia;
        const float t = (t1 >= T_MIN) ? t1 : t2;
        if (t >= T_MIN && t < best && (!GATE || aabb_hit(cx, cy, cz, radius[id], o, inv))) {
            best = t;
            bi = id;
        }
    }
}

// Both roots behind the origin (outside the sphere, moving away from it): no report in [tmin,
// tmax], so the exact tail need not run. Exact: a >= 0 and c >= 0 give RN(a c) >= 0, so D =
// RN(b^2 - RN(a c)) <= RN(b^2) and sqrt_cr(D) <= sqrt_cr(RN(b^2)) = b (b >= 2^-60: b^2 is normal;
// an overflowing b^2 gives t2 = +inf, rejected by t <= best); then t1 and t2 are <= 0 < tmin.
// Typical cases: the sphere a bounce ray leaves (origin on it, c >= 0 after rounding) and spheres
// behind the ray whose line still crosses them.
__device__ __forceinline__ bool behind(float b, float c) { return b >= 0x1p-60f && c >= 0.0f; }

// 16-B reload of an LDS record inside a rarely run loop (volatile: not merged with the first
// load, so the record's registers are free in between).
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 lds_reload(const float4* p) {
    const f4v v = *(const volatile __attribute__((address_space(3))) f4v*)(p);
    return make_float4(v.x, v.y, v.z, v.w);
}

// Launch parameters that a lane selects per lane, staged in LDS by every walk kernel before its
// first barrier (stage_walk_params): per grid axis the DDA step's (cell size, origin, linear cell
// stride, cell count), one 16-B load per step, and the two absolute cull slacks. Read with a
// per-lane LDS address (lgkmcnt wait only) instead of the compiler's per-lane select of
// kernel-argument addresses and a global load, whose vmcnt(0) wait also waited for every store
// and atomic the wave had in flight; and the stride and count from the table instead of per-step
// integer multiplies and a scalar reload of a kernel argument that the SGPR budget evicted
// (config 3 -3.1 %, reference stream -2.9 %, config 5 -1.3 %).
__shared__ float4 s_walk_axis[3];   // (cs[k], gmin[k], stride[k], n[k]): stride and n as uint bits
__shared__ float2 s_walk_slack;     // (cull_near_abs, cull_abs)
// ... and the grid walk's entry parameters (the widened grid box, 1 / cell size, the last cell
// index per axis) from LDS as well, instead of kernel-argument reloads (an s_load and an
// lgkmcnt(0) wait, which also drains the wave's LDS reads, at every walk's entry) and spilled
// SGPRs (together with the early big-sphere loads of setup_ray: config 3 -2.2 %, reference
// stream -4.6 %, config 5 -1.5 %).
__shared__ float4 s_walk_entry[3];   // per axis: (lo_m, hi_m, inv_cs, n - 1 as uint bits)
__device__ __forceinline__ void stage_walk_params(const rt::TraceParams& P, uint32_t tid) {
    if (tid < 3u) {
        const uint32_t stride = tid == 0u ? 1u : tid == 1u ? P.grid.n[0] : P.grid.n[0] * P.grid.n[1];
        s_walk_axis[tid] = make_float4(P.grid.cs[tid], P.grid.gmin[tid], __uint_as_float(stride),
                                       __uint_as_float(P.grid.n[tid]));
        s_walk_entry[tid] = make_float4(P.grid.lo_m[tid], P.grid.hi_m[tid], P.grid.inv_cs[tid],
                                        __uint_as_float(P.grid.n[tid] - 1u));
    }
    if (tid == 3u) s_walk_slack = make_float2(P.cull_near_abs, P.cull_abs);
}

// One DDA step of the grid walks: the axis whose boundary comes first (x before y before z on
// ties; tm = the smallest boundary t). Only the stepped coordinate can leave the grid (false:
// the ray left). The new boundary's t is recomputed from the cell coordinate, never accumulated.
__device__ __forceinline__ bool dda_step(float tm, float& tx, float& ty, float& tz, int& cx, int& cy, int& cz,
                                         int sx, int sy, int sz, uint32_t& cell, V3 o, V3 inv) {
    const bool mx = tx == tm, my = !mx && ty == tm, mz = !mx && !my;
    const float4 ax = s_walk_axis[mx ? 0 : my ? 1 : 2];
    const int s = mx ? sx : my ? sy : sz;
    const int c = (mx ? cx : my ? cy : cz) + s;
    if (uint32_t(c) >= __float_as_uint(ax.w)) return false;
    cx = mx ? c : cx;
    cy = my ? c : cy;
    cz = mz ? c : cz;
    cell = s > 0 ? cell + __float_as_uint(ax.z) : cell - __float_as_uint(ax.z);
    const float ok = mx ? o.x : my ? o.y : o.z, ik = mx ? inv.x : my ? inv.y : inv.z;
    const float tnew = (__builtin_fmaf(float(c + (s > 0 ? 1 : 0)), ax.x, ax.y) - ok) * ik;
    tx = mx ? tnew : tx;
    ty = my ? tnew : ty;
    tz = mz ? tnew : tz;
    return true;
}

// dda_step for a grid one cell thick in y (every ray is in cell row 0): the same cells in the same
// order. With one y cell a y step always leaves the grid, so the walk ends where dda_step would
// return false; only x and z step (x before z on ties, as there).
__device__ __forceinline__ bool dda_step_xz(float tm, float& tx, float ty, float& tz, int& cx, int& cz, int sx,
                                            int sz, uint32_t& cell, V3 o, V3 inv) {
    const bool mx = tx == tm;
    if (!mx && ty == tm) return false;
    const float4 ax = s_walk_axis[mx ? 0 : 2];
    const int s = mx ? sx : sz;
    const int c = (mx ? cx : cz) + s;
    if (uint32_t(c) >= __float_as_uint(ax.w)) return false;
    cx = mx ? c : cx;
    cz = mx ? cz : c;
    cell = s > 0 ? cell + __float_as_uint(ax.z) : cell - __float_as_uint(ax.z);
    const float ok = mx ? o.x : o.z, ik = mx ? inv.x : inv.z;
    const float tnew = (__builtin_fmaf(float(c + (s > 0 ? 1 : 0)), ax.x, ax.y) - ok) * ik;
    tx = mx ? tnew : tx;
    tz = mx ? tz : tnew;
    return true;
}

// Cull limit of a closest-so-far t: best + cull_abs + cull_rel best, with
// the smaller absolute slack of grid walks for t <= cull_near_t (rt_api.cpp; -1 elsewhere).
__device__ __forceinline__ float cull_limit(const rt::TraceParams& P, float t) {
    const float* slack = reinterpret_cast<const float*>(&s_walk_slack);
    const float abs_slack = slack[t <= P.cull_near_t ? 0 : 1];
    return fminf(__builtin_fmaf(t, P.cull_rel, t + abs_slack), 10000.0f);
}

// Four spheres at once (a leaf, or a batch of big spheres): the discriminants of all four are
// computed branch-free, then each lane loops over only ITS candidates (D >= 0). Inside the loop
// sits the expensive exact part (correctly rounded sqrt); t2 is computed only when t1 < tmin. The
// AABB gate is not tested here: only the segment's winner is gated, once (winner_gated).
// Candidates are accepted by (t, lowest index), so the visit order of leaves does not matter: the
// result is the brute-force closest hit. The loop reloads a candidate's record
// (rec_of, from LDS or L2) and recomputes its b and D (the same operations, so the same bits)
// instead of keeping four records and eight partial results live across it: this loop is where
// the trace kernels' register pressure peaks, and 24 fewer live VGPRs there let them run at 6
// waves per SIMD without spilling (1080p / 1000 spp: 164.7 -> 155.9 ms).
template <typename RecOf, typename IdOf>
__device__ __forceinline__ void test4(const float4 s0, const float4 s1, const float4 s2, const float4 s3,
                                      RecOf rec_of, IdOf id_of, V3 o, V3 d, V3 inv, float a, float ia,
                                      float& best, uint32_t& bi, float& limit, const rt::TraceParams& P) {
    const float4 sv[4] = {s0, s1, s2, s3};
    uint32_t cand = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float rr = sv[k].w * sv[k].w;
        const float ocx = o.x - sv[k].x, ocy = o.y - sv[k].y, ocz = o.z - sv[k].z;
        const float b = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
        const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
        cand |= (__builtin_fmaf(b, b, -(a * c)) >= 0.0f && !behind(b, c) ? 1u : 0u) << k;
    }
    while (cand) {
        UTIL(2, true);
        const uint32_t k = __builtin_ctz(cand);
        cand &= cand - 1u;
        const float4 sp = rec_of(k);
        const float rr = sp.w * sp.w;
        const float ocx = o.x - sp.x, ocy = o.y - sp.y, ocz = o.z - sp.z;
        const float b = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
        const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
        const float D = __builtin_fmaf(b, b, -(a * c));
        const float sq = sqrt_cr(D);
        float t = (-b - sq) * ia;
        if (!(t >= T_MIN)) t = (-b + sq) * ia;     // report t1 if t1 >= tmin, else t2
        if (t >= T_MIN && t <= best) {
            const uint32_t id = id_of(k);
            if (t < best || id < bi) {   // AABB gate deferred to the segment's winner (winner_gated)
                best = t;
                bi = id;
                limit = cull_limit(P, t);
            }
        }
    }
}

// One sphere (a grid cell's reference {cx, cy, cz, r^2}): test4's arithmetic for a single record,
// with r*r precomputed by the grid build (the same binary32 product). IdAt yields the sphere id
// when a candidate needs it (an LDS read, or a value loaded with the record from L2); ID_READY:
// the id is already in a register, so the two acceptance tests fold into one branch.
template <bool ID_READY = false, typename IdAt>
__device__ __forceinline__ void test1(const float4 sp, IdAt id_at, V3 o, V3 d, V3 inv,
                                      float a, float ia, float& best, uint32_t& bi, float& limit,
                                      const rt::TraceParams& P) {
    const float rr = sp.w;
    const float ocx = o.x - sp.x, ocy = o.y - sp.y, ocz = o.z - sp.z;
    const float b = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
    const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
    const float D = __builtin_fmaf(b, b, -(a * c));
    if (D >= 0.0f && !behind(b, c)) {
        UTIL(2, true);
        const float sq = sqrt_cr(D);
        float t = (-b - sq) * ia;
        if (!(t >= T_MIN)) t = (-b + sq) * ia;     // report t1 if t1 >= tmin, else t2
#ifdef RT_UTIL
        {   // grid walks: what the candidate tails find (12 beyond the closest so far, 13 the current
            // winner again from a later cell, 14 both roots below tmin, 15 passes no lane needed)
            const uint32_t idd = id_at();
            UTIL(12, t > best);
            UTIL(13, t == best && idd == bi);
            UTIL(14, !(t >= T_MIN));
            if (!__ballot((t >= T_MIN) & ((t < best) | ((t == best) & (idd < bi))))) UTIL(15, true);
        }
#endif
        if (ID_READY) {
            const uint32_t id = id_at();
            if ((t >= T_MIN) & (t <= best) & ((t < best) | (id < bi))) {   // one predicate, one branch
                best = t;
                bi = id;
                limit = cull_limit(P, t);
            }
        } else if (t >= T_MIN && t <= best) {
            const uint32_t id = id_at();
            if (t < best || id < bi) {   // AABB gate deferred to the segment's winner (winner_gated)
                best = t;
                bi = id;
                limit = cull_limit(P, t);
            }
        }
    }
}

// Brute force: every lane tests every sphere. The sphere index is wave-uniform, so the geometry
// comes through the scalar cache: 8 spheres (128 B) per iteration as two s_load_dwordx16 issued
// before any of the 8 tests, feeding the VALU as SGPR operands (13 VALU per sphere, no VGPR
// loads, no LDS). The host pads geom to a multiple of 8 with spheres that can never report.
template <bool GATE>
__device__ __forceinline__ void closest_brute(const rt::TraceParams& P, V3 o, V3 d, V3 inv, float a,
                                              float ia, float& best, uint32_t& bi) {
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
            test_sphere<GATE>(b[4 * k], b[4 * k + 1], b[4 * k + 2], b[4 * k + 3], P.radius, o, d, inv, a, ia,
                        ib * 8u + k, best, bi);
    }
}

// ---------------------------------------------------------------------------------------------
// Per-lane path state and the pieces of shader.rgen / rchit / rmiss shared by every kernel.
// ---------------------------------------------------------------------------------------------
struct Camera { V3 lf, hor, ver, ulc, cup, crt; };

__device__ __forceinline__ Camera load_camera(const rt::TraceParams& P) {
    return Camera{v3(P.lf[0], P.lf[1], P.lf[2]), v3(P.hor[0], P.hor[1], P.hor[2]),
                  v3(P.ver[0], P.ver[1], P.ver[2]), v3(P.ulc[0], P.ulc[1], P.ulc[2]),
                  v3(P.cup[0], P.cup[1], P.cup[2]), v3(P.crt[0], P.crt[1], P.crt[2])};
}

// One lane's work unit: samples [s, s_end) of pixel px. STREAM sums in double (the dvec3 of
// shader.rgen:55); HASH sums 8.24 fixed point (q) over at most kFixedFlush samples, then adds the
// partial to the pixel's 64-bit sum in HBM.
struct Path {
    uint32_t px;           // lx | ly << 16 (band-local launch id)
    uint32_t pixel_seed;   // TEA(TEA(x, y), number)
    uint32_t seed;         // LCG state (random.glsl)
    uint32_t s, s_end;     // next sample of the unit, end of the unit's samples
    uint32_t depth;        // segments traced in this sample
    uint32_t segs;         // segments traced for this unit (tile cost for the hand-out order)
    V3 thr;                // reflectedColor (shader.rgen:71)
    double sx, sy, sz;     // STREAM: dvec3 sum
    uint32_t qx, qy, qz;   // HASH: fixed-point partial sum since the last flush
};

// Global load of a rarely taken branch, waited for at once. vmcnt counts loads and stores alike
// (gfx9): a load left pending across a branch makes the compiler wait vmcnt(0) at the loop head
// (the register is reused there), which then also waits for the pixel stores still in flight —
// about 10 us per finished pixel. Waiting here, inside the branch, keeps the head
// free of it.
typedef const volatile __attribute__((address_space(1))) uint32_t* GlobalVU32;
typedef const volatile __attribute__((address_space(1))) f4v* GlobalVF4;
__device__ __forceinline__ uint32_t load_now(const uint32_t* p) {
    const uint32_t v = *(GlobalVU32)p;
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt/lgkmcnt untouched
    return v;
}
__device__ __forceinline__ float4 load_now4(const float4* p) {
    const f4v v = *(GlobalVF4)p;
    __builtin_amdgcn_s_waitcnt(0x0F70);
    return make_float4(v.x, v.y, v.z, v.w);
}

// RT_RNG_SAMPLE_HASH: LCG start of sample s of a pixel. One multiply-add
// spreads consecutive sample indices (golden ratio), then the "lowbias32" integer finaliser
// (two multiplies, three xor-shifts) scrambles: ~8 VALU per sample instead of a 16-round TEA.
__device__ __forceinline__ uint32_t sample_seed_hash(uint32_t pixel_seed, uint32_t s) {
    uint32_t x = pixel_seed + 0x9E3779B9u * s;
    x ^= x >> 16;
    x *= 0x21F0AAADu;
    x ^= x >> 15;
    x *= 0x735A2D97u;
    x ^= x >> 15;
    return x;
}

// RT_RNG_SAMPLE_HASH accumulation: a colour channel in [0, 1] as 8.24 fixed point, truncated
// (rt_internal.h kFixedFracBits). Integer sums are associative, so the order in which chunks and
// partial sums of a pixel land does not change a bit. The clamp only defines NaN (-> 0); colours
// lie in [0, 1].
__device__ __forceinline__ uint32_t sample_fixed(float c) {
    const float v = fminf(fmaxf(c, 0.0f), 1.0f) * 0x1p24f;
    return uint32_t(v);
}

// Adds fixed-point sums to a pixel's 64-bit sums in HBM (fire-and-forget relaxed atomics);
// rt_resolve_fixed_kernel stores the pixel.
__device__ __forceinline__ void add_fixed(const rt::TraceParams& P, const Path& ps, unsigned long long x,
                                          unsigned long long y, unsigned long long z) {
    const uint32_t lx = ps.px & 0xffffu, ly = ps.px >> 16;
    const size_t n = size_t(P.band_w) * P.band_h, texel = size_t(ly) * P.band_w + lx;
    __hip_atomic_fetch_add(P.fixed + texel, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(P.fixed + n + texel, y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(P.fixed + 2 * n + texel, z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-lane 64-bit unit sums in LDS (LSUM kernels: the grid kernels, whose LDS has room for them,
// 24 B per thread): the 32-bit lane partial, which must be emptied every kFixedFlush samples, is
// added here, and the unit's sum goes to HBM once when the unit ends, instead of three
// device-scope atomics per lane every kFixedFlush samples (config 3: ~486 M atomics, 16 GB of
// memory-side write requests per frame). Lane-private slots: no contention.
__shared__ unsigned long long s_lane_sum[3 * RT_TRACE_BLOCK];
// A thread's slot from the wave's first thread (wave-uniform: an SGPR) and the lane id (mbcnt),
// so no thread-id VGPR stays live across the segment loop for it.
__device__ __forceinline__ unsigned long long* lane_sum_slot() {
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
    return s_lane_sum + wave0 + __lane_id();
}
static_assert(sizeof(s_lane_sum) == rt::kLaneSumLdsBytes, "rt_internal.h");

// Empties a lane's 32-bit partial sums (every kFixedFlush samples and at the unit's end).
template <bool LSUM>
__device__ __forceinline__ void flush_fixed(const rt::TraceParams& P, Path& ps) {
    if (LSUM) {
        unsigned long long* s = lane_sum_slot();   // ds_add_u64 without return: no read back
        __hip_atomic_fetch_add(s, (unsigned long long)ps.qx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(s + RT_TRACE_BLOCK, (unsigned long long)ps.qy, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(s + 2 * RT_TRACE_BLOCK, (unsigned long long)ps.qz, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WAVEFRONT);
    } else {
        add_fixed(P, ps, ps.qx, ps.qy, ps.qz);
    }
    ps.qx = ps.qy = ps.qz = 0u;
}

// Global row of band row ly: the row map (rows), staged in LDS by the walk kernels when it fits
// their LDS plan (an lgkmcnt wait instead of a global load whose vmcnt(0) wait also drains the
// wave's stores and atomics; N > 1 strips: one per sample start), else loaded
// from global memory; without a map, off_y + ly.
extern __shared__ float4 rt_dyn_lds[];   // the dynamic LDS of the launch (the kernels' `lds`)
__device__ __forceinline__ uint32_t band_row(const rt::TraceParams& P, uint32_t ly) {
    if (!P.rows) return P.off_y + ly;
    if (P.rows_lds != rt::kNoRowsLds)
        return reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(rt_dyn_lds) + P.rows_lds)[ly];
    return load_now(P.rows + ly);
}
// (before the prologue's barrier)
__device__ __forceinline__ void stage_rows(const rt::TraceParams& P, uint32_t tid, uint32_t nthr) {
    if (!P.rows || P.rows_lds == rt::kNoRowsLds) return;
    uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(rt_dyn_lds) + P.rows_lds);
    for (uint32_t i = tid; i < P.band_h; i += nthr) dst[i] = P.rows[i];
}

// shader.rgen:40 seed of pixel w (0..63) of 8x8 tile t of the band.
__device__ __forceinline__ uint32_t tile_pixel_seed(const rt::TraceParams& P, uint32_t t, uint32_t w) {
    const uint32_t lx = (t % P.tiles_x) * 8u + (w & 7u);
    const uint32_t ly = (t / P.tiles_x) * 8u + (w >> 3);
    const uint32_t gx = P.off_x + lx;
    const uint32_t gy = band_row(P, ly < P.band_h ? ly : P.band_h - 1u);   // ragged edge: unused
    return tea(tea(P.seed_local ? lx : gx, P.seed_local ? ly : gy), P.number);
}

// Block b's tile rank, chunk c and chunk count n: the head ranks' blocks come first, n =
// head_chunks, then the others', n = chunks (TraceParams). Chunk c of n runs samples
// [chunk_begin(c, n), chunk_begin(c + 1, n)); the host keeps n * spp below 2^32.
struct BlockChunk { uint32_t rank, c, n; };

__device__ __forceinline__ BlockChunk block_chunk(const rt::TraceParams& P, uint32_t b) {
    const uint32_t hb = P.head_tiles * P.head_chunks;
    if (b < hb) {
        const uint32_t rank = b / P.head_chunks;
        return BlockChunk{rank, b - rank * P.head_chunks, P.head_chunks};
    }
    const uint32_t b2 = b - hb, r2 = b2 / P.chunks;
    return BlockChunk{P.head_tiles + r2, b2 - r2 * P.chunks, P.chunks};
}

__device__ __forceinline__ uint32_t chunk_begin(const rt::TraceParams& P, uint32_t c, uint32_t n) {
    return (c * P.spp) / n;
}

// Unit hand-out. A wave takes whole 64-unit blocks (one chunk of one 8x8 tile, one atomic) from
// the device counter and gives their pixels to its lanes as they free, so a unit costs 1/64 of an
// atomic round trip and of a hand-out-order load instead of one each; the last units (>=
// n_block_units, the last 8 Ki) go out one by one. Per-pixel atomics on the one counter were the
// cost: 1080p at 13 spp took 10.5 ms with them, 4.8 ms with tiles (scripts/refill_ab.py).
// `blk` is wave-uniform: next unit and end of the wave's current block, its tile and chunk
// sample range; `dry` once the block phase is exhausted; `done` once the per-unit phase is
// exhausted too (later refills retire lanes without touching the counter: one address, every
// atomic on it queues behind the others). `seed` (per lane) is the pixel seed of the block's pixel
// `lane`: the 64 seeds of a tile are computed together when the block is taken (two TEAs, 16
// rounds each, with every lane busy) instead of one lane at a time as its unit starts.
struct WaveBlock {
    uint32_t next = 0, end = 0, tile = 0, s0 = 0, s1 = 0;
    bool dry = false, done = false;
    uint32_t seed = 0;
};

__device__ __forceinline__ void take_block(const rt::TraceParams& P, uint32_t lane, WaveBlock& blk,
                                           uint32_t b, uint32_t tile) {
    const BlockChunk bc = block_chunk(P, b);
    blk.next = b * 64u;
    blk.end = blk.next + 64u;
    blk.tile = tile;
    blk.s0 = chunk_begin(P, bc.c, bc.n);
    blk.s1 = chunk_begin(P, bc.c + 1u, bc.n);
    blk.seed = tile_pixel_seed(P, tile, lane);
}

__device__ __forceinline__ uint32_t block_tile(const rt::TraceParams& P, uint32_t b) {
    const uint32_t rank = block_chunk(P, b).rank;
    return P.tile_order ? load_now(P.tile_order + rank) : rank;
}

template <int MODE>
__device__ __forceinline__ void begin_unit(const rt::TraceParams& P, Path& ps, uint32_t lx, uint32_t ly,
                                           uint32_t seed, uint32_t s0, uint32_t s1) {
    ps.px = lx | (ly << 16);
    ps.pixel_seed = seed;
    ps.seed = seed;
    ps.s = s0;
    ps.s_end = s1;
    ps.segs = 0;
    if (MODE == rt::MODE_HASH) {
        ps.qx = ps.qy = ps.qz = 0u;
    } else if (P.accumulate) {  // shader.rgen:53-55
        const float4 acc = load_now4(reinterpret_cast<const float4*>(P.accum) + size_t(ly) * P.band_w + lx);
        ps.sx = acc.x; ps.sy = acc.y; ps.sz = acc.z;
    } else {
        ps.sx = ps.sy = ps.sz = 0.0;
    }
}

// Tail stealing (counter-based stream only: any lane may run any sample of a pixel). Once the
// work queue is exhausted, a lane without work takes the upper half of the samples not yet started
// by the wave's lane with the most left (ties: lowest lane), one steal per call (one loop
// iteration), while the victim has at least 2 kStealMin left. The wave's last units are thus shared by its idle
// lanes instead of ending at the longest one; chunk sums are integers, so the split changes no bit.
constexpr uint32_t kStealMin = 4;

template <bool COUNT>
__device__ __forceinline__ void steal_tail(const rt::TraceParams& P, uint32_t lane, uint32_t& st, Path& ps) {
    const unsigned long long idle = __ballot(st == ST_RETIRED);
    if (!idle) return;
    const uint32_t rem = st == ST_TRACING ? ps.s_end - ps.s - 1u : st == ST_NEED_SAMPLE ? ps.s_end - ps.s : 0u;
    uint32_t key = (min(rem, (1u << 25) - 1u) << 6) | (63u - lane);
    for (int off = 32; off > 0; off >>= 1) key = max(key, (uint32_t)__shfl_xor(key, off));
    const uint32_t vrem = key >> 6;
    if (vrem < 2u * kStealMin) return;   // wave-uniform
    const int v = int(63u - (key & 63u));
    const int th = __ffsll(idle) - 1;
    const uint32_t k = vrem / 2u;
    const uint32_t vend = __shfl(ps.s_end, v), vpx = __shfl(ps.px, v), vseed = __shfl(ps.pixel_seed, v);
    if (int(lane) == v) ps.s_end -= k;
    if (COUNT && lane == 0) atomicAdd(&P.counters->steals, 1ull);
    if (int(lane) == th) {
        ps.px = vpx;
        ps.pixel_seed = vseed;
        ps.seed = vseed;
        ps.s = vend - k;
        ps.s_end = vend;
        ps.segs = 0;
        ps.qx = ps.qy = ps.qz = 0u;
        st = ST_NEED_SAMPLE;
    }
}

template <int MODE, bool COUNT>
__device__ __forceinline__ void refill(const rt::TraceParams& P, uint32_t lane, uint32_t& st, Path& ps,
                                       WaveBlock& blk, Stamps& stamps) {
    if (MODE == rt::MODE_HASH && blk.done) steal_tail<COUNT>(P, lane, st, ps);   // wave-uniform condition
    const unsigned long long need = __ballot(st == ST_NEED_UNIT);
    if (!need) return;
    STAMP(5);
    const uint32_t cnt = __popcll(need);
    const uint32_t rank = __popcll(need & ((1ull << lane) - 1ull));
    const uint32_t avail = blk.end - blk.next;
    const int leader = __ffsll(need) - 1;
    uint32_t u = 0, t = 0, s0 = blk.s0, s1 = blk.s1;
    bool per_lane = false;
    uint32_t seed = __shfl(blk.seed, int((blk.next + rank) & 63u));   // all lanes: uniform control flow
    if (rank < avail) { u = blk.next + rank; t = blk.tile; }
    if (cnt <= avail) {
        blk.next += cnt;
    } else {
        STAMP(6);
        const uint32_t rest = cnt - avail;   // lanes beyond the current block's units
        uint32_t nb = 0xffffffffu;
        if (!blk.dry) {
            if (int(lane) == leader) nb = atomicAdd(&P.counters->work_head, 64u);
            nb = __builtin_amdgcn_readfirstlane(__shfl(nb, leader));
            if (nb >= P.n_block_units) blk.dry = true;
        }
        if (!blk.dry) {
            take_block(P, lane, blk, nb >> 6, block_tile(P, nb >> 6));
            const uint32_t sn = __shfl(blk.seed, int((rank - avail) & 63u));
            if (rank >= avail) { u = nb + (rank - avail); t = blk.tile; seed = sn; s0 = blk.s0; s1 = blk.s1; }
            blk.next = nb + rest;
        } else {
            uint32_t tb = P.n_units;   // exhausted: the lanes retire
            if (!blk.done) {
                if (int(lane) == leader) tb = atomicAdd(&P.counters->work_tail, rest);
                tb = P.n_block_units + __shfl(tb, leader);
                if (tb + rest >= P.n_units) blk.done = true;
            }
            if (rank >= avail) { u = tb + (rank - avail); per_lane = true; }
            blk.next = blk.end;
        }
    }
    if (st != ST_NEED_UNIT) return;
    if (per_lane) {
        if (u >= P.n_units) { st = ST_RETIRED; return; }
        const uint32_t b = u >> 6;
        const BlockChunk bc = block_chunk(P, b);
        t = P.tile_order ? load_now(P.tile_order + bc.rank) : bc.rank;
        s0 = chunk_begin(P, bc.c, bc.n);
        s1 = chunk_begin(P, bc.c + 1u, bc.n);
    }
    const uint32_t w = u & 63u;
    const uint32_t lx = (t % P.tiles_x) * 8u + (w & 7u);
    const uint32_t ly = (t / P.tiles_x) * 8u + (w >> 3);
    if (lx >= P.band_w || ly >= P.band_h) return;   // ragged edge: stays NEED_UNIT, refetches
    if (per_lane) seed = tile_pixel_seed(P, t, w);
    begin_unit<MODE>(P, ps, lx, ly, seed, s0, s1);
    st = ST_NEED_SAMPLE;
}

// First block of a wave: by wave id, not through the counter (the host starts the counter past
// them): 16 Ki waves asking one address at once would queue for ~0.1 ms. Block ranks are dealt
// across blocks of the grid first (rank = wave-in-block * grid + block), so the longest chains of
// the LPT order start on different CUs (and XCDs) instead of sharing block 0's SIMDs.
__device__ __forceinline__ void first_block(const rt::TraceParams& P, uint32_t lane, WaveBlock& blk) {
    const uint32_t wid = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    if (wid < P.first_blocks) {
        take_block(P, lane, blk, wid, block_tile(P, wid));
        if (wid < P.isolate_blocks) blk.dry = blk.done = true;   // no work beyond its first block
    }
}

// shader.rgen:61-66: store the finished pixel (dvec3 sum rounded to float, rgba8 resolve).
__device__ __forceinline__ void store_pixel(const rt::TraceParams& P, const Path& ps) {
    const uint32_t lx = ps.px & 0xffffu, ly = ps.px >> 16;
    const float s0 = float(ps.sx), s1 = float(ps.sy), s2 = float(ps.sz);
    const size_t texel = size_t(ly) * P.band_w + lx;
    reinterpret_cast<float4*>(P.accum)[texel] = make_float4(s0, s1, s2, 1.0f);
    const float spp = float(P.spp);
    const uint32_t r8 = unorm8(__builtin_sqrtf(s0 / spp));
    const uint32_t g8 = unorm8(__builtin_sqrtf(s1 / spp));
    const uint32_t b8 = unorm8(__builtin_sqrtf(s2 / spp));
    P.out[texel] = r8 | (g8 << 8) | (b8 << 16) | (255u << 24);
}

// Finished unit. STREAM: the unit is the whole pixel: store it. HASH: flush the chunk's remaining
// partial fixed-point sum.
template <int MODE, bool LSUM>
__device__ __forceinline__ void finish_unit(const rt::TraceParams& P, Path& ps) {
    if (MODE == rt::MODE_HASH && LSUM) {   // the unit's whole sum from LDS, once
        unsigned long long* s = lane_sum_slot();
        const unsigned long long x = s[0] + ps.qx, y = s[RT_TRACE_BLOCK] + ps.qy, z = s[2 * RT_TRACE_BLOCK] + ps.qz;
        if (x | y | z) add_fixed(P, ps, x, y, z);
        s[0] = s[RT_TRACE_BLOCK] = s[2 * RT_TRACE_BLOCK] = 0ull;
        ps.qx = ps.qy = ps.qz = 0u;
    } else if (MODE == rt::MODE_HASH) {
        if (ps.qx | ps.qy | ps.qz) flush_fixed<false>(P, ps);
    } else {
        store_pixel(P, ps);
    }
}

// shader.rgen:56-58 + 107-115: camera ray of sample ps.s of the lane's unit: origin o and the
// direction before normalisation, v = to - from (the caller normalises it).
// FAST: a launch the host proved pinhole_lf for (the one-layer L2 grid kernel, lbvh_loop SPEC).
template <int MODE, bool FAST = false>
__device__ __forceinline__ void camera_ray(const rt::TraceParams& P, const Camera& cam, Path& ps, V3& o, V3& v) {
    UTIL(7, true);
    const uint32_t lx = ps.px & 0xffffu, ly = ps.px >> 16;
    const uint32_t gx = P.off_x + lx;
    const uint32_t gy = band_row(P, ly);
    if (MODE == rt::MODE_HASH) ps.seed = sample_seed_hash(ps.pixel_seed, P.sample_base + ps.s);
    else if (P.rng_counter) ps.seed = tea(ps.pixel_seed, P.sample_base + ps.s);
    float ux = float(gx) + rnd(ps.seed);
    float uy = float(gy) + rnd(ps.seed);
    // ux / size_x, correctly rounded, as one double multiply by the host's double 1/size (3 VALU
    // instead of 11): binary32 quotients lie at least 2^-49 (relative) from a binary32 rounding
    // boundary and never on one, and the double product is within 2^-52 of the quotient, so its
    // rounding to float is the correctly rounded quotient.
    ux = float(double(ux) * P.inv_size_x);
    uy = float(double(uy) * P.inv_size_y);
    const float lxr = rnd_pm1(ps.seed);
    const float lyr = rnd_pm1(ps.seed);
    V3 from;
    if (FAST || P.pinhole_lf) {   // wave-uniform (launch parameter): the reference camera (aperture 0), every
        // component of lf nonzero, crt and cup finite: rx and ry below are +-0 (or both NaN when the
        // disk sample is (0, 0)), so lf + (rx crt + ry cup) is lf itself (or NaN), without the six
        // products and sums and the 6 SGPRs of crt / cup (config 3 -0.65 %, reference stream -1.5 %,
        // config 5 -0.75 %)
        const bool nan = lxr == 0.0f && lyr == 0.0f;
        const float q = __builtin_nanf("");
        from = nan ? v3(q, q, q) : cam.lf;
    } else {
    float rx, ry;
    if (P.half_aperture != 0.0f) {   // wave-uniform (launch parameter)
        const float l2 = __builtin_sqrtf(__builtin_fmaf(lyr, lyr, lxr * lxr));
        const float il = 1.0f / l2;
        rx = P.half_aperture * (lxr * il);
        ry = P.half_aperture * (lyr * il);
    } else {
        // Pinhole (the reference camera, aperture 0): the same values without the sqrt and the
        // divide. lxr * il has the sign of lxr (il = 1/l2 > 0), so 0 * it is a zero of sign
        // sign(aperture) ^ sign(lxr); when lxr = lyr = 0 exactly, il = inf and 0 * (0 * inf) = NaN.
        const bool nan = lxr == 0.0f && lyr == 0.0f;
        const uint32_t sa = __float_as_uint(P.half_aperture) & 0x80000000u;
        rx = nan ? __builtin_nanf("") : __uint_as_float(sa ^ (__float_as_uint(lxr) & 0x80000000u));
        ry = nan ? __builtin_nanf("") : __uint_as_float(sa ^ (__float_as_uint(lyr) & 0x80000000u));
    }
    from = add(cam.lf, add(scale(rx, cam.crt), scale(ry, cam.cup)));
    }
    const V3 to = sub(add(cam.ulc, scale(ux, cam.hor)), scale(uy, cam.ver));
    o = from;
    v = sub(to, from);
    ps.thr = v3(1.0f, 1.0f, 1.0f);
    ps.depth = 0;
}

// First camera ray of a unit just taken. Returns false when the unit has no samples (spp = 0:
// stored at once); later samples start inside shade().
template <int MODE, bool LSUM, bool FAST = false>
__device__ __forceinline__ bool start_sample(const rt::TraceParams& P, const Camera& cam, Path& ps,
                                             V3& o, V3& d) {
    if (ps.s >= ps.s_end) {
        finish_unit<MODE, LSUM>(P, ps);
        return false;
    }
    V3 v;
    camera_ray<MODE, FAST>(P, cam, ps, o, v);
    d = normalize(v);
    return true;
}

// The sample's colour added to the unit's sum (shader.rgen:85-88, 59-60).
template <int MODE, bool LSUM>
__device__ __forceinline__ void sample_end(const rt::TraceParams& P, Path& ps, const V3 col) {
    ps.s++;
    if (MODE == rt::MODE_HASH) {
        ps.qx += sample_fixed(col.x);
        ps.qy += sample_fixed(col.y);
        ps.qz += sample_fixed(col.z);
        // a partial never spans a multiple of kFixedFlush samples: <= kFixedFlush * 2^24 < 2^32
        if ((ps.s & (rt::kFixedFlush - 1u)) == 0u) flush_fixed<LSUM>(P, ps);
    } else {
        ps.sx += double(col.x);
        ps.sy += double(col.y);
        ps.sz += double(col.z);
    }
}

// shader.rchit:38-133 / shader.rmiss:13-18 + shader.rgen:77-88 for one finished trace. When the
// sample ends, its colour is added to the unit's sum and the unit's next sample starts here
// (`fresh`): the scattered and the camera direction share one normalisation, and the loop head's
// sample start runs only for units just taken. Returns true when the lane traces again (o, d hold
// the next ray), false when its unit's samples are done.
// The hit sphere's records shade() reads: its geometry record and its two material records.
struct HitRec {
    float4 g, m0, m1;
};

__device__ __forceinline__ HitRec load_hit(const float4* __restrict__ geom4, const float4* __restrict__ mat4,
                                           uint32_t bi) {
    return HitRec{geom4[bi], mat4[2 * bi], mat4[2 * bi + 1]};
}

// The REC grid kernels' gate and shading records, {c, r} + the material record of a sphere side by
// side (48 B), in a static LDS table at a fixed address: a record's address is 48 bi with no base
// register (the dynamic table's two bases were spilled SGPRs reloaded every segment: config 3
// -0.5 %). Scenes of at most kRecStatic spheres (the host's choice of the form).
__shared__ float4 s_rec[3 * rt::kRecStatic];
__device__ __forceinline__ HitRec load_hit_rec(uint32_t bi) {
    return HitRec{s_rec[3 * bi], s_rec[3 * bi + 1], s_rec[3 * bi + 2]};
}

// hr: the records of sphere bi (load_hit), loaded by the caller so that they can travel with the
// winner gate's loads (lbvh_loop); unused on a miss.
template <int MODE, bool LSUM, bool FAST = false>
__device__ __forceinline__ bool shade_rec(const rt::TraceParams& P, const Camera& cam, const HitRec& hr, Path& ps,
                                          uint32_t bi, float best, V3& o, V3& d, bool& fresh) {
    V3 att;
    bool scatter = false;
    V3 sd = v3(0.0f, 0.0f, 0.0f);
    V3 p = o;
    UTIL(3, true);
    if (bi == 0xffffffffu) {
        att = v3(0.7f, 0.8f, 1.0f);  // shader.rmiss:15
    } else {
        // shader.rint:33/37 hit attribute; shader.rchit:38-49
        UTIL(10, true);
        p = v3(__builtin_fmaf(best, d.x, o.x), __builtin_fmaf(best, d.y, o.y),
               __builtin_fmaf(best, d.z, o.z));
        const float4 gc4 = hr.g;
        const float4 m0 = hr.m0;
        const float4 m1 = hr.m1;
        const uint32_t tt = __float_as_uint(m1.w);
        const uint32_t mtype = tt & 0xffu, ttype = (tt >> 8) & 0xffu;
        const V3 outward = normalize(sub(p, v3(gc4.x, gc4.y, gc4.z)));
        const bool front = dot(d, outward) < 0.0f;
        const V3 n = front ? outward : neg(outward);
        // shader.rchit:53-64
        att = v3(m0.x, m0.y, m0.z);
        if (ttype == 1u && !checker_positive(p.x, p.y, p.z)) att = v3(m1.x, m1.y, m1.z);
        // diffuse and metal both draw one random unit vector first (shader.rchit:69, :80): one
        // copy of that code serves a wave holding both materials
        V3 ru = v3(0.0f, 0.0f, 0.0f);
        if (mtype < 2u) { UTIL(9, true); ru = random_unit_vector(ps.seed); }
        if (mtype == 0u) {                       // diffuse, shader.rchit:68-76
            UTIL(4, true);
            sd = add(n, ru);
            if (fabsf(sd.x) < 1e-8f && fabsf(sd.y) < 1e-8f && fabsf(sd.z) < 1e-8f) sd = n;
        } else if (mtype == 1u) {                // metal, shader.rchit:78-89
            UTIL(5, true);
            const V3 refl = reflect(d, n);
            const V3 fuzz = scale(m0.w, ru);
            const V3 sc = normalize(add(refl, fuzz));
            if (dot(sc, n) > 0.0f) sd = sc;
        } else if (mtype == 2u) {                // dielectric, shader.rchit:91-100,125-133
            UTIL(6, true);
            // eta and r0 = ((1 - eta) / (1 + eta))^2 per face: from the record (solid dielectrics,
            // rt_internal.h make_mat) or computed here (checkered ones: colors[1] is taken)
            float eta, r;
            if (tt & rt::kMatDielConst) {
                eta = front ? m1.x : m0.w;
                r = front ? m1.y : m1.z;
            } else {
                eta = front ? (1.0f / m0.w) : m0.w;
                const float q = (1.0f - eta) / (1.0f + eta);
                r = q * q;
            }
            const float cos_t = dot(neg(d), n);
            bool refracts = false;
            if (eta * sqrt_cr(1.0f - cos_t * cos_t) <= 1.0f) {
                const float refl = r + (1.0f - r) * pow5(1.0f - cos_t);
                refracts = refl < rnd(ps.seed);
            }
            sd = refracts ? refract(d, n, eta) : reflect(d, n);
        }
        scatter = !(sd.x == 0.0f && sd.y == 0.0f && sd.z == 0.0f);  // shader.rchit:48
    }
    // shader.rgen:77-88
    V3 col, v = sd;
    bool more;
    if (scatter) {
        ps.thr = mul(ps.thr, att);
        o = p;
        ps.depth++;
        more = ps.depth < P.max_depth;
        col = mul(ps.thr, v3(0.0f, 0.0f, 0.0f));   // depth exhausted: light stays 0 (Q6)
    } else {
        col = mul(ps.thr, att);
        more = false;
    }
    if (!more) {
        sample_end<MODE, LSUM>(P, ps, col);
        if (ps.s < ps.s_end) {   // the unit's next sample
            camera_ray<MODE, FAST>(P, cam, ps, o, v);
            more = fresh = true;
        }
    }
    if (more) d = normalize(v);
    return more;
}

template <int MODE, bool LSUM>
__device__ __forceinline__ bool shade(const rt::TraceParams& P, const Camera& cam, const float4* __restrict__ geom4,
                                      const float4* __restrict__ mat4, Path& ps, uint32_t bi,
                                      float best, V3& o, V3& d, bool& fresh) {
    HitRec hr{};
    if (bi != 0xffffffffu) hr = load_hit(geom4, mat4, bi);
    return shade_rec<MODE, LSUM>(P, cam, hr, ps, bi, best, o, d, fresh);
}


// Finished unit: its chain length (traced segments) feeds the next launch's hand-out order. HASH:
// only the units of the tile's 16 pixels with even coordinates record (a quarter of the
// memory-side atomic requests; the image does not depend on the order); STREAM: every pixel, the
// frame ends with the longest chain.
template <int MODE>
__device__ __forceinline__ void record_tile_cost(const rt::TraceParams& P, const Path& ps) {
    // (P.tile_cost is set for every walk kernel, the only callers)
    if (MODE == rt::MODE_HASH && (ps.px & 0x00010001u)) return;
    const uint32_t lx = ps.px & 0xffffu, ly = ps.px >> 16;
    uint32_t* c = &P.tile_cost[(ly >> 3) * P.tiles_x + (lx >> 3)];
#ifdef RT_TILE_COST_SUM   // A/B build: order tiles by their summed chains instead
    atomicAdd(c, ps.segs);
#else
    atomicMax(c, ps.segs);
#endif
}

// Waves per SIMD the register budget is sized for. Brute force: 6 (71 VGPRs, no spills). LBVH:
// 6 (80 VGPRs) in 768-thread blocks (12 waves, 3 per SIMD), two blocks per CU: the staged octant
// tree (73 KB) and the depth-10 treelet (64 KB) fit twice in the 160 KB LDS. Measured at 1080p /
// 1000 spp (scripts/perf_variants.py): 165 ms against 193 ms for one 1024-thread
// block per CU at 4 waves per SIMD (98 VGPRs), although the 80-VGPR budget spills ~31 VGPRs
// outside the walk loop; 8 waves per SIMD (64 VGPRs) spill more and took 180 ms; blocks whose
// wave count is not a multiple of 4 (640, 896 threads) leave SIMDs unevenly loaded (+50 %).
#ifndef RT_BRUTE_WAVES_PER_SIMD
#define RT_BRUTE_WAVES_PER_SIMD 6
#endif
#ifndef RT_TRACE_WAVES_PER_SIMD
#define RT_TRACE_WAVES_PER_SIMD 6
#endif
constexpr uint32_t kBruteBlock = 256;
constexpr uint32_t kTraceBlock = RT_TRACE_BLOCK;   // one block per CU shares one staged tree / treelet

// ---------------------------------------------------------------------------------------------
// Brute-force kernel: one segment per loop iteration for every lane (the sphere loop is
// wave-uniform, so there is no traversal divergence to manage).
// ---------------------------------------------------------------------------------------------
template <bool COUNT, int MODE>
__global__ __launch_bounds__(kBruteBlock, RT_BRUTE_WAVES_PER_SIMD) void rt_trace_brute_kernel(const rt::TraceParams P) {
    const uint32_t lane = lane_id();
    const Camera cam = load_camera(P);
    uint32_t st = ST_NEED_UNIT;
    Path ps{};
    V3 o = v3(0, 0, 0), d = v3(0, 0, 1);
    uint32_t n_seg = 0, n_smp = 0, n_sph = 0;
    WaveBlock blk;
    first_block(P, lane, blk);
    STAMP_DECL;
    for (;;) {
        refill<MODE, COUNT>(P, lane, st, ps, blk, stamps);
        if (st == ST_NEED_SAMPLE) {
            if (start_sample<MODE, false>(P, cam, ps, o, d)) { st = ST_TRACING; n_smp++; }
            else st = ST_NEED_UNIT;
        }
        if (__ballot(st == ST_NEED_UNIT)) continue;   // refill before the next trace
        if (!__ballot(st == ST_TRACING)) break;        // every lane retired
        if (st == ST_TRACING) {
            float best = T_MAX_SUCC;
            uint32_t bi = 0xffffffffu;
            const V3 inv = v3(rcp_cr(d.x), rcp_cr(d.y), rcp_cr(d.z));
            const float a = dot(d, d);
            const float ia = rcp_cr(a);
            // AABB gate of the winner only: the ungated minimum is the
            // gated one when it passes; otherwise the gated pass (rare, one lane's own cost)
            closest_brute<false>(P, o, d, inv, a, ia, best, bi);
            if (bi != 0xffffffffu) {
                const float4 g = reinterpret_cast<const float4*>(P.geom)[bi];
                if (!aabb_hit(g.x, g.y, g.z, P.radius[bi], o, inv)) {
                    best = T_MAX_SUCC;
                    bi = 0xffffffffu;
                    closest_brute<true>(P, o, d, inv, a, ia, best, bi);
                }
            }
            if (COUNT) n_sph += P.n_spheres;
            n_seg++;
            ps.segs++;
            bool fresh = false;
            if (!shade<MODE, false>(P, cam, reinterpret_cast<const float4*>(P.geom),
                                    reinterpret_cast<const float4*>(P.mat), ps, bi, best, o, d, fresh)) {
                finish_unit<MODE, false>(P, ps);
                st = ST_NEED_UNIT;
            }
            if (fresh) n_smp++;
        }
    }
    atomicAdd(&P.counters->segments, (unsigned long long)n_seg);
    atomicAdd(&P.counters->samples, (unsigned long long)n_smp);
    if (COUNT) atomicAdd(&P.counters->sphere_tests, (unsigned long long)n_sph);
}

// ---------------------------------------------------------------------------------------------
// LBVH traversal state and walks.
// ---------------------------------------------------------------------------------------------
struct Ray {
    V3 o, d, inv;          // origin, direction, 1/d (the AABB gate's own reciprocals)
    float a, ia;           // dot(d, d) and its reciprocal
    float limit;           // node cull limit: min(best + cull_abs + cull_rel * best, tmax)
    float best;
    uint32_t bi;           // closest so far
    bool walk;             // the segment has a tree to walk
};
constexpr uint32_t END = 0xffffffffu;

// Walk forms (template LAYOUT): GLOBAL = escape-link BvhNode pairs from L2 (A/B reference of TOP),
// LDS1 = one node copy in LDS (AB layout), OCT = 8 octant-specialised copies in LDS, TOP = LDS
// treelet over L2 subtrees.
enum : int { LAYOUT_GLOBAL = 0, LAYOUT_LDS1 = 1, LAYOUT_OCT = 2, LAYOUT_TOP = 3, LAYOUT_GRID = 4, LAYOUT_GRID_L2 = 5,
             LAYOUT_GRID_COOP = 6, LAYOUT_GRID_CQ = 7 };

// Node slab test: one fma per plane, t = fma(plane, inv, -o * inv) (a sub-then-mul form is exact
// in the gate's own arithmetic but costs twice the issue cycles: packed f32 ops take 4 cycles on
// gfx950). Node boxes are padded at build time by 12u x (scene + camera radius),
// which covers the rounding of this form against the spheres' AABB gates.
// A zero (or denormal) direction component makes 1/d infinite; the fma form would then produce
// inf - inf = NaN for a plane on the far side of the origin and cull a box the ray runs inside, so
// the node reciprocal is clamped to +-2^100: the slab then spans (-huge, +huge) exactly when the
// origin lies inside the padded slab, which is what the gate's (plane - o) * inf gives.
// Node layout "AB" (LDS): A = (x0, y0, x1, y1), B = (z0, z1, miss link, hit link). OCT: the node
// copy is specialised to the ray's direction octant, (x0, y0, z0) are the near planes and (x1, y1,
// z1) the far ones, so no per-axis min/max is needed.
struct RayBox { V3 inv, oi; };

__device__ __forceinline__ float node_inv(float inv) {
    return __builtin_isinf(inv) ? __builtin_copysignf(0x1p100f, inv) : inv;
}
__device__ __forceinline__ RayBox ray_box(const V3 o, const V3 inv) {
    const V3 n = v3(node_inv(inv.x), node_inv(inv.y), node_inv(inv.z));
    return RayBox{n, v3(o.x * n.x, o.y * n.y, o.z * n.z)};
}

template <uint32_t NOCT>   // node copies per ray direction class: 1 (none) or 8 (octants)
__device__ __forceinline__ bool node_hit(const float4 A, const float4 B, const RayBox& q, float limit) {
    const float tx0 = __builtin_fmaf(A.x, q.inv.x, -q.oi.x), ty0 = __builtin_fmaf(A.y, q.inv.y, -q.oi.y);
    const float tx1 = __builtin_fmaf(A.z, q.inv.x, -q.oi.x), ty1 = __builtin_fmaf(A.w, q.inv.y, -q.oi.y);
    const float tz0 = __builtin_fmaf(B.x, q.inv.z, -q.oi.z), tz1 = __builtin_fmaf(B.y, q.inv.z, -q.oi.z);
    float tn, tf;
    if (NOCT == 8) {
        tn = fmaxf(fmaxf(tx0, ty0), fmaxf(tz0, T_MIN));
        tf = fminf(fminf(tx1, ty1), tz1);
    } else {
        tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), T_MIN));
        tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    }
    // == tn <= min(tf, limit): limit is never NaN, so splitting the min into a second compare
    // gives the same answer without re-canonicalising the loop-invariant limit every visit.
    return tn <= tf && tn <= limit;
}

// 16-B load from an LDS address held in a register (ds_read_b128 addr, no base add).
__device__ __forceinline__ float4 lds_f4(uint32_t addr) {
    const f4v v = *(const __attribute__((address_space(3))) f4v*)(uintptr_t)addr;
    return make_float4(v.x, v.y, v.z, v.w);
}

// Octant of a direction: bit k set when component k is negative (sign bit, so -0 -> 1/d = -inf
// counts as negative, matching the copy whose near plane is the box's high side).
__device__ __forceinline__ uint32_t octant(const V3 d) {
    return (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) | ((__float_as_uint(d.z) >> 31) << 2);
}

// Four big spheres (records sb, ids ib; SGPR operands): the discriminants, then a candidate tail
// per sphere that any lane needs (wave-uniform record: no reload, no per-lane select).
__device__ __forceinline__ void big_group(Ray& r, const float (&sb)[16], const uint32_t (&ib)[4]) {
    float bk[4], Dk[4];
    uint32_t cand = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float rr = sb[4 * k + 3] * sb[4 * k + 3];
        const float ocx = r.o.x - sb[4 * k], ocy = r.o.y - sb[4 * k + 1], ocz = r.o.z - sb[4 * k + 2];
        bk[k] = __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
        const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
        Dk[k] = __builtin_fmaf(bk[k], bk[k], -(r.a * c));
        cand |= (Dk[k] >= 0.0f && !behind(bk[k], c) ? 1u : 0u) << k;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if ((cand >> k) & 1u) {
            const float sq = sqrt_cr(Dk[k]);
            float t = (-bk[k] - sq) * r.ia;
            if (!(t >= T_MIN)) t = (-bk[k] + sq) * r.ia;   // report t1 if t1 >= tmin, else t2
            const uint32_t id = ib[k];
            if ((t >= T_MIN) & (t <= r.best) & ((t < r.best) | (id < r.bi))) {
                r.best = t;
                r.bi = id;
            }
        }
    }
}

// New segment: hoisted per-ray terms and the exhaustive big spheres.
template <bool FAST = false>   // FAST: at most 4 big spheres (the one-layer L2 grid kernel, lbvh_loop SPEC)
__device__ __forceinline__ void setup_ray(const rt::TraceParams& P, Ray& r) {
    // records and ids through the scalar cache (TraceParams::big_tab, SGPR operands, no LDS round
    // trip: config 3 -1.6 %, reference stream -1.7 %, config 5 -2.2 % against an LDS table); the
    // four discriminants stay in registers for the candidate passes, which run per sphere with a
    // wave-uniform record (no reload, no per-lane record select)
    typedef const __attribute__((address_space(4))) float* ConstF;
    typedef const __attribute__((address_space(4))) uint32_t* ConstU;
    const ConstF g = (ConstF)(P.big_tab);
    const ConstU gid = (ConstU)(P.big_tab + 4u * rt::kBigMax);
    // the first four records and ids are requested before the reciprocals, so the scalar loads'
    // latency runs under them (the table always holds kBigMax entries: reading the first four is
    // safe whatever n_big); the ids come with the records, not one dependent load per candidate
    float sb0[16];
    uint32_t ib0[4];
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) sb0[k] = g[k];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) ib0[k] = gid[k];
    r.a = dot(r.d, r.d);
    r.ia = rcp_cr(r.a);
    r.inv = v3(rcp_cr(r.d.x), rcp_cr(r.d.y), rcp_cr(r.d.z));
    // closest so far: none, with t <= tMax (shader.rint:32-39 reports t <= tMax). The walks accept
    // (t <= best, lowest id on ties), so best = 10000 exactly accepts a report at tMax and nothing
    // beyond it, and the (t bits, id) keys of the cooperative walk order the same way.
    r.best = 10000.0f;
    r.bi = 0xffffffffu;
    big_group(r, sb0, ib0);   // (without big spheres the table holds four inert records: no test)
    for (uint32_t k0 = 4; !FAST && k0 < P.n_big; k0 += 4) {
        float sb[16];
        uint32_t ib[4];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) sb[k] = g[k0 * 4u + k];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) ib[k] = gid[k0 + k];
        big_group(r, sb, ib);
    }
    r.limit = cull_limit(P, r.best);
    r.walk = P.nodes != nullptr || P.cell_start != nullptr;
}

// Leaf of 4 slots (dummy-padded), loads issued together; the candidate loop reloads a record
// (test4 RELOAD) from LDS (LDS_LEAF: staged leaves) or from L2. Reloading from L2 in the treelet
// kernel measured 6.5 % faster (config 5 at 20 spp: 39.6 -> 37.0 ms; its spills 34 -> 0).
template <bool COUNT, bool LDS_LEAF>
__device__ __forceinline__ void leaf_test(const rt::TraceParams& P, const float4* __restrict__ leaf4,
                                          const uint32_t* __restrict__ leaf_ids, uint32_t first,
                                          uint32_t count, Ray& r, uint32_t& n_sph) {
    const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
    test4(s0, s1, s2, s3, [&](uint32_t k) {
                       if (LDS_LEAF) return lds_reload(leaf4 + first + k);
                       const f4v v = *(const volatile __attribute__((address_space(1))) f4v*)(leaf4 + first + k);
                       return make_float4(v.x, v.y, v.z, v.w);
                   },
                    [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a, r.ia, r.best,
                    r.bi, r.limit, P);
    if (COUNT) n_sph += count;
}

// Escape-link walk over BvhNode pairs in global memory (L2), nodes [gi, bound): escape in lo.w,
// leaf field (first << 4 | count, 0 = inner) in hi.w. While-while (Aila & Laine 2009): the cheap
// node loop runs until every lane has found a hit leaf or left the range; then the pending leaves
// are tested together.
template <bool COUNT>
__device__ __forceinline__ void walk_global_range(const rt::TraceParams& P, const float4* __restrict__ gnodes,
                                                  const float4* __restrict__ leaf4,
                                                  const uint32_t* __restrict__ leaf_ids, const RayBox& q,
                                                  uint32_t gi, uint32_t bound, Ray& r, uint32_t& n_box,
                                                  uint32_t& n_sph) {
    uint32_t pending = 0u;
    for (;;) {
        while (gi < bound && pending == 0u) {
            UTIL(11, true);
            const float4 n0 = gnodes[2 * gi];
            const float4 n1 = gnodes[2 * gi + 1];
            if (COUNT) n_box++;
            const bool h = node_hit<1>(make_float4(n0.x, n0.y, n1.x, n1.y), make_float4(n0.z, n1.z, 0.0f, 0.0f),
                                       q, r.limit);
            const uint32_t fc = __float_as_uint(n1.w);
            if (h && fc != 0u) pending = fc;
            gi = (h && fc == 0u) ? gi + 1u : __float_as_uint(n0.w);
        }
        if (pending == 0u) break;
        leaf_test<COUNT, false>(P, leaf4, leaf_ids, pending >> 4, pending & 15u, r, n_sph);
        pending = 0u;
    }
}

// Uniform-grid walk (ACCEL_GRID, rt_grid.h): a 3D DDA from the ray's entry into the grid box
// (widened by the registration margin, over [tmin, limit], in the AABB gate's arithmetic) through
// the cells in order of t, testing each cell's references, until the next cell starts beyond the
// cull limit or the ray leaves the grid. Every cell boundary's t is computed afresh from the cell
// coordinate (no accumulated rounding), so the cells visited cover the ray up to rounding distance
// of the boundaries, which the margin covers. Ties step one axis at a time (an
// extra cell, never a skipped one).
template <bool COUNT, bool PAIRS, bool FLAT = false>
__device__ __forceinline__ void grid_walk(const rt::TraceParams& P, const uint32_t* __restrict__ cstart,
                                          const float4* __restrict__ rec, const uint32_t* __restrict__ ids,
                                          Ray& r, uint32_t& n_cell, uint32_t& n_sph, uint32_t& n_empty) {
    // grid parameters from the block's LDS tables (stage_walk_params), not from the kernel arguments
    const float4 ex = s_walk_entry[0], ey = s_walk_entry[1], ez = s_walk_entry[2];
    const float4 axx = s_walk_axis[0], axy = s_walk_axis[1], axz = s_walk_axis[2];
    const float lo0 = ex.x, lo1 = ey.x, lo2 = ez.x, hi0 = ex.y, hi1 = ey.y, hi2 = ez.y;
    const float ics[3] = {ex.z, ey.z, ez.z}, gmn[3] = {axx.y, axy.y, axz.y}, csz[3] = {axx.x, axy.x, axz.x};
    const int nm1[3] = {int(__float_as_uint(ex.w)), int(__float_as_uint(ey.w)), int(__float_as_uint(ez.w))};
    const uint32_t n0 = __float_as_uint(axx.w), n1 = __float_as_uint(axy.w);
    const float x0 = (lo0 - r.o.x) * r.inv.x, x1 = (hi0 - r.o.x) * r.inv.x;
    const float y0 = (lo1 - r.o.y) * r.inv.y, y1 = (hi1 - r.o.y) * r.inv.y;
    const float z0 = (lo2 - r.o.z) * r.inv.z, z1 = (hi2 - r.o.z) * r.inv.z;
    const float tn = fmaxf(fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1)), T_MIN);
    const float tf = fminf(fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)), r.limit);
    if (!(tn <= tf)) return;
    // entry cell (clamped: a point rounded just outside belongs to the border cell)
    auto cell_of = [&](float p, int k) {
        const int c = int(floorf((p - gmn[k]) * ics[k]));
        return min(max(c, 0), nm1[k]);
    };
    int cx = cell_of(__builtin_fmaf(tn, r.d.x, r.o.x), 0);
    int cy = FLAT ? 0 : cell_of(__builtin_fmaf(tn, r.d.y, r.o.y), 1);
    int cz = cell_of(__builtin_fmaf(tn, r.d.z, r.o.z), 2);
    const int sx = r.d.x > 0.0f ? 1 : (r.d.x < 0.0f ? -1 : 0);
    const int sy = r.d.y > 0.0f ? 1 : (r.d.y < 0.0f ? -1 : 0);
    const int sz = r.d.z > 0.0f ? 1 : (r.d.z < 0.0f ? -1 : 0);
    // t of the boundary ahead on each axis (+inf on an axis the ray does not move along)
    auto bound_t = [&](int c, int s, int k, float o, float inv) {
        const float plane = __builtin_fmaf(float(c + (s > 0 ? 1 : 0)), csz[k], gmn[k]);
        return s == 0 ? __builtin_inff() : (plane - o) * inv;
    };
    float tx = bound_t(cx, sx, 0, r.o.x, r.inv.x);
    float ty = bound_t(cy, sy, 1, r.o.y, r.inv.y);
    float tz = bound_t(cz, sz, 2, r.o.z, r.inv.z);
    // linear cell index (a step adds the stepped axis's stride, dda_step)
    uint32_t cell = FLAT ? uint32_t(cz) * n0 + uint32_t(cx) : (uint32_t(cz) * n1 + uint32_t(cy)) * n0 + uint32_t(cx);
    // One-layer grid walked from L2 (config 5): the DDA steps before the cell's references are
    // tested (the step does not depend on them; the cull test still uses this cell's exit t and the
    // limit they leave), so the next cell's two offsets are requested before this cell's records
    // and arrive while they are tested: one dependent L2 round trip per cell instead of two, the
    // same cells and references in the same order. Config 5 -0.3 % (1 000 spp) / -0.9 % (100 spp),
    // no new spills.
    if constexpr (FLAT && PAIRS) {
        uint32_t b = cstart[cell], e = cstart[cell + 1];
        for (;;) {
            const float tm = fminf(fminf(tx, ty), tz);
            uint32_t ncell = cell;   // unchanged when the step leaves the grid: a valid address
            const bool more = dda_step_xz(tm, tx, ty, tz, cx, cz, sx, sz, ncell, r.o, r.inv);
            const uint32_t nb = cstart[ncell], ne = cstart[ncell + 1];
            if (COUNT) {
                n_cell++;
                n_empty += b == e ? 1u : 0u;
            }
            uint32_t j = b;
            for (; j + 1 < e; j += 2) {
                UTIL(1, true);
                const float4 s0 = rec[j], s1 = rec[j + 1];
                const uint32_t i0 = ids[j], i1 = ids[j + 1];
                test1<true>(s0, [&] { return i0; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
                test1<true>(s1, [&] { return i1; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
                if (COUNT) n_sph += 2;
            }
            if (j < e) {
                UTIL(1, true);
                const float4 s0 = rec[j];
                const uint32_t i0 = ids[j];
                test1<true>(s0, [&] { return i0; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
                if (COUNT) n_sph++;
            }
            UTIL(0, true);
            if (!(tm <= r.limit) || !more) break;
            b = nb;
            e = ne;
            cell = ncell;
        }
        return;
    }
    for (;;) {
        // the cell's reference run [b, e): from L2 through one address, so both offsets come in one
        // 8-byte load (config 5 -1.0 %); the LDS pair is one ds_read2 either way
        const uint32_t* cp = cstart + cell;
        const uint32_t b = PAIRS ? cp[0] : cstart[cell], e = PAIRS ? cp[1] : cstart[cell + 1];
        if (COUNT) {
            n_cell++;
            n_empty += b == e ? 1u : 0u;
        }
        uint32_t j = b;
        if (PAIRS) {   // references from L2: two at a time (two record loads in flight; config 5 -3.5 %)
          // the ids are loaded with the records (one L2 round trip instead of a second, dependent
          // one for every candidate that passes the t test)
          for (; j + 1 < e; j += 2) {
            UTIL(1, true);
            const float4 s0 = rec[j], s1 = rec[j + 1];
            const uint32_t i0 = ids[j], i1 = ids[j + 1];
            test1<true>(s0, [&] { return i0; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
            test1<true>(s1, [&] { return i1; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
            if (COUNT) n_sph += 2;
          }
          if (j < e) {
            UTIL(1, true);
            const float4 s0 = rec[j];
            const uint32_t i0 = ids[j];
            test1<true>(s0, [&] { return i0; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
            if (COUNT) n_sph++;
            ++j;
          }
        }
        if (!PAIRS && j < e) {   // LDS: two records in flight, no register copies (unrolled by two)
            float4 A = rec[j], B;
            for (;;) {
                UTIL(1, true);
                B = rec[j + 1];   // one past the run: the next cell's record or the id array (LDS)
                test1(A, [&] { return ids[j]; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
                if (COUNT) n_sph++;
                if (++j >= e) break;
                UTIL(1, true);
                A = rec[j + 1];
                test1(B, [&] { return ids[j]; }, r.o, r.d, r.inv, r.a, r.ia, r.best, r.bi, r.limit, P);
                if (COUNT) n_sph++;
                if (++j >= e) break;
            }
        }
        UTIL(0, true);
        const float tm = fminf(fminf(tx, ty), tz);
        if (!(tm <= r.limit)) break;   // the next cell starts beyond every closer candidate
        if (FLAT) {
            if (!dda_step_xz(tm, tx, ty, tz, cx, cz, sx, sz, cell, r.o, r.inv)) break;
        } else if (!dda_step(tm, tx, ty, tz, cx, cy, cz, sx, sy, sz, cell, r.o, r.inv)) {
            break;
        }
    }
}

// Compiler-only ordering of LDS accesses made by different lanes of one wave: the LDS executes a
// wave's instructions in issue order, so no wait or barrier is needed, only no reordering.
__device__ __forceinline__ void lane_order() { asm volatile("" ::: "memory"); }

// ---- wave-wide candidate queue (LAYOUT_GRID_CQ) --------------------------------
// The LDS grid walk with the candidate tails (sqrt, roots, acceptance) taken out of the divergent
// reference loop: a reference whose discriminant passes is pushed as (lane, reference) into a
// per-wave LDS queue (ballot ranks), and at the end of each cell the wave's walking lanes resolve
// the queue together, every lane taking entries, before any of them takes its DDA step. An entry's
// ray comes from its owner lane by ds_bpermute (every owner is active at the flush: it pushed in
// this cell), its candidate lowers the owner's (t bits, id) key by an LDS 64-bit atomic minimum
// (t >= tmin > 0: the u64 minimum is the walks' (t, lowest id) rule). Per-lane queue overflow
// (more than kCqCap entries in one cell) falls back to the lane's own tail. The cells visited, the
// references tested and the closest hit are grid_walk's: bit-exact.
constexpr uint32_t kCqCap = 128;   // queue entries per wave
__shared__ uint32_t s_cq_q[kCqCap * (RT_TRACE_BLOCK / 64)];
__shared__ unsigned long long s_cq_key[RT_TRACE_BLOCK];
__shared__ uint32_t s_cq_n[RT_TRACE_BLOCK / 64];
static_assert(sizeof(s_cq_q) + sizeof(s_cq_key) + sizeof(s_cq_n) == rt::kCqLdsBytes, "rt_internal.h");

template <bool COUNT>
__device__ __forceinline__ void grid_walk_cq(const rt::TraceParams& P, const uint32_t* __restrict__ cstart,
                                             const float4* __restrict__ rec, const uint32_t* __restrict__ ids,
                                             Ray& r, uint32_t& n_cell, uint32_t& n_sph, uint32_t& n_empty) {
    const rt::GridInfo& G = P.grid;
    const float x0 = (G.lo_m[0] - r.o.x) * r.inv.x, x1 = (G.hi_m[0] - r.o.x) * r.inv.x;
    const float y0 = (G.lo_m[1] - r.o.y) * r.inv.y, y1 = (G.hi_m[1] - r.o.y) * r.inv.y;
    const float z0 = (G.lo_m[2] - r.o.z) * r.inv.z, z1 = (G.hi_m[2] - r.o.z) * r.inv.z;
    const float tn = fmaxf(fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1)), T_MIN);
    const float tf = fminf(fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)), r.limit);
    if (!(tn <= tf)) return;
    auto cell_of = [&](float p, int k) {
        const int c = int(floorf((p - G.gmin[k]) * G.inv_cs[k]));
        return min(max(c, 0), int(G.n[k]) - 1);
    };
    int cx = cell_of(__builtin_fmaf(tn, r.d.x, r.o.x), 0);
    int cy = cell_of(__builtin_fmaf(tn, r.d.y, r.o.y), 1);
    int cz = cell_of(__builtin_fmaf(tn, r.d.z, r.o.z), 2);
    const int sx = r.d.x > 0.0f ? 1 : (r.d.x < 0.0f ? -1 : 0);
    const int sy = r.d.y > 0.0f ? 1 : (r.d.y < 0.0f ? -1 : 0);
    const int sz = r.d.z > 0.0f ? 1 : (r.d.z < 0.0f ? -1 : 0);
    auto bound_t = [&](int c, int s, int k, float o, float inv) {
        const float plane = __builtin_fmaf(float(c + (s > 0 ? 1 : 0)), G.cs[k], G.gmin[k]);
        return s == 0 ? __builtin_inff() : (plane - o) * inv;
    };
    float tx = bound_t(cx, sx, 0, r.o.x, r.inv.x);
    float ty = bound_t(cy, sy, 1, r.o.y, r.inv.y);
    float tz = bound_t(cz, sz, 2, r.o.z, r.inv.z);
    uint32_t cell = (uint32_t(cz) * G.n[1] + uint32_t(cy)) * G.n[0] + uint32_t(cx);
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* const q = s_cq_q + wave * kCqCap;
    unsigned long long* const key = s_cq_key + wave * 64u;
    for (;;) {
        const uint32_t b = cstart[cell], e = cstart[cell + 1];
        if (COUNT) {
            n_cell++;
            n_empty += b == e ? 1u : 0u;
        }
        s_cq_n[wave] = 0u;   // every active lane writes the same value
        lane_order();
        uint32_t qn = 0u;   // equal on every lane still in the reference loop (they ran the same pushes)
        for (uint32_t j = b; j < e; ++j) {
            UTIL(1, true);
            const float4 sp = rec[j];
            const float ocx = r.o.x - sp.x, ocy = r.o.y - sp.y, ocz = r.o.z - sp.z;
            const float bb = __builtin_fmaf(ocz, r.d.z, __builtin_fmaf(ocy, r.d.y, ocx * r.d.x));
            const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - sp.w;
            const float D = __builtin_fmaf(bb, bb, -(r.a * c));
            if (COUNT) n_sph++;
            const bool cand = D >= 0.0f && !behind(bb, c);
            const unsigned long long m = __ballot(cand);
            if (m) {   // wave-uniform
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
                const uint32_t slot = qn + rank;
                qn = min(qn + uint32_t(__popcll(m)), kCqCap);
                if (cand) {
                    if (rank == 0u) s_cq_n[wave] = qn;
                    if (slot < kCqCap) {
                        q[slot] = lane | (j << 6);
                    } else {   // the queue is full: this lane's own tail (rare)
                        UTIL(2, true);
                        const float sq = sqrt_cr(D);
                        float t = (-bb - sq) * r.ia;
                        if (!(t >= T_MIN)) t = (-bb + sq) * r.ia;
                        const uint32_t id = ids[j];
                        if ((t >= T_MIN) & (t <= r.best) & ((t < r.best) | (id < r.bi))) {
                            r.best = t;
                            r.bi = id;
                        }
                    }
                }
            }
        }
        lane_order();
        const uint32_t qtot = __builtin_amdgcn_readfirstlane(s_cq_n[wave]);
        if (qtot) {   // resolve the cell's candidates with every walking lane
            key[lane] = (static_cast<unsigned long long>(__float_as_uint(r.best)) << 32) | r.bi;
            lane_order();
            const unsigned long long act = __ballot(true);
            const uint32_t rk = __builtin_amdgcn_mbcnt_hi(uint32_t(act >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(act), 0u));
            const uint32_t nact = __popcll(act);
            for (uint32_t base = 0; base < qtot; base += nact) {   // wave-uniform trip count
                const uint32_t k = base + rk;
                const bool valid = k < qtot;
                const uint32_t ent = q[valid ? k : 0u];
                const int L = int(ent & 63u);
                const uint32_t jj = ent >> 6;
                const V3 o = v3(__shfl(r.o.x, L), __shfl(r.o.y, L), __shfl(r.o.z, L));
                const V3 d = v3(__shfl(r.d.x, L), __shfl(r.d.y, L), __shfl(r.d.z, L));
                const float a = __shfl(r.a, L), ia = __shfl(r.ia, L);
                UTIL(2, valid);
                const float4 sp = rec[jj];
                const uint32_t id = ids[jj];
                const float ocx = o.x - sp.x, ocy = o.y - sp.y, ocz = o.z - sp.z;
                const float bb = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
                const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - sp.w;
                const float D = __builtin_fmaf(bb, bb, -(a * c));   // the push's D: >= 0
                const float sq = sqrt_cr(D);
                float t = (-bb - sq) * ia;
                if (!(t >= T_MIN)) t = (-bb + sq) * ia;   // report t1 if t1 >= tmin, else t2
                if (valid && t >= T_MIN)
                    __hip_atomic_fetch_min(&key[L], (static_cast<unsigned long long>(__float_as_uint(t)) << 32) | id,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            lane_order();
            const unsigned long long kk = key[lane];
            r.best = __uint_as_float(uint32_t(kk >> 32));
            r.bi = uint32_t(kk);
        }
        r.limit = cull_limit(P, r.best);
        UTIL(0, true);
        const float tm = fminf(fminf(tx, ty), tz);
        if (!(tm <= r.limit)) break;   // the next cell starts beyond every closer candidate
        if (!dda_step(tm, tx, ty, tz, cx, cy, cz, sx, sy, sz, cell, r.o, r.inv)) break;
    }
}

// ---- wave-cooperative grid walk (LAYOUT_GRID_COOP) ---------------------------
// Wave64 inclusive scans through DPP: row_shr 1/2/4/8 inside each 16-lane row (zero fill), then
// row_bcast:15 (lane 15 of rows 0 / 2 into rows 1 / 3) and row_bcast:31 (lane 31 into rows 2, 3).
// Every lane of the wave must be active (exec full): DPP reads disabled lanes as the fill value.
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) {
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false)));
    return v;
}

// Per wave (64 slots of its block's arrays): the rays of the segment (o, a | d, 1/a), the closest
// hit so far as a (t bits, sphere id) key, and the slot markers of one pass.
__shared__ float4 s_coop_ray[2 * RT_TRACE_BLOCK];
__shared__ unsigned long long s_coop_key[RT_TRACE_BLOCK];
__shared__ uint32_t s_coop_mark[RT_TRACE_BLOCK];
static_assert(sizeof(s_coop_ray) + sizeof(s_coop_key) + sizeof(s_coop_mark) == rt::kCoopLdsBytes, "rt_internal.h");

// The grid walk of grid_walk with the reference tests of a wave's rays spread over all 64 lanes.
// Rounds: every walking lane takes its current cell's n references; an exclusive scan of n gives
// each ray its run [start, start + n) of the round's `total` (ray, reference) pairs, which the
// wave tests in ceil(total / 64) passes with every lane busy instead of max-over-lanes passes at
// one reference per lane. A pass finds each slot's ray by a max-scan of the runs' start markers;
// a candidate lowers its ray's key by an LDS 64-bit atomic minimum. t >= tmin > 0, so the float
// bits order like the values and the u64 minimum of (t bits << 32 | id) is exactly the walks'
// (t, lowest id) rule: the order of tests cannot change the result. After the passes each ray
// reads its key, updates its cull limit and takes its DDA step, as grid_walk does after a cell:
// the cells visited, the references tested and the closest hit are grid_walk's. Called with every
// lane of the wave (tracing or not), never inside divergent control flow.
template <bool COUNT>
__device__ __forceinline__ void grid_walk_coop(const rt::TraceParams& P, const uint32_t* __restrict__ cstart,
                                               const float4* __restrict__ rec, const uint32_t* __restrict__ ids,
                                               Ray& r, bool tracing, uint32_t& n_cell, uint32_t& n_sph) {
    const rt::GridInfo& G = P.grid;
    const uint32_t lane = lane_id();
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
    float4* const rayA = s_coop_ray + wave0;
    float4* const rayB = s_coop_ray + RT_TRACE_BLOCK + wave0;
    unsigned long long* const key = s_coop_key + wave0;
    uint32_t* const mark = s_coop_mark + wave0;
    bool walking = tracing && r.walk;
    int cx = 0, cy = 0, cz = 0, sx = 0, sy = 0, sz = 0;
    float tx = 0.0f, ty = 0.0f, tz = 0.0f;
    uint32_t cell = 0;
    if (walking) {   // entry cell and DDA state: grid_walk's arithmetic
        const float x0 = (G.lo_m[0] - r.o.x) * r.inv.x, x1 = (G.hi_m[0] - r.o.x) * r.inv.x;
        const float y0 = (G.lo_m[1] - r.o.y) * r.inv.y, y1 = (G.hi_m[1] - r.o.y) * r.inv.y;
        const float z0 = (G.lo_m[2] - r.o.z) * r.inv.z, z1 = (G.hi_m[2] - r.o.z) * r.inv.z;
        const float tn = fmaxf(fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1)), T_MIN);
        const float tf = fminf(fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)), r.limit);
        walking = tn <= tf;
        if (walking) {
            auto cell_of = [&](float p, int k) {
                const int c = int(floorf((p - G.gmin[k]) * G.inv_cs[k]));
                return min(max(c, 0), int(G.n[k]) - 1);
            };
            cx = cell_of(__builtin_fmaf(tn, r.d.x, r.o.x), 0);
            cy = cell_of(__builtin_fmaf(tn, r.d.y, r.o.y), 1);
            cz = cell_of(__builtin_fmaf(tn, r.d.z, r.o.z), 2);
            sx = r.d.x > 0.0f ? 1 : (r.d.x < 0.0f ? -1 : 0);
            sy = r.d.y > 0.0f ? 1 : (r.d.y < 0.0f ? -1 : 0);
            sz = r.d.z > 0.0f ? 1 : (r.d.z < 0.0f ? -1 : 0);
            auto bound_t = [&](int c, int s, int k, float o, float inv) {
                const float plane = __builtin_fmaf(float(c + (s > 0 ? 1 : 0)), G.cs[k], G.gmin[k]);
                return s == 0 ? __builtin_inff() : (plane - o) * inv;
            };
            tx = bound_t(cx, sx, 0, r.o.x, r.inv.x);
            ty = bound_t(cy, sy, 1, r.o.y, r.inv.y);
            tz = bound_t(cz, sz, 2, r.o.z, r.inv.z);
            cell = (uint32_t(cz) * G.n[1] + uint32_t(cy)) * G.n[0] + uint32_t(cx);
            rayA[lane] = make_float4(r.o.x, r.o.y, r.o.z, r.a);
            rayB[lane] = make_float4(r.d.x, r.d.y, r.d.z, r.ia);
            key[lane] = (static_cast<unsigned long long>(__float_as_uint(r.best)) << 32) | r.bi;
        }
    }
    while (__ballot(walking)) {
        uint32_t b = 0u, n = 0u;
        if (walking) {
            b = cstart[cell];
            n = cstart[cell + 1] - b;
            if (COUNT) { n_cell++; n_sph += n; }
        }
        const uint32_t incl = wave_scan_add(n);
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        const uint32_t start = incl - n;
        const uint32_t off = b - start;   // reference of slot s of this ray: s + off
        uint32_t carry = 0u;              // marker (owner + 1) of the last slot of the previous pass
        for (uint32_t base = 0; base < total; base += 64u) {
            mark[lane] = 0u;
            lane_order();
            if (n != 0u && start - base < 64u) mark[start - base] = lane + 1u;
            lane_order();
            const uint32_t m = max(wave_scan_max(mark[lane]), carry);
            carry = __builtin_amdgcn_readlane(m, 63);
            const uint32_t L = (m - 1u) & 63u;   // the slot's ray
            const uint32_t offL = __shfl(off, int(L));
            const uint32_t s = base + lane;
            UTIL(1, s < total);
            if (s < total) {
                const uint32_t j = s + offL;
                const float4 A = rayA[L], B = rayB[L], sp = rec[j];
                const float rr = sp.w;   // grid record: r^2
                const float ocx = A.x - sp.x, ocy = A.y - sp.y, ocz = A.z - sp.z;
                const float bb = __builtin_fmaf(ocz, B.z, __builtin_fmaf(ocy, B.y, ocx * B.x));
                const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
                const float D = __builtin_fmaf(bb, bb, -(A.w * c));
                if (D >= 0.0f && !behind(bb, c)) {
                    UTIL(2, true);
                    const float sq = sqrt_cr(D);
                    float t = (-bb - sq) * B.w;
                    if (!(t >= T_MIN)) t = (-bb + sq) * B.w;   // report t1 if t1 >= tmin, else t2
                    if (t >= T_MIN) {
                        const unsigned long long k = (static_cast<unsigned long long>(__float_as_uint(t)) << 32) | ids[j];
                        __hip_atomic_fetch_min(&key[L], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    }
                }
            }
            lane_order();
        }
        if (walking) {
            const unsigned long long k = key[lane];
            r.best = __uint_as_float(uint32_t(k >> 32));
            r.bi = uint32_t(k);
            r.limit = cull_limit(P, r.best);
            UTIL(0, true);
            // DDA step (grid_walk): the axis whose boundary comes first, x before y before z on ties
            const float tm = fminf(fminf(tx, ty), tz);
            if (!(tm <= r.limit)) {
                walking = false;   // the next cell starts beyond every closer candidate
            } else {
                walking = dda_step(tm, tx, ty, tz, cx, cy, cz, sx, sy, sz, cell, r.o, r.inv);
            }
        }
    }
}

// The AABB gate of the segment's closest hit, tested once after the walk instead of for every
// candidate that improves the running best (in a divergent tail, each such pass cost the whole
// wave ~30 VALU). Exact: let R be the ungated winner (smallest (t, id) among the quadratic's
// reports the walk tested) and W the gated one (the contract's answer). If R passes the gate, R is
// in the gated set, so W <= R; the walk stops only once the next cell / node starts beyond
// limit(R) >= limit(W) (t_W <= t_R), and W's AABB entry lies before limit(W) (DESIGN.md §4.3
// (iii)), so W was tested and R <= W: R = W. If R fails the gate (a rounding corner: the quadratic
// reports a hit whose ray misses the box; ~1 segment in 7e7 on config 3), the segment's answer is
// recomputed by the contract's rule itself: gated brute force (regate_brute).
// REC: geom4 holds {cx, cy, cz, r} records staged in LDS (rt_trace_grid_kernel<..., REC>), else
// the HBM GeomRec array {cx, cy, cz, r^2} with the radii in P.radius.
template <bool REC>
__device__ __forceinline__ bool winner_gated(const rt::TraceParams& P, const float4* __restrict__ geom4, const Ray& r) {
    if (r.bi == 0xffffffffu) return true;
    const float4 g = geom4[r.bi];
    return aabb_hit(g.x, g.y, g.z, REC ? g.w : P.radius[r.bi], r.o, r.inv);
}

// Gated brute force for the lanes in `need` (wave-uniform), one ray at a time with the whole wave:
// lane k tests spheres k, k + 64, ... in index order (the contract's `t < best` rule keeps the
// lowest index on ties within a lane), then the wave takes the minimum of (t bits, id) — t >= tmin
// > 0, so float bits order like the values and the u64 minimum is the (t, lowest id) rule. 64x
// shorter than one lane walking the whole list (config 5: 99 860 spheres).
template <bool COUNT>
__device__ __forceinline__ void regate_brute(const rt::TraceParams& P, const float4* __restrict__ geom4, uint32_t lane,
                                          unsigned long long need, Ray& r) {
    if (COUNT && lane == 0) atomicAdd(&P.counters->util[30], (unsigned long long)__popcll(need));
    while (need) {
        const int L = __ffsll(need) - 1;
        need &= need - 1ull;
        const V3 o = v3(__shfl(r.o.x, L), __shfl(r.o.y, L), __shfl(r.o.z, L));
        const V3 d = v3(__shfl(r.d.x, L), __shfl(r.d.y, L), __shfl(r.d.z, L));
        const V3 inv = v3(__shfl(r.inv.x, L), __shfl(r.inv.y, L), __shfl(r.inv.z, L));
        const float a = __shfl(r.a, L), ia = __shfl(r.ia, L);
        float best = T_MAX_SUCC;
        uint32_t bi = 0xffffffffu;
        for (uint32_t i = lane; i < P.n_spheres; i += 64u) {
            const float4 s = geom4[i];
            test_sphere(s.x, s.y, s.z, s.w, P.radius, o, d, inv, a, ia, i, best, bi);
        }
        unsigned long long key = (uint64_t(__float_as_uint(best)) << 32) | bi;
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long k2 = __shfl_xor(key, off);
            key = k2 < key ? k2 : key;
        }
        if (int(lane) == L) {
            r.best = __uint_as_float(uint32_t(key >> 32));
            r.bi = uint32_t(key);
        }
    }
}

// The whole walk of one segment. FLAT: the grid is one cell thick in y (grid_walk).
template <bool COUNT, int LAYOUT, bool FLAT = false>
__device__ __forceinline__ void walk(const rt::TraceParams& P, const float4* __restrict__ nodes4,
                                     const float4* __restrict__ leaf4, const uint32_t* __restrict__ leaf_ids,
                                     Ray& r, uint32_t& n_box, uint32_t& n_sph, uint32_t& n_empty) {
    if (LAYOUT == LAYOUT_GRID_CQ) {
        if (r.walk)
            grid_walk_cq<COUNT>(P, reinterpret_cast<const uint32_t*>(nodes4), leaf4, leaf_ids, r, n_box, n_sph, n_empty);
        return;
    }
    if (LAYOUT == LAYOUT_GRID || LAYOUT == LAYOUT_GRID_L2) {   // nodes4 = cell offsets, leaf4 / leaf_ids = references
        if (r.walk)
            grid_walk<COUNT, LAYOUT == LAYOUT_GRID_L2, FLAT>(P, reinterpret_cast<const uint32_t*>(nodes4), leaf4, leaf_ids,
                                                             r, n_box, n_sph, n_empty);
        return;
    }
    const RayBox q = ray_box(r.o, r.inv);
    typedef const __attribute__((address_space(3))) float4* LdsF4;
    if (LAYOUT == LAYOUT_GLOBAL) {
        walk_global_range<COUNT>(P, nodes4, leaf4, leaf_ids, q, r.walk ? 0u : P.n_nodes, P.n_nodes, r, n_box,
                                 n_sph);
    } else if (LAYOUT == LAYOUT_TOP) {
        // Treelet in LDS (top kTreeletDepth levels, AB layout with LDS-address links), the
        // subtrees below the cut and all leaf spheres from L2. A lane leaves the LDS loop at a hit
        // word — a leaf, or a subtree root at the cut — remembering the node's miss link, where it
        // continues afterwards (the escape of a leaf or of a whole subtree). In a balanced
        // 100 k-sphere tree the top 11 levels take ~72 % of the visits (scripts/visit_depths.py).
        const uint32_t nbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)nodes4));
        const float4* gnodes = reinterpret_cast<const float4*>(P.nodes);
        uint32_t ni = r.walk ? nbase : END;
        for (;;) {
            uint32_t cont = END;
            while (int32_t(ni) >= 0) {
                UTIL(0, true);
                const float4 A = lds_f4(ni);
                const float4 B = lds_f4(ni + 16u);
                if (COUNT) n_box++;
                const bool hit = node_hit<1u>(A, B, q, r.limit);
                cont = __float_as_uint(B.z);
                ni = __float_as_uint(hit ? B.w : B.z);
            }
            const bool at = ni != END;
            if (!__ballot(at)) break;
            if (at) {
                UTIL(1, true);
                if (ni & 0x40000000u) {   // subtree of global node g (inner, its box was hit): [g + 1, escape(g))
                    const uint32_t g = ni & 0x3fffffffu;
                    const uint32_t eg = __float_as_uint(gnodes[2 * g].w);
                    walk_global_range<COUNT>(P, gnodes, leaf4, leaf_ids, q, g + 1u, eg == END ? P.n_nodes : eg, r,
                                             n_box, n_sph);
                } else {                  // leaf above the cut
                    const uint32_t fc = ni & 0x3fffffffu;
                    leaf_test<COUNT, false>(P, leaf4, leaf_ids, fc >> 4, fc & 15u, r, n_sph);
                }
                ni = cont;
            }
        }
    } else {
        // AB layout staged in LDS by the kernel: links are LDS addresses of the node, so a visit
        // needs no address arithmetic; B.z = link when the box is missed, B.w = link when it is
        // hit: the next node (inner node) or, bit 31 set, a leaf word (escape node | leaf index |
        // count - 1). END and leaf words are negative, so `continue` is one sign test. A lane
        // leaves the inner loop at a hit leaf holding its leaf word; the leaves are tested
        // together after the loop (while-while).
        const uint32_t nbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)nodes4));   // LDS address of node 0
        constexpr uint32_t kNB = 32u, kBOff = 16u;
        uint32_t ni = r.walk ? nbase + (LAYOUT == LAYOUT_OCT ? octant(r.d) * P.n_nodes * kNB : 0u) : END;
        for (;;) {
            while (int32_t(ni) >= 0) {
                UTIL(0, true);
#ifdef RT_UTIL
                {   // node passes by active lanes: [12] <= 8 lanes, [13] <= 16, [14] <= 32 (+ lanes)
                    const uint32_t na = __popcll(__ballot(true));
                    if (na <= 8) UTIL(12, true);
                    if (na <= 16) UTIL(13, true);
                    if (na <= 32) UTIL(14, true);
                }
#endif
                const float4 A = lds_f4(ni);          // links are LDS addresses:
                const float4 B = lds_f4(ni + kBOff);  // no address arithmetic per visit
                if (COUNT) n_box++;
                const bool hit = node_hit<LAYOUT == LAYOUT_OCT ? 8u : 1u>(A, B, q, r.limit);
                ni = __float_as_uint(hit ? B.w : B.z);
            }
            const bool at_leaf = ni != END;
            if (!__ballot(at_leaf)) break;   // no lane stopped at a leaf: all walks done
            if (at_leaf) {
                UTIL(1, true);
                const uint32_t esc = (ni >> 12) & 0x7ffffu;
                leaf_test<COUNT, true>(P, leaf4, leaf_ids, ((ni >> 2) & 1023u) * 4u, (ni & 3u) + 1u, r, n_sph);
                ni = esc == 0x7ffffu ? END : nbase + esc * kNB;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// LBVH segment loop: one segment per lane per loop iteration; the wave's walk runs until its
// longest walk ends. Stamp slots: 0 loop head, 4 sample start, 5 refill, 6 block fetch, 1 ray
// setup (big spheres), 2 LBVH walk, 3 shading, 7 other.
// ---------------------------------------------------------------------------------------------
template <bool COUNT, int LAYOUT, int MODE, bool REC = false, bool FLAT = false>
__device__ __forceinline__ void lbvh_loop(const rt::TraceParams& P, const float4* __restrict__ nodes4,
                                          const float4* __restrict__ leaf4,
                                          const uint32_t* __restrict__ leaf_ids,
                                          const float4* __restrict__ geom4, const float4* __restrict__ mat4) {
    // the one-layer L2 grid kernel (config 5's) also takes pinhole_lf and at most four big spheres
    // as compile-time facts (flat_grid_form: the host proves both): no camera test and no further
    // big-sphere groups in its segment loop (config 5 -0.5 %; the same for the LDS kernels measured
    // +0.64 % on config 3)
    constexpr bool SPEC = FLAT && LAYOUT == LAYOUT_GRID_L2;
    constexpr bool LSUM = MODE == rt::MODE_HASH &&
                          (LAYOUT == LAYOUT_GRID || LAYOUT == LAYOUT_GRID_L2 || LAYOUT == LAYOUT_GRID_COOP ||
                           LAYOUT == LAYOUT_GRID_CQ);
    const uint32_t lane = lane_id();
    const Camera cam = load_camera(P);
    uint32_t st = ST_NEED_UNIT;
    Path ps{};
    Ray r{};
    if (LSUM) {   // this thread's unit sums (read and written by this thread only: no barrier)
        unsigned long long* s = lane_sum_slot();
        s[0] = s[RT_TRACE_BLOCK] = s[2 * RT_TRACE_BLOCK] = 0ull;
    }
    // traced segments and started samples of this wave (wave-uniform: ballot counts, no per-lane
    // registers); per-lane test counters in COUNT builds only
    uint32_t seg_w = 0, smp_w = 0, n_box = 0, n_sph = 0, n_empty = 0;
    unsigned long long wave_iters = 0;
    bool saw_dry = false;
    WaveBlock blk;
    first_block(P, lane, blk);
    // launch telemetry (3 atomics per wave): first start, work queue dry, last exit
    if (lane == 0) atomicMin(&P.counters->t_first, __builtin_amdgcn_s_memrealtime());
    STAMP_DECL;
    for (;;) {
        STAMP(0);
        refill<MODE, COUNT>(P, lane, st, ps, blk, stamps);
        if (!saw_dry && __ballot(st == ST_RETIRED)) {   // this wave saw the queue run dry
            saw_dry = true;
            if (lane == 0) atomicMin(&P.counters->t_dry, __builtin_amdgcn_s_memrealtime());
        }
        STAMP(4);
        bool started = false;
        if (st == ST_NEED_SAMPLE) {
            if (start_sample<MODE, LSUM, SPEC>(P, cam, ps, r.o, r.d)) {
                st = ST_TRACING;
                started = true;
            } else {   // empty unit (spp = 0): stored at once
                st = ST_NEED_UNIT;
                record_tile_cost<MODE>(P, ps);
            }
        }
        smp_w += __popcll(__ballot(started));
        if (__ballot(st == ST_NEED_UNIT)) continue;   // refill before the next trace
        const unsigned long long tracing = __ballot(st == ST_TRACING);
        if (!tracing) break;                           // every lane retired
        seg_w += __popcll(tracing);
        if (COUNT && lane == 0) atomicAdd(&P.counters->lane_hist[__popcll(tracing)], 1ull);
        STAMP(1);
        UTIL(8, st == ST_TRACING);
        const uint32_t box0 = n_box;
        // Wave priority 1 from the ray setup to the winner's records (the segment's dependent
        // L2 / LDS round trips), 0 in shading and refill: on a SIMD the waves waiting on the walk
        // issue their next load ahead of the ones in shading's long VALU runs. Config 3 -0.5 %,
        // reference stream -4.2 %, config 5 -1.1 % (profiles/r06t_ab_*).
        __builtin_amdgcn_s_setprio(1);
        // every lane (a lane that is not tracing computes on its last ray and discards the result):
        // inside a per-lane branch the big-sphere loop's launch-uniform bound became a spilled lane mask
        setup_ray<SPEC>(P, r);
        if (COUNT && st == ST_TRACING) n_sph += P.n_big;
        // Grid kernels always have a grid to walk: a compile-time fact instead of the launch test
        // (a loop-invariant lane mask the compiler spilled and reloaded every segment). With the
        // two changes beside it (the inert big-sphere records, the regate flag as a scalar select):
        // config 3 -1.2 %, DESIGN.md §5.
        if constexpr (LAYOUT == LAYOUT_GRID || LAYOUT == LAYOUT_GRID_L2 || LAYOUT == LAYOUT_GRID_COOP ||
                      LAYOUT == LAYOUT_GRID_CQ)
            r.walk = true;
        STAMP(2);
        if constexpr (LAYOUT == LAYOUT_GRID_COOP) {   // every lane of the wave takes part (tracing or not)
            grid_walk_coop<COUNT>(P, reinterpret_cast<const uint32_t*>(nodes4), leaf4, leaf_ids, r, st == ST_TRACING,
                                  n_box, n_sph);
        } else {
            if (st == ST_TRACING) walk<COUNT, LAYOUT, FLAT>(P, nodes4, leaf4, leaf_ids, r, n_box, n_sph, n_empty);
        }
        // the AABB gate of the winner only (winner_gated); the rare lanes whose winner fails it
        // get the contract's answer by a wave-cooperative gated brute force. The winner's shading
        // records are loaded with the gate's (one round trip to L2 per segment, not two).
        HitRec hr{};
        float rad = 0.0f;
        if (st == ST_TRACING && r.bi != 0xffffffffu) {
            if constexpr (REC) hr = load_hit_rec(r.bi);
            else hr = load_hit(geom4, mat4, r.bi);
            rad = REC ? hr.g.w : P.radius[r.bi];
        }
        // (the test-only flag replaces the ballot by a scalar select: folded into the per-lane
        // predicate it became a loop-invariant 64-bit lane mask the compiler spilled and reloaded)
        unsigned long long regate = __ballot(
            st == ST_TRACING && r.bi != 0xffffffffu && !aabb_hit(hr.g.x, hr.g.y, hr.g.z, rad, r.o, r.inv));
        if (P.force_regate) regate = __ballot(st == ST_TRACING);
        if (__builtin_expect(regate != 0ull, 0)) {
            regate_brute<COUNT>(P, reinterpret_cast<const float4*>(P.geom), lane, regate, r);
            if (((regate >> lane) & 1ull) && r.bi != 0xffffffffu) {
                if constexpr (REC) hr = load_hit_rec(r.bi);
                else hr = load_hit(geom4, mat4, r.bi);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        if (COUNT && st == ST_TRACING) {   // walk-length histogram (diagnostic, COUNT builds only)
            const uint32_t len = min(n_box - box0, 63u);
            atomicAdd(&P.counters->walk_hist[r.bi != 0xffffffffu ? 1 : 0][len], 1ull);
        }
        if (COUNT) {   // wave iterations of this walk = the longest lane walk
            uint32_t m = n_box - box0;
            for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor(m, off));
            if (lane == 0) wave_iters += m;
        }
        STAMP(3);
        bool fresh = false;   // a sample started inside shade()
        if (st == ST_TRACING) {
            ps.segs++;
            if (!shade_rec<MODE, LSUM, SPEC>(P, cam, hr, ps, r.bi, r.best, r.o, r.d, fresh)) {
                // The unit's last sample ended: finish it here, and the lane asks for a unit at
                // the top of the next iteration.
                finish_unit<MODE, LSUM>(P, ps);
                record_tile_cost<MODE>(P, ps);
                st = ST_NEED_UNIT;
            }
        }
        smp_w += __popcll(__ballot(fresh));
    }
    STAMP_FLUSH;
    if (lane == 0) {
        atomicAdd(&P.counters->segments, (unsigned long long)seg_w);
        atomicAdd(&P.counters->samples, (unsigned long long)smp_w);
        atomicMax(&P.counters->t_last, __builtin_amdgcn_s_memrealtime());
    }
    if (COUNT) {
        atomicAdd(&P.counters->box_tests, (unsigned long long)n_box);
        atomicAdd(&P.counters->sphere_tests, (unsigned long long)n_sph);
        if (n_empty) atomicAdd(&P.counters->cells_empty, (unsigned long long)n_empty);
        if (lane == 0) atomicAdd(&P.counters->wave_iters, wave_iters);
    }
    UTIL_FLUSH;
}

// LBVH kernel, tree in global memory (A/B reference: every node and leaf from L2).
template <bool COUNT, int MODE>
__global__ __launch_bounds__(kTraceBlock, RT_TRACE_WAVES_PER_SIMD) void rt_trace_global_kernel(const rt::TraceParams P) {
    UTIL_INIT;
    PLACEMENT_RECORD(P);
    stage_walk_params(P, threadIdx.x);
    stage_rows(P, threadIdx.x, kTraceBlock);
    __syncthreads();
    lbvh_loop<COUNT, LAYOUT_GLOBAL, MODE>(P, reinterpret_cast<const float4*>(P.nodes),
                                          reinterpret_cast<const float4*>(P.leaf_geom), P.leaf_ids,
                                          reinterpret_cast<const float4*>(P.geom),
                                          reinterpret_cast<const float4*>(P.mat));
}

// LBVH kernel with the whole tree staged in LDS, once per persistent block (one 1024-thread block
// per CU). Staged nodes use the AB layout (node_hit); NOCT = 8 stages one copy per ray direction
// octant, each in its own near-child-first order when the host provides one (nodes_oct). LDS:
// [nodes | leaf spheres | leaf ids]. The geometry + material records read by
// shading stay in HBM: one random record per hit is an L2 hit (staging them in LDS measured the
// same), and the LDS they would take fits bigger trees as octant copies.
template <bool COUNT, uint32_t NOCT, int MODE>
__global__ __launch_bounds__(kTraceBlock, RT_TRACE_WAVES_PER_SIMD) void rt_trace_lds_kernel(const rt::TraceParams P) {
    UTIL_INIT;
    PLACEMENT_RECORD(P);
    extern __shared__ float4 lds[];
    typedef const __attribute__((address_space(3))) float4* LdsF4;
    const uint32_t lbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)lds));   // LDS address of lds[0]
    const uint32_t n_node4 = 2u * NOCT * P.n_nodes, n_leaf4 = P.n_leaf, n_id4 = (P.n_leaf + 3u) / 4u;
    constexpr uint32_t kNodeBytes = 32u;
    const float4* nodes4 = reinterpret_cast<const float4*>(P.nodes);
    for (uint32_t oi = threadIdx.x; oi < NOCT * P.n_nodes; oi += kTraceBlock) {
        const uint32_t o = oi / P.n_nodes, i = oi - o * P.n_nodes;   // copy o, node i
        // BvhNode: lo.xyz escape, hi.xyz leaf.
        const float4* src = (NOCT == 8 && P.nodes_oct)
                                ? reinterpret_cast<const float4*>(P.nodes_oct + size_t(o) * P.n_nodes)
                                : nodes4;
        const float4 lo = src[2 * i], hi = src[2 * i + 1];
        // Links (walk, AB layout): LDS address of the target node in this copy, END = ~0; a hit
        // leaf yields 0x80000000 | escape node << 12 | leaf index << 2 | (count - 1), escape node
        // = 0x7ffff for END. (Trees staged in LDS have < 2^14 nodes and < 1024 leaves of <= 4
        // slots, checked by the host.)
        const uint32_t esc = __float_as_uint(lo.w), fc = __float_as_uint(hi.w);
        const bool nx = NOCT == 8 && (o & 1u), ny = NOCT == 8 && (o & 2u), nz = NOCT == 8 && (o & 4u);
        const uint32_t cb = o * P.n_nodes;   // first node of copy o
        const uint32_t miss = esc == END ? END : lbase + (cb + esc) * kNodeBytes;
        // (kept as separate statements: one combined expression crashed the ROCm 7.2 instruction
        // selector)
        const uint32_t escf = esc == END ? 0x7ffffu : cb + esc;
        const uint32_t leafw = 0x80000000u + (escf << 12) + ((fc >> 6) << 2) + ((fc - 1u) & 3u);
        const uint32_t hit = fc ? leafw : lbase + (cb + i + 1u) * kNodeBytes;
        const size_t b = size_t(cb + i) * 2u, bb = b + 1u;
        lds[b] = make_float4(nx ? hi.x : lo.x, ny ? hi.y : lo.y, nx ? lo.x : hi.x, ny ? lo.y : hi.y);
        lds[bb] = make_float4(nz ? hi.z : lo.z, nz ? lo.z : hi.z, __uint_as_float(miss), __uint_as_float(hit));
    }
    const float4* leaf4 = reinterpret_cast<const float4*>(P.leaf_geom);
    for (uint32_t i = threadIdx.x; i < n_leaf4; i += kTraceBlock) lds[n_node4 + i] = leaf4[i];
    const uint4* ids4 = reinterpret_cast<const uint4*>(P.leaf_ids);
    for (uint32_t i = threadIdx.x; i < n_id4; i += kTraceBlock) {
        const uint4 v = ids4[i];
        lds[n_node4 + n_leaf4 + i] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y),
                                                 __uint_as_float(v.z), __uint_as_float(v.w));
    }
    const float4* geom4 = reinterpret_cast<const float4*>(P.geom);
    const float4* mat4 = reinterpret_cast<const float4*>(P.mat);
    stage_walk_params(P, threadIdx.x);
    stage_rows(P, threadIdx.x, kTraceBlock);
    __syncthreads();
    lbvh_loop<COUNT, NOCT == 8 ? LAYOUT_OCT : LAYOUT_LDS1, MODE>(
        P, lds, lds + n_node4, reinterpret_cast<const uint32_t*>(lds + n_node4 + n_leaf4), geom4, mat4);
}

// Grid kernel (ACCEL_GRID): the grid's cell offsets and references staged in LDS once per
// persistent block: [references (float4) | reference ids | cell offsets] in dynamic LDS, and with
// REC the shading records in the static table s_rec.
// FLAT: the grid is one cell thick in y, as every grid of a scene whose small spheres lie in one
// layer is (configs 3 and 5): the DDA steps x and z only (grid_walk; launch_trace picks it).
template <bool COUNT, int MODE, bool IN_LDS, bool COOP = false, bool REC = false, bool CQ = false, bool FLAT = false>
__global__ __launch_bounds__(kTraceBlock, RT_TRACE_WAVES_PER_SIMD) void rt_trace_grid_kernel(const rt::TraceParams P) {
    UTIL_INIT;
    PLACEMENT_RECORD(P);
    extern __shared__ float4 lds[];
    if (!IN_LDS) {   // grids too big for LDS: offsets and references from L2 / HBM
        stage_walk_params(P, threadIdx.x);
        stage_rows(P, threadIdx.x, kTraceBlock);
        __syncthreads();
        lbvh_loop<COUNT, COOP ? LAYOUT_GRID_COOP : LAYOUT_GRID_L2, MODE, false, FLAT>(P, reinterpret_cast<const float4*>(P.cell_start),
                                            reinterpret_cast<const float4*>(P.grid_rec), P.grid_ids,
                                            reinterpret_cast<const float4*>(P.geom),
                                            reinterpret_cast<const float4*>(P.mat));
        return;
    }
    const uint32_t nr = P.grid.n_refs, nc1 = P.grid.n_cells + 1u;
    const uint32_t n_id4 = (nr + 3u) / 4u;
    const float4* rec = reinterpret_cast<const float4*>(P.grid_rec);
    for (uint32_t i = threadIdx.x; i < nr; i += kTraceBlock) lds[i] = rec[i];
    uint32_t* ids = reinterpret_cast<uint32_t*>(lds + nr);
    for (uint32_t i = threadIdx.x; i < nr; i += kTraceBlock) ids[i] = P.grid_ids[i];
    uint32_t* cst = reinterpret_cast<uint32_t*>(lds + nr + n_id4);
    for (uint32_t i = threadIdx.x; i < nc1; i += kTraceBlock) cst[i] = P.cell_start[i];
    stage_walk_params(P, threadIdx.x);
    stage_rows(P, threadIdx.x, kTraceBlock);
    if (REC) {   // the winner's gate and shading records in LDS too: {cx, cy, cz, r} + 2 x MatRec float4
        const float4* mat4 = reinterpret_cast<const float4*>(P.mat);
        const uint32_t n = min(P.n_spheres, rt::kRecStatic);   // the host picks REC only within the table
        for (uint32_t i = threadIdx.x; i < n; i += kTraceBlock) {
            const rt::GeomRec g = P.geom[i];
            s_rec[3 * i] = make_float4(g.cx, g.cy, g.cz, P.radius[i]);
            s_rec[3 * i + 1] = mat4[2 * i];
            s_rec[3 * i + 2] = mat4[2 * i + 1];
        }
        __syncthreads();
        lbvh_loop<COUNT, CQ ? LAYOUT_GRID_CQ : LAYOUT_GRID, MODE, true, FLAT>(P, reinterpret_cast<const float4*>(cst), lds,
                                                                              ids, s_rec, s_rec);   // (load_hit_rec)
        return;
    }
    __syncthreads();
    lbvh_loop<COUNT, COOP ? LAYOUT_GRID_COOP : CQ ? LAYOUT_GRID_CQ : LAYOUT_GRID, MODE, false, FLAT>(P, reinterpret_cast<const float4*>(cst), lds, ids,
                                        reinterpret_cast<const float4*>(P.geom),
                                        reinterpret_cast<const float4*>(P.mat));
}

// LBVH kernel for trees too big for LDS: the treelet (rt_build.hip build_treelet) is staged in LDS
// with its rank links turned into LDS addresses; leaves, subtrees below the cut, geometry and
// materials stay in HBM/L2.
template <bool COUNT, int MODE>
__global__ __launch_bounds__(kTraceBlock, RT_TRACE_WAVES_PER_SIMD) void rt_trace_top_kernel(const rt::TraceParams P) {
    UTIL_INIT;
    PLACEMENT_RECORD(P);
    extern __shared__ float4 lds[];
    typedef const __attribute__((address_space(3))) float4* LdsF4;
    const uint32_t lbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)lds));
    const uint32_t n_top = min(*P.treelet_count, rt::kTreeletCap);
    for (uint32_t i = threadIdx.x; i < n_top; i += kTraceBlock) {
        const float4* tl = reinterpret_cast<const float4*>(P.treelet);
        const float4 A = tl[2 * i], B = tl[2 * i + 1];
        const uint32_t miss = __float_as_uint(B.z), hit = __float_as_uint(B.w);
        lds[2 * i] = A;
        lds[2 * i + 1] = make_float4(B.x, B.y, __uint_as_float(miss == END ? END : lbase + miss * 32u),
                                     __uint_as_float(int32_t(hit) >= 0 ? lbase + hit * 32u : hit));
    }
    stage_walk_params(P, threadIdx.x);
    stage_rows(P, threadIdx.x, kTraceBlock);
    __syncthreads();
    lbvh_loop<COUNT, LAYOUT_TOP, MODE>(P, lds, reinterpret_cast<const float4*>(P.leaf_geom), P.leaf_ids,
                                       reinterpret_cast<const float4*>(P.geom),
                                       reinterpret_cast<const float4*>(P.mat));
}

// HASH-mode resolve (shader.rgen:53-66 for the chunked frame): per texel, the fixed-point sum of
// this launch's samples plus the incoming float accumulator (accumulate = 1), rounded once to
// float, stored with alpha 1, tonemapped to rgba8; the fixed-point planes are zeroed for the next
// launch. HBM-bound: 24 B read + 24 B zeroed + 20 B stored per texel (+16 B read when accumulating).
// The big-sphere table of a launch (TraceParams::big_tab): records {cx, cy, cz, r} of the n_big
// spheres, padded to a multiple of 4 by repeating the last (a duplicate never changes (best, bi)),
// then their ids. One wave, before the trace kernel on the same stream.
// Per-launch preparation in one kernel instead of five stream operations: block 0
// zeroes the counters, starts the first-time stamps at the maximum (atomicMin), sets the work
// counter past the blocks the waves take by wave id, and fills the big-sphere table; every block
// zeroes its share of the tile-cost table this launch records into.
__global__ __launch_bounds__(256) void rt_launch_prep_kernel(rt::Counters* __restrict__ counters, uint32_t work_head,
                                                             const rt::GeomRec* __restrict__ geom,
                                                             const float* __restrict__ radius,
                                                             const uint32_t* __restrict__ big_ids, uint32_t n_big,
                                                             float4* __restrict__ tab, uint32_t* __restrict__ cost,
                                                             uint32_t n_cost) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n_cost; i += gridDim.x * 256u) cost[i] = 0u;
    if (blockIdx.x != 0) return;
    static_assert(sizeof(rt::Counters) % 8 == 0, "counters are zeroed as u64 words");
    unsigned long long* w = reinterpret_cast<unsigned long long*>(counters);
    for (uint32_t i = threadIdx.x; i < sizeof(rt::Counters) / 8u; i += 256u) w[i] = 0ull;
    const uint32_t nb4 = (n_big + 3u) & ~3u;
    if (threadIdx.x < nb4 && n_big != 0u) {
        const uint32_t id = big_ids[min(threadIdx.x, n_big - 1u)];
        const rt::GeomRec g = geom[id];
        tab[threadIdx.x] = make_float4(g.cx, g.cy, g.cz, radius[id]);
        reinterpret_cast<uint32_t*>(tab + rt::kBigMax)[threadIdx.x] = id;
    }
    if (n_big == 0u && threadIdx.x < 4u) {   // four inert records (setup_ray tests the first four
        // unconditionally): centre (1e19, 1e19, 1e19), radius 0: c = |oc|^2 >= 0 and D <= 0 by
        // Cauchy-Schwarz, and any rounding-made candidate reports t ~ 1e19 > tMax
        tab[threadIdx.x] = make_float4(1e19f, 1e19f, 1e19f, 0.0f);
        reinterpret_cast<uint32_t*>(tab + rt::kBigMax)[threadIdx.x] = 0xffffffffu;
    }
    __syncthreads();   // the words below were zeroed by other threads of the block
    if (threadIdx.x == 0) {
        counters->t_first = ~0ull;
        counters->t_dry = ~0ull;
        counters->work_head = work_head;
    }
}

__global__ __launch_bounds__(256) void rt_resolve_fixed_kernel(unsigned long long* __restrict__ fixed, uint64_t n,
                                                               uint32_t accumulate, float spp,
                                                               float4* __restrict__ accum,
                                                               uint32_t* __restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        const unsigned long long q0 = fixed[i], q1 = fixed[n + i], q2 = fixed[2 * n + i];
        fixed[i] = 0ull;
        fixed[n + i] = 0ull;
        fixed[2 * n + i] = 0ull;
        const float4 a = accumulate ? accum[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float s0 = float(double(a.x) + double(q0) * 0x1p-24);
        const float s1 = float(double(a.y) + double(q1) * 0x1p-24);
        const float s2 = float(double(a.z) + double(q2) * 0x1p-24);
        accum[i] = make_float4(s0, s1, s2, 1.0f);
        out[i] = unorm8(__builtin_sqrtf(s0 / spp)) | (unorm8(__builtin_sqrtf(s1 / spp)) << 8) |
                 (unorm8(__builtin_sqrtf(s2 / spp)) << 16) | (255u << 24);
    }
}

// Band rows -> full image rows (the reorder after the multi-GPU gather).
// Rows mapping at or beyond dst_rows are skipped (the host validates the map; this keeps a bad
// map from writing out of bounds).
__global__ __launch_bounds__(256) void rt_scatter_rows_kernel(const float4* __restrict__ src_acc,
                                                              const uint32_t* __restrict__ src_px,
                                                              const uint32_t* __restrict__ rows,
                                                              uint32_t n_rows, uint32_t width, uint32_t dst_rows,
                                                              float4* __restrict__ dst_acc,
                                                              uint32_t* __restrict__ dst_px) {
    const uint32_t r = blockIdx.y;
    if (r >= n_rows) return;
    const uint32_t dr = rows[r];
    if (dr >= dst_rows) return;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < width; x += gridDim.x * blockDim.x) {
        if (dst_acc) dst_acc[size_t(dr) * width + x] = src_acc[size_t(r) * width + x];
        if (dst_px) dst_px[size_t(dr) * width + x] = src_px[size_t(r) * width + x];
    }
}

// Full image rows -> band rows (the inverse of rt_scatter_rows_kernel): the running sums an
// accumulating multi-GPU frame hands each device before it renders (rt_multi.cpp). Rows mapping at
// or beyond src_rows leave their band row untouched.
__global__ __launch_bounds__(256) void rt_gather_rows_kernel(const float4* __restrict__ src_acc,
                                                             const uint32_t* __restrict__ rows, uint32_t n_rows,
                                                             uint32_t width, uint32_t src_rows,
                                                             float4* __restrict__ dst_acc) {
    const uint32_t r = blockIdx.y;
    if (r >= n_rows) return;
    const uint32_t sr = rows[r];
    if (sr >= src_rows) return;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < width; x += gridDim.x * blockDim.x)
        dst_acc[size_t(r) * width + x] = src_acc[size_t(sr) * width + x];
}

// Tonemap of a summed accumulator, exactly the trace kernel's pixel store (shader.rgen:65-66).
__global__ __launch_bounds__(256) void rt_tonemap_kernel(const float4* __restrict__ acc, uint64_t n, float spp,
                                                         uint32_t* __restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        const float4 s = acc[i];
        out[i] = unorm8(__builtin_sqrtf(s.x / spp)) | (unorm8(__builtin_sqrtf(s.y / spp)) << 8) |
                 (unorm8(__builtin_sqrtf(s.z / spp)) << 16) | (255u << 24);
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
        case 6: r = __uint_as_float(sample_seed_hash(__float_as_uint(x), __float_as_uint(y))); break;
        case 7: r = __uint_as_float(sample_fixed(x)); break;
        case 8: r = 0.0f; break;   // high word of the (32-bit) per-sample value
        case 9: r = checker_positive(x, y, 0.5f * (x - y)) ? 1.0f : 0.0f; break;
        default: r = 0.0f;
    }
    out[i] = r;
}

// Diagnostic: rcp_cr / sqrt_cr against hipcc's correctly rounded 1.0f / x and sqrtf over all 2^32
// inputs (base .. base + grid * 256); mismatches counted in bad[0] / bad[1] (NaN equals NaN). With
// div_b != 0: the camera's float(double(x) * (1 / double(div_b))) against x / div_b for every
// x in [0, 65536) (the camera's numerators), mismatches in bad[2].
__global__ __launch_bounds__(256) void rt_debug_exact_kernel(uint64_t base, float div_b, unsigned long long* bad) {
    const uint32_t bits = uint32_t(base + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    if (div_b != 0.0f) {
        if (bits >= 0x47800000u) return;   // x >= 65536
        const float q0 = float(double(x) * (1.0 / double(div_b))), q1 = x / div_b;
        const unsigned long long mq = __ballot(__float_as_uint(q0) != __float_as_uint(q1));
        if (lane_id() == 0 && mq) atomicAdd(&bad[2], (unsigned long long)__popcll(mq));
        return;
    }
    const float r0 = rcp_cr(x), r1 = 1.0f / x, s0 = sqrt_cr(x), s1 = __builtin_sqrtf(x);
    const bool rb = __float_as_uint(r0) != __float_as_uint(r1) && !(r0 != r0 && r1 != r1);
    const bool sb = __float_as_uint(s0) != __float_as_uint(s1) && !(s0 != s0 && s1 != s1);
    const unsigned long long mr = __ballot(rb), ms = __ballot(sb);
    if (lane_id() == 0 && (mr | ms)) {
        atomicAdd(&bad[0], (unsigned long long)__popcll(mr));
        atomicAdd(&bad[1], (unsigned long long)__popcll(ms));
    }
}

}  // namespace

// ---- host-callable launchers (rt_api.cpp) ---------------------------------------------------
namespace rt {

template <int MODE>
static const void* pick_mode(uint32_t accel, bool count, bool flat) {
#define RT_FN(...) reinterpret_cast<const void*>(__VA_ARGS__)
    if (flat && !count) {   // the grid walks of one-layer grids (instrumented builds count the same cells)
        switch (accel) {
            case ACCEL_GRID: return RT_FN(rt_trace_grid_kernel<false, MODE, true, false, false, false, true>);
            case ACCEL_GRID_REC: return RT_FN(rt_trace_grid_kernel<false, MODE, true, false, true, false, true>);
            case ACCEL_GRID_GLOBAL: return RT_FN(rt_trace_grid_kernel<false, MODE, false, false, false, false, true>);
            default: break;
        }
    }
    switch (accel) {
        case ACCEL_BRUTE:
            return count ? RT_FN(rt_trace_brute_kernel<true, MODE>) : RT_FN(rt_trace_brute_kernel<false, MODE>);
        case ACCEL_LBVH_LDS:
            return count ? RT_FN(rt_trace_lds_kernel<true, 1u, MODE>) : RT_FN(rt_trace_lds_kernel<false, 1u, MODE>);
        case ACCEL_LBVH_OCT:
            return count ? RT_FN(rt_trace_lds_kernel<true, 8u, MODE>) : RT_FN(rt_trace_lds_kernel<false, 8u, MODE>);
        case ACCEL_LBVH_TOP:
            return count ? RT_FN(rt_trace_top_kernel<true, MODE>) : RT_FN(rt_trace_top_kernel<false, MODE>);
        case ACCEL_GRID:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, true>) : RT_FN(rt_trace_grid_kernel<false, MODE, true>);
        case ACCEL_GRID_COOP:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, true, true>)
                         : RT_FN(rt_trace_grid_kernel<false, MODE, true, true>);
        case ACCEL_GRID_REC:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, true, false, true>)
                         : RT_FN(rt_trace_grid_kernel<false, MODE, true, false, true>);
        case ACCEL_GRID_CQ:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, true, false, false, true>)
                         : RT_FN(rt_trace_grid_kernel<false, MODE, true, false, false, true>);
        case ACCEL_GRID_REC_CQ:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, true, false, true, true>)
                         : RT_FN(rt_trace_grid_kernel<false, MODE, true, false, true, true>);
        case ACCEL_GRID_GLOBAL_COOP:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, false, true>)
                         : RT_FN(rt_trace_grid_kernel<false, MODE, false, true>);
        case ACCEL_GRID_GLOBAL:
            return count ? RT_FN(rt_trace_grid_kernel<true, MODE, false>)
                         : RT_FN(rt_trace_grid_kernel<false, MODE, false>);
        default:
            return count ? RT_FN(rt_trace_global_kernel<true, MODE>) : RT_FN(rt_trace_global_kernel<false, MODE>);
    }
#undef RT_FN
}

static const void* pick(uint32_t accel, bool count, int mode, bool flat) {
    return mode == MODE_HASH ? pick_mode<MODE_HASH>(accel, count, flat) : pick_mode<MODE_STREAM>(accel, count, flat);
}

bool flat_grid_form(const TraceParams& P, uint32_t accel, bool count) {
    if (accel == ACCEL_GRID_GLOBAL && !(P.n_big <= 4u && P.pinhole_lf)) return false;   // (lbvh_loop SPEC)
    return !count && P.cell_start != nullptr && P.grid.n[1] == 1u &&
           (accel == ACCEL_GRID || accel == ACCEL_GRID_REC || accel == ACCEL_GRID_GLOBAL);
}

uint32_t block_size(uint32_t accel) { return accel == ACCEL_BRUTE ? kBruteBlock : kTraceBlock; }

hipError_t launch_trace(const TraceParams& P, uint32_t accel, bool count, int mode, int grid, size_t lds_bytes,
                        hipStream_t st) {
    void* args[] = {const_cast<TraceParams*>(&P)};
    return hipLaunchKernel(pick(accel, count, mode, flat_grid_form(P, accel, count)), dim3(grid), dim3(block_size(accel)),
                           args, lds_bytes, st);
}

hipError_t trace_occupancy(uint32_t accel, bool count, int mode, bool flat, size_t lds_bytes, int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, pick(accel, count, mode, flat),
                                                        block_size(accel), lds_bytes);
}

static uint32_t stream_blocks(uint64_t n) {
    const uint64_t need = (n + 255) / 256;
    return uint32_t(need < 8192 ? need : 8192);
}

hipError_t launch_prep(const TraceParams& P, uint32_t work_head, float* tab, uint32_t n_cost, hipStream_t st) {
    const uint32_t blocks = n_cost > 4096u ? min(64u, (n_cost + 4095u) / 4096u) : 1u;
    hipLaunchKernelGGL(rt_launch_prep_kernel, dim3(blocks), dim3(256), 0, st, P.counters, work_head, P.geom, P.radius,
                       P.big_ids, P.n_big, reinterpret_cast<float4*>(tab), P.tile_cost, n_cost);
    return hipGetLastError();
}

hipError_t launch_resolve_fixed(unsigned long long* fixed, uint64_t n_texels, uint32_t accumulate, uint32_t spp,
                                float* accum, uint8_t* out, hipStream_t st) {
    if (n_texels == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_resolve_fixed_kernel, dim3(stream_blocks(n_texels)), dim3(256), 0, st, fixed, n_texels,
                       accumulate, float(spp), reinterpret_cast<float4*>(accum), reinterpret_cast<uint32_t*>(out));
    return hipGetLastError();
}

hipError_t launch_scatter_rows(const float* src_acc, const uint8_t* src_px, const uint32_t* rows,
                               uint32_t n_rows, uint32_t width, uint32_t dst_rows, float* dst_acc, uint8_t* dst_px,
                               hipStream_t st) {
    if (n_rows == 0 || width == 0) return hipSuccess;
    dim3 g((width + 255) / 256, n_rows), b(256);
    hipLaunchKernelGGL(rt_scatter_rows_kernel, g, b, 0, st,
                       reinterpret_cast<const float4*>(src_acc), reinterpret_cast<const uint32_t*>(src_px),
                       rows, n_rows, width, dst_rows, reinterpret_cast<float4*>(dst_acc),
                       reinterpret_cast<uint32_t*>(dst_px));
    return hipGetLastError();
}

hipError_t launch_gather_rows(const float* src_acc, const uint32_t* rows, uint32_t n_rows, uint32_t width,
                              uint32_t src_rows, float* dst_acc, hipStream_t st) {
    if (n_rows == 0 || width == 0) return hipSuccess;
    dim3 g((width + 255) / 256, n_rows), b(256);
    hipLaunchKernelGGL(rt_gather_rows_kernel, g, b, 0, st, reinterpret_cast<const float4*>(src_acc), rows, n_rows,
                       width, src_rows, reinterpret_cast<float4*>(dst_acc));
    return hipGetLastError();
}

hipError_t launch_tonemap(const float* accum, uint64_t n_texels, uint32_t spp, uint8_t* out, hipStream_t st) {
    if (n_texels == 0) return hipSuccess;
    hipLaunchKernelGGL(rt_tonemap_kernel, dim3(stream_blocks(n_texels)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(accum), n_texels, float(spp), reinterpret_cast<uint32_t*>(out));
    return hipGetLastError();
}

hipError_t launch_debug_exact(unsigned long long* bad, hipStream_t st) {
    const uint32_t grid = 1u << 22;   // 2^30 inputs per launch, 4 launches
    for (uint64_t base = 0; base < (1ull << 32); base += uint64_t(grid) * 256u)
        hipLaunchKernelGGL(rt_debug_exact_kernel, dim3(grid), dim3(256), 0, st, base, 0.0f, bad);
    // camera divisors: the BASELINE sizes, small and odd ones, the largest band extent
    const float divs[] = {1920.0f, 1080.0f, 3840.0f, 2160.0f, 64.0f, 36.0f, 1.0f, 3.0f, 7.0f, 1000.0f, 65535.0f};
    for (float b : divs)
        for (uint64_t base = 0; base < 0x47800000ull; base += uint64_t(grid) * 256u)
            hipLaunchKernelGGL(rt_debug_exact_kernel, dim3(grid), dim3(256), 0, st, base, b, bad);
    return hipGetLastError();
}

hipError_t launch_debug_math(int op, const float* in, float* out, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(rt_debug_math_kernel, dim3((n + 255) / 256), dim3(256), 0, st, op, in, out, n);
    return hipGetLastError();
}

}  // namespace rt
