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

enum : uint32_t { ST_NEED_PIXEL = 0, ST_NEED_SAMPLE = 1, ST_TRACING = 2, ST_RETIRED = 3, ST_READY = 4 };

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
#define STAMP_ARG , stamps
#else
#define STAMP(k) do {} while (0)
#define STAMP_DECL [[maybe_unused]] Stamps stamps
#define STAMP_FLUSH do {} while (0)
#define STAMP_ARG , stamps
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

// Four spheres at once (a leaf, or a batch of big spheres): the discriminants of all four are
// computed branch-free, then each lane loops over only ITS candidates (D >= 0). Inside the loop
// sit the expensive exact parts (correctly rounded sqrt and divide, the AABB gate); t2 is
// computed only when t1 < tmin. Identical arithmetic to test_sphere per sphere, and candidates
// are accepted with the same (t, index) rule, so the result is the same; but the wave executes the
// expensive block max-over-lanes-of-candidates times instead of once per slot in which any lane
// has a candidate.
struct Sph4 { float4 s[4]; };

template <typename IdOf>
__device__ __forceinline__ void test4(const float4 s0, const float4 s1, const float4 s2, const float4 s3,
                                      IdOf id_of, V3 o, V3 d, V3 inv, float a, float& best,
                                      uint32_t& bi, float& limit, float cull_abs, float cull_rel) {
    float bv[4], Dv[4];
    const float4 sv[4] = {s0, s1, s2, s3};
    uint32_t cand = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float rr = sv[k].w * sv[k].w;
        const float ocx = o.x - sv[k].x, ocy = o.y - sv[k].y, ocz = o.z - sv[k].z;
        bv[k] = __builtin_fmaf(ocz, d.z, __builtin_fmaf(ocy, d.y, ocx * d.x));
        const float c = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx)) - rr;
        Dv[k] = __builtin_fmaf(bv[k], bv[k], -(a * c));
        cand |= (Dv[k] >= 0.0f ? 1u : 0u) << k;
    }
    while (cand) {
        const uint32_t k = __builtin_ctz(cand);
        cand &= cand - 1u;
        // per-lane select of slot k (no dynamic register indexing)
        const float b = k == 0 ? bv[0] : k == 1 ? bv[1] : k == 2 ? bv[2] : bv[3];
        const float D = k == 0 ? Dv[0] : k == 1 ? Dv[1] : k == 2 ? Dv[2] : Dv[3];
        const float sq = __builtin_sqrtf(D);
        float t = (-b - sq) / a;
        if (!(t >= T_MIN)) t = (-b + sq) / a;     // report t1 if t1 >= tmin, else t2
        if (t >= T_MIN && t <= best) {
            const uint32_t id = id_of(k);
            if (t < best || id < bi) {
                const float4 sp = k == 0 ? s0 : k == 1 ? s1 : k == 2 ? s2 : s3;
                if (aabb_hit(sp.x, sp.y, sp.z, sp.w, o, inv)) {
                    best = t;
                    bi = id;
                    limit = fminf(__builtin_fmaf(t, cull_rel, t + cull_abs), 10000.0f);
                }
            }
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

// ---------------------------------------------------------------------------------------------
// Per-lane path state and the pieces of shader.rgen / rchit / rmiss shared by both loops.
// ---------------------------------------------------------------------------------------------
struct Camera { V3 lf, hor, ver, ulc, cup, crt; };

__device__ __forceinline__ Camera load_camera(const rt::TraceParams& P) {
    return Camera{v3(P.lf[0], P.lf[1], P.lf[2]), v3(P.hor[0], P.hor[1], P.hor[2]),
                  v3(P.ver[0], P.ver[1], P.ver[2]), v3(P.ulc[0], P.ulc[1], P.ulc[2]),
                  v3(P.cup[0], P.cup[1], P.cup[2]), v3(P.crt[0], P.crt[1], P.crt[2])};
}

struct Path {
    uint32_t px;           // lx | ly << 16 (band-local launch id)
    uint32_t pixel_seed;   // TEA(TEA(x, y), number)
    uint32_t seed;         // LCG state (random.glsl)
    uint32_t s;            // samples done for this pixel
    uint32_t depth;        // segments traced in this sample
    uint32_t segs;         // segments traced for this pixel (tile cost for the hand-out order)
    V3 thr;                // reflectedColor (shader.rgen:71)
    double sx, sy, sz;     // dvec3 sum (shader.rgen:55)
};

// Global load of a rarely taken branch, waited for at once. vmcnt counts loads and stores alike
// (gfx9): a load left pending across a branch makes the compiler wait vmcnt(0) at the loop head
// (the register is reused there), which then also waits for the pixel stores still in flight —
// about 10 us per finished pixel. Waiting here, inside the branch, keeps the head
// free of it.
typedef float f4v __attribute__((ext_vector_type(4)));
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

// Pixel refill: lanes in `st == ST_NEED_PIXEL` take the next units of the device work counter
// (one atomic per wave, ranks from the ballot). Units are pixels in 8x8-tile order.
__device__ __forceinline__ void refill(const rt::TraceParams& P, uint32_t lane, uint32_t& st,
                                       Path& ps) {
    const unsigned long long need = __ballot(st == ST_NEED_PIXEL);
    if (!need) return;
    const uint32_t cnt = __popcll(need);
    const int leader = __ffsll(need) - 1;
    uint32_t base = 0;
    if (int(lane) == leader) base = atomicAdd(&P.counters->work_head, cnt);
    base = __shfl(base, leader);
    if (st != ST_NEED_PIXEL) return;
    const uint32_t u = base + __popcll(need & ((1ull << lane) - 1ull));
    if (u >= P.n_units) { st = ST_RETIRED; return; }
    const uint32_t t = P.tile_order ? load_now(P.tile_order + (u >> 6)) : (u >> 6), w = u & 63u;
    const uint32_t lx = (t % P.tiles_x) * 8u + (w & 7u);
    const uint32_t ly = (t / P.tiles_x) * 8u + (w >> 3);
    if (lx >= P.band_w || ly >= P.band_h) return;   // ragged edge: stays NEED_PIXEL, refetches
    // shader.rgen:40
    const uint32_t gx = P.off_x + lx;
    const uint32_t gy = P.rows ? load_now(P.rows + ly) : P.off_y + ly;
    ps.px = lx | (ly << 16);
    ps.pixel_seed = tea(tea(P.seed_local ? lx : gx, P.seed_local ? ly : gy), P.number);
    ps.seed = ps.pixel_seed;
    ps.s = 0;
    ps.segs = 0;
    if (P.accumulate) {  // shader.rgen:53-55
        const float4 acc = load_now4(reinterpret_cast<const float4*>(P.accum) + size_t(ly) * P.band_w + lx);
        ps.sx = acc.x; ps.sy = acc.y; ps.sz = acc.z;
    } else {
        ps.sx = ps.sy = ps.sz = 0.0;
    }
    st = ST_NEED_SAMPLE;
}

// Chunked pixel refill (LBVH kernels). A wave takes whole 8x8 tiles (64 consecutive units, one
// atomic) from the device counter and hands their pixels to its lanes as they free, so a pixel
// costs 1/64 of an atomic round trip and of a hand-out-order load instead of one each; the last
// units (>= n_chunk_units, the last 8 Ki) go out pixel by pixel as in refill(). Per-pixel
// atomics on the one counter were the cost: 1080p at 13 spp took 10.5 ms with them, 4.8 ms
// with tiles (scripts/refill_ab.py). `ch_*` are
// wave-uniform: next unit and end of the wave's current tile, its tile index; `ch_dry` once the
// tile phase is exhausted. `seed` (per lane) is the pixel seed of the tile's pixel `lane`: the
// 64 seeds of a tile are computed together when the tile is taken (two TEAs, 16 rounds each,
// with every lane busy) instead of one lane at a time as its pixel starts.
// `done` once the pixel-by-pixel units are exhausted too: later refills retire lanes without
// touching the counter (one address: every atomic on it queues behind the others).
struct WaveChunk { uint32_t next = 0, end = 0, tile = 0; bool dry = false, done = false; uint32_t seed = 0; };

// shader.rgen:40 seed of pixel w (0..63) of 8x8 tile t of the band.
__device__ __forceinline__ uint32_t tile_pixel_seed(const rt::TraceParams& P, uint32_t t, uint32_t w) {
    const uint32_t lx = (t % P.tiles_x) * 8u + (w & 7u);
    const uint32_t ly = (t / P.tiles_x) * 8u + (w >> 3);
    const uint32_t gx = P.off_x + lx;
    const uint32_t gy = P.rows ? load_now(P.rows + (ly < P.band_h ? ly : P.band_h - 1u)) : P.off_y + ly;   // ragged edge: unused
    return tea(tea(P.seed_local ? lx : gx, P.seed_local ? ly : gy), P.number);
}

__device__ __forceinline__ void refill_chunked(const rt::TraceParams& P, uint32_t lane, uint32_t& st,
                                               Path& ps, WaveChunk& ch, Stamps& stamps) {
    const unsigned long long need = __ballot(st == ST_NEED_PIXEL);
    if (!need) return;
    STAMP(5);
    const uint32_t cnt = __popcll(need);
    const uint32_t rank = __popcll(need & ((1ull << lane) - 1ull));
    const uint32_t avail = ch.end - ch.next;
    const int leader = __ffsll(need) - 1;
    uint32_t u = 0, t = 0;
    bool per_lane = false;
    uint32_t seed = __shfl(ch.seed, int((ch.next + rank) & 63u));   // all lanes: uniform control flow
    if (rank < avail) { u = ch.next + rank; t = ch.tile; }
    if (cnt <= avail) {
        ch.next += cnt;
    } else {
        STAMP(6);
        const uint32_t rest = cnt - avail;   // lanes beyond the current tile's pixels
        uint32_t nb = 0xffffffffu, nt = 0;
        if (!ch.dry) {
            if (int(lane) == leader) {
                nb = atomicAdd(&P.counters->work_head, 64u);
                if (nb < P.n_chunk_units) nt = P.tile_order ? load_now(P.tile_order + (nb >> 6)) : (nb >> 6);
            }
            nb = __shfl(nb, leader);
            nt = __shfl(nt, leader);
            if (nb >= P.n_chunk_units) ch.dry = true;
        }
        if (!ch.dry) {
            ch.seed = tile_pixel_seed(P, nt, lane);
            const uint32_t sn = __shfl(ch.seed, int((rank - avail) & 63u));
            if (rank >= avail) { u = nb + (rank - avail); t = nt; seed = sn; }
            ch.next = nb + rest;
            ch.end = nb + 64u;
            ch.tile = nt;
        } else {
            uint32_t tb = P.n_units;   // exhausted: the lanes retire
            if (!ch.done) {
                if (int(lane) == leader) tb = atomicAdd(&P.counters->work_tail, rest);
                tb = P.n_chunk_units + __shfl(tb, leader);
                if (tb + rest >= P.n_units) ch.done = true;
            }
            if (rank >= avail) { u = tb + (rank - avail); per_lane = true; }
            ch.next = ch.end;
        }
    }
    if (st != ST_NEED_PIXEL) return;
    if (per_lane) {
        if (u >= P.n_units) { st = ST_RETIRED; return; }
        t = P.tile_order ? load_now(P.tile_order + (u >> 6)) : (u >> 6);
    }
    const uint32_t w = u & 63u;
    const uint32_t lx = (t % P.tiles_x) * 8u + (w & 7u);
    const uint32_t ly = (t / P.tiles_x) * 8u + (w >> 3);
    if (lx >= P.band_w || ly >= P.band_h) return;   // ragged edge: stays NEED_PIXEL, refetches
    if (per_lane) seed = tile_pixel_seed(P, t, w);
    ps.px = lx | (ly << 16);
    ps.pixel_seed = seed;
    ps.seed = ps.pixel_seed;
    ps.s = 0;
    ps.segs = 0;
    if (P.accumulate) {  // shader.rgen:53-55
        const float4 acc = load_now4(reinterpret_cast<const float4*>(P.accum) + size_t(ly) * P.band_w + lx);
        ps.sx = acc.x; ps.sy = acc.y; ps.sz = acc.z;
    } else {
        ps.sx = ps.sy = ps.sz = 0.0;
    }
    st = ST_NEED_SAMPLE;
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

// shader.rgen:56-58 + 107-115: next camera ray of the lane's pixel. Returns false (and stores
// the pixel, shader.rgen:61-66) when the pixel's samples are done.
__device__ __forceinline__ bool start_sample(const rt::TraceParams& P, const Camera& cam, Path& ps,
                                             V3& o, V3& d) {
    const uint32_t lx = ps.px & 0xffffu, ly = ps.px >> 16;
    if (ps.s >= P.spp) {
        store_pixel(P, ps);
        return false;
    }
    const uint32_t gx = P.off_x + lx;
    const uint32_t gy = P.rows ? load_now(P.rows + ly) : P.off_y + ly;
    if (P.rng_counter) ps.seed = tea(ps.pixel_seed, P.sample_base + ps.s);
    float ux = float(gx) + rnd(ps.seed);
    float uy = float(gy) + rnd(ps.seed);
    ux = ux / P.size_x;
    uy = uy / P.size_y;
    const float lxr = rnd_pm1(ps.seed);
    const float lyr = rnd_pm1(ps.seed);
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
    const V3 from = add(cam.lf, add(scale(rx, cam.crt), scale(ry, cam.cup)));
    const V3 to = sub(add(cam.ulc, scale(ux, cam.hor)), scale(uy, cam.ver));
    o = from;
    d = normalize(sub(to, from));
    ps.thr = v3(1.0f, 1.0f, 1.0f);
    ps.depth = 0;
    return true;
}

// shader.rchit:38-133 / shader.rmiss:13-18 + shader.rgen:77-88 for one finished trace.
// Returns true when the path continues (o, d hold the next ray), false when the sample ended
// (its colour has been added to the pixel sum).
__device__ __forceinline__ bool shade(const rt::TraceParams& P, const float4* __restrict__ geom4,
                                      const float4* __restrict__ mat4, Path& ps, uint32_t bi,
                                      float best, V3& o, V3& d) {
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
        const float4 gc4 = geom4[bi];
        const rt::GeomRec gc{gc4.x, gc4.y, gc4.z, gc4.w};
        const float4 m0 = mat4[2 * bi];
        const float4 m1 = mat4[2 * bi + 1];
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
        // diffuse and metal both draw one random unit vector first (shader.rchit:69, :80): one
        // copy of that code serves a wave holding both materials
        V3 ru = v3(0.0f, 0.0f, 0.0f);
        if (mtype < 2u) ru = random_unit_vector(ps.seed);
        if (mtype == 0u) {                       // diffuse, shader.rchit:68-76
            sd = add(n, ru);
            if (fabsf(sd.x) < 1e-8f && fabsf(sd.y) < 1e-8f && fabsf(sd.z) < 1e-8f) sd = n;
        } else if (mtype == 1u) {                // metal, shader.rchit:78-89
            const V3 refl = reflect(d, n);
            const V3 fuzz = scale(m0.w, ru);
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
                refracts = refl < rnd(ps.seed);
            }
            sd = refracts ? refract(d, n, eta) : reflect(d, n);
        }
        scatter = !(sd.x == 0.0f && sd.y == 0.0f && sd.z == 0.0f);  // shader.rchit:48
    }
    // shader.rgen:77-88
    V3 col;
    if (scatter) {
        ps.thr = mul(ps.thr, att);
        o = p;
        d = normalize(sd);
        ps.depth++;
        if (ps.depth < P.max_depth) return true;
        col = mul(ps.thr, v3(0.0f, 0.0f, 0.0f));   // depth exhausted: light stays 0 (Q6)
    } else {
        col = mul(ps.thr, att);
    }
    ps.sx += double(col.x);
    ps.sy += double(col.y);
    ps.sz += double(col.z);
    ps.s++;
    return false;
}

// ---------------------------------------------------------------------------------------------
// LBVH traversal state and the one-node step.
// ---------------------------------------------------------------------------------------------
struct Ray {
    V3 o, d, inv;          // origin, direction, 1/d (the AABB gate's own reciprocals)
    float a;               // dot(d, d)
    float limit;           // node cull limit: min(best + cull_abs + cull_rel * best, tmax)
    float best;
    uint32_t bi, ni;       // closest so far, next node (END = done)
};
constexpr uint32_t END = 0xffffffffu;
constexpr uint32_t kLeafFlagD = 0x80000000u;

// Node slab test: one fma per plane, t = fma(plane, inv, -o * inv) (a sub-then-mul form is exact
// in the gate's own arithmetic but costs twice the issue cycles: packed f32 ops take 4 cycles on
// gfx950). Node boxes are padded at build time by 12u x (scene + camera radius),
// which covers the rounding of this form against the spheres' AABB gates.
// A zero (or denormal) direction component makes 1/d infinite; the fma form would then produce
// inf - inf = NaN for a plane on the far side of the origin and cull a box the ray runs inside, so
// the node reciprocal is clamped to +-2^100: the slab then spans (-huge, +huge) exactly when the
// origin lies inside the padded slab, which is what the gate's (plane - o) * inf gives.
// Node layout "AB" (LDS): A = (x0, y0, x1, y1), B = (z0, z1, escape, leaf). OCT: the node copy
// is specialised to the ray's direction octant, (x0, y0, z0) are the near planes and (x1, y1,
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

// New segment: hoisted per-ray terms, the exhaustive big spheres, walk from the root.
__device__ __forceinline__ void setup_ray(const rt::TraceParams& P, Ray& r, uint32_t& n_sph) {
    r.a = dot(r.d, r.d);
    r.inv = v3(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    r.best = T_MAX_SUCC;
    r.bi = 0xffffffffu;
    typedef const __attribute__((address_space(4))) uint32_t* ConstU;
    typedef const __attribute__((address_space(4))) float* ConstF;
    const ConstU ids = (ConstU)(P.big_ids);
    const ConstF g = (ConstF)(P.geom);
    const ConstF rad = (ConstF)(P.radius);
    for (uint32_t k0 = 0; k0 < P.n_big; k0 += 4) {   // wave-uniform: scalar loads, 4 at a time
        uint32_t id[4];
        float sp[16], rs[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) id[j] = ids[min(k0 + j, P.n_big - 1)];
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) sp[j] = g[4 * id[j >> 2] + (j & 3)];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) rs[j] = rad[id[j]];
        // records of absent batch members (k0 + j >= n_big) repeat the last big sphere: a
        // duplicate of an already tested sphere can never change (best, bi).
        const float4 b0 = make_float4(sp[0], sp[1], sp[2], rs[0]), b1 = make_float4(sp[4], sp[5], sp[6], rs[1]);
        const float4 b2 = make_float4(sp[8], sp[9], sp[10], rs[2]), b3 = make_float4(sp[12], sp[13], sp[14], rs[3]);
        float unused_limit = 0.0f;
        test4(b0, b1, b2, b3, [&](uint32_t k) { return k == 0 ? id[0] : k == 1 ? id[1] : k == 2 ? id[2] : id[3]; },
              r.o, r.d, r.inv, r.a, r.best, r.bi, unused_limit, 0.0f, 0.0f);
    }
    n_sph += P.n_big;
    r.limit = fminf(__builtin_fmaf(r.best, P.cull_rel, r.best + P.cull_abs), 10000.0f);
    r.ni = P.nodes ? 0u : END;
}

// One node of the stackless escape-link walk. Node test: slab test over
// [T_MIN, min(T_MAX, best + cull)] with one fma per plane, widened by the fma form's rounding
// allowance; cull = cull_abs + cull_rel * best bounds how far a candidate's AABB entry can lie
// beyond its reported t, so no node holding a possible winner is skipped and
// the result equals brute force bit for bit.
template <bool COUNT>
__device__ __forceinline__ void visit_node(const rt::TraceParams& P, const float4* __restrict__ nodes4,
                                           const float4* __restrict__ leaf4,
                                           const uint32_t* __restrict__ leaf_ids, Ray& r,
                                           uint32_t& n_box, uint32_t& n_sph) {
    const float4 n0 = nodes4[2 * r.ni];
    const float4 n1 = nodes4[2 * r.ni + 1];
    if (COUNT) n_box++;
    const bool hit = node_hit<1>(make_float4(n0.x, n0.y, n1.x, n1.y), make_float4(n0.z, n1.z, 0.0f, 0.0f),
                                     ray_box(r.o, r.inv), r.limit);
    const uint32_t fc = __float_as_uint(n1.w);
    if (hit && fc != 0u) {   // leaf: always 4 slots (dummy-padded), loads issued together
        const uint32_t first = fc >> 4;
        const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
        test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a,
              r.best, r.bi, r.limit, P.cull_abs, P.cull_rel);
        if (COUNT) n_sph += fc & 15u;
    }
    r.ni = (hit && fc == 0u) ? r.ni + 1u : __float_as_uint(n0.w);
}

// ---------------------------------------------------------------------------------------------
// Ordered LBVH walk (two-wide nodes, per-lane stack in LDS): each visit tests both children's
// boxes with the same conservative slab test as visit_node, processes hit leaf children at once
// (4-slot block), descends into the nearer hit inner child and pushes the farther one. Nearest-
// first order finds the closest sphere early, so `best` culls the rest of the walk.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void leaf_block(const rt::TraceParams& P, uint32_t ref,
                                           const float4* __restrict__ leaf4,
                                           const uint32_t* __restrict__ leaf_ids, Ray& r) {
    const uint32_t first = (ref & ~kLeafFlagD) >> 3;
    const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
    test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a, r.best,
          r.bi, r.limit, P.cull_abs, P.cull_rel);
}

__device__ __forceinline__ float slab_near(float4 lo, float4 hi, const Ray& r, float& tfar_out) {
    const RayBox q = ray_box(r.o, r.inv);   // (hoisted by the compiler: loop-invariant)
    const float tx0 = __builtin_fmaf(lo.x, q.inv.x, -q.oi.x), tx1 = __builtin_fmaf(hi.x, q.inv.x, -q.oi.x);
    const float ty0 = __builtin_fmaf(lo.y, q.inv.y, -q.oi.y), ty1 = __builtin_fmaf(hi.y, q.inv.y, -q.oi.y);
    const float tz0 = __builtin_fmaf(lo.z, q.inv.z, -q.oi.z), tz1 = __builtin_fmaf(hi.z, q.inv.z, -q.oi.z);
    tfar_out = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return fmaxf(fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1)), T_MIN);
}

template <bool COUNT>
__device__ __forceinline__ void walk_ordered(const rt::TraceParams& P, const float4* __restrict__ nodes4,
                                             const float4* __restrict__ leaf4,
                                             const uint32_t* __restrict__ leaf_ids,
                                             uint32_t* __restrict__ stk, uint32_t stride, Ray& r,
                                             uint32_t& n_box, uint32_t& n_sph) {
    if (P.n_leaf == 0) return;   // no small spheres: nothing to walk
    uint32_t cur = P.root2;
    if (cur & kLeafFlagD) {   // the whole tree is one leaf
        leaf_block(P, cur, leaf4, leaf_ids, r);
        if (COUNT) n_sph += cur & 7u;
        return;
    }
    uint32_t sp = 0;
    for (;;) {
        const float4 a0 = nodes4[4 * cur], a1 = nodes4[4 * cur + 1];
        const float4 b0 = nodes4[4 * cur + 2], b1 = nodes4[4 * cur + 3];
        if (COUNT) n_box += 2;
        float tf0, tf1;
        const float tn0 = slab_near(a0, a1, r, tf0);
        const float tn1 = slab_near(b0, b1, r, tf1);
        bool hit0 = tn0 <= fminf(tf0, r.limit);   // padded boxes: no tolerance term (visit_node)
        bool hit1 = tn1 <= fminf(tf1, r.limit);
        const uint32_t c0 = __float_as_uint(a0.w), c1 = __float_as_uint(b0.w);
        // hit leaf children: test their spheres now
        uint32_t lp0 = (hit0 && (c0 & kLeafFlagD)) ? c0 : 0u;
        uint32_t lp1 = (hit1 && (c1 & kLeafFlagD)) ? c1 : 0u;
        hit0 = hit0 && !(c0 & kLeafFlagD);
        hit1 = hit1 && !(c1 & kLeafFlagD);
        if (lp0 == 0u) { lp0 = lp1; lp1 = 0u; }
        while (lp0) {
            leaf_block(P, lp0, leaf4, leaf_ids, r);
            if (COUNT) n_sph += lp0 & 7u;
            lp0 = lp1;
            lp1 = 0u;
        }
        if (hit0 && hit1) {
            const bool first0 = tn0 <= tn1;
            stk[sp * stride] = first0 ? c1 : c0;
            ++sp;
            cur = first0 ? c0 : c1;
        } else if (hit0 || hit1) {
            cur = hit0 ? c0 : c1;
        } else {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * stride];
        }
    }
}

// The whole escape-link walk of one segment. LAYOUT: 0 = BvhNode pairs (global memory), 1 = AB
// layout (LDS), 2 = AB layout with one node copy per ray direction octant.
template <bool COUNT, int LAYOUT>
__device__ __forceinline__ void walk_escape(const rt::TraceParams& P, const float4* __restrict__ nodes4,
                                            const float4* __restrict__ leaf4,
                                            const uint32_t* __restrict__ leaf_ids, Ray& r,
                                            uint32_t& n_box, uint32_t& n_sph) {
    const RayBox q = ray_box(r.o, r.inv);
#ifdef RT_LEAF_INLINE
    while (r.ni != END) visit_node<COUNT>(P, nodes4, leaf4, leaf_ids, r, n_box, n_sph);
#else
    // while-while (Aila & Laine 2009): the cheap inner-node loop runs until every active lane has
    // found a hit leaf (postponed in `pending`) or finished its walk; then all pending leaves are
    // tested together, so the 4-sphere leaf block runs once per batch instead of in every visit
    // in which any lane of the wave happens to be at a leaf.
    if (LAYOUT == 3) {
        // Treelet in LDS (top kTreeletDepth levels, AB layout with LDS-address links), the
        // subtrees below the cut and all leaf spheres from L2 (ACCEL_LBVH_TOP). A lane leaves
        // the LDS loop at a hit word — a leaf, or a subtree root at the cut — remembering the
        // node's miss link, where it continues afterwards (the escape of a leaf or of a whole
        // subtree). In a balanced 100 k-sphere tree the top 11 levels take ~72 % of the visits
        // (scripts/visit_depths.py).
        typedef const __attribute__((address_space(3))) float4* LdsF4;
        const uint32_t nbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)nodes4));
        const float4* gnodes = reinterpret_cast<const float4*>(P.nodes);
        uint32_t ni = r.ni == END ? END : nbase;
        for (;;) {
            uint32_t cont = END;
            while (int32_t(ni) >= 0) {
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
                uint32_t pending = 0u;
                if (ni & 0x40000000u) {   // subtree of global node g (inner, its box was hit): [g + 1, escape(g))
                    const uint32_t g = ni & 0x3fffffffu;
                    const uint32_t eg = __float_as_uint(gnodes[2 * g].w);
                    const uint32_t bound = eg == END ? P.n_nodes : eg;
                    uint32_t gi = g + 1u;
                    for (;;) {
                        while (gi < bound && pending == 0u) {
                            const float4 n0 = gnodes[2 * gi];
                            const float4 n1 = gnodes[2 * gi + 1];
                            if (COUNT) n_box++;
                            const bool h = node_hit<1>(make_float4(n0.x, n0.y, n1.x, n1.y),
                                                       make_float4(n0.z, n1.z, 0.0f, 0.0f), q, r.limit);
                            const uint32_t fc = __float_as_uint(n1.w);
                            if (h && fc != 0u) pending = fc;
                            gi = (h && fc == 0u) ? gi + 1u : __float_as_uint(n0.w);
                        }
                        if (pending == 0u) break;
                        const uint32_t first = pending >> 4;
                        const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
                        test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a,
                              r.best, r.bi, r.limit, P.cull_abs, P.cull_rel);
                        if (COUNT) n_sph += pending & 15u;
                        pending = 0u;
                    }
                } else {                  // leaf above the cut
                    pending = ni & 0x3fffffffu;
                    const uint32_t first = pending >> 4;
                    const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
                    test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a,
                          r.best, r.bi, r.limit, P.cull_abs, P.cull_rel);
                    if (COUNT) n_sph += pending & 15u;
                }
                ni = cont;
            }
        }
        r.ni = END;
    } else if (LAYOUT == 0) {   // BvhNode pairs: escape in lo.w, leaf field (first << 4 | count, 0 = inner) in hi.w
        uint32_t pending = 0u;
        for (;;) {
            while (r.ni != END && pending == 0u) {
                const float4 n0 = nodes4[2 * r.ni];
                const float4 n1 = nodes4[2 * r.ni + 1];
                if (COUNT) n_box++;
                const bool hit = node_hit<1>(make_float4(n0.x, n0.y, n1.x, n1.y),
                                                 make_float4(n0.z, n1.z, 0.0f, 0.0f), q, r.limit);
                const uint32_t fc = __float_as_uint(n1.w);
                if (hit && fc != 0u) pending = fc;
                r.ni = (hit && fc == 0u) ? r.ni + 1u : __float_as_uint(n0.w);
            }
            if (pending == 0u) break;   // walk finished with no leaf left to test
            const uint32_t first = pending >> 4;
            const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
            test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a,
                  r.best, r.bi, r.limit, P.cull_abs, P.cull_rel);
            if (COUNT) n_sph += pending & 15u;
            pending = 0u;
        }
    } else {
        // AB layout (staged in LDS by the kernel, see rt_trace_lbvh_kernel): links are LDS
        // addresses of the node, so a visit needs no address arithmetic;
        // B.z = link when the box is missed, B.w = link when it is hit: the next node (inner
        // node) or, bit 31 set, a leaf word (escape node | leaf index | count - 1). END and leaf
        // words are negative, so `continue` is one sign test. A lane leaves the inner loop at a
        // hit leaf holding its leaf word; the leaves are tested together after the loop.
        typedef const __attribute__((address_space(3))) float4* LdsF4;
        const uint32_t nbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)nodes4));   // LDS address of node 0
        uint32_t ni = r.ni == END ? END : nbase + (LAYOUT == 2 ? octant(r.d) * P.n_nodes * 32u : 0u);
        for (;;) {
            while (int32_t(ni) >= 0) {
                const float4 A = lds_f4(ni);         // links are LDS addresses:
                const float4 B = lds_f4(ni + 16u);   // no address arithmetic per visit
                if (COUNT) n_box++;
                const bool hit = node_hit<LAYOUT == 2 ? 8u : 1u>(A, B, q, r.limit);
                ni = __float_as_uint(hit ? B.w : B.z);
            }
            const bool at_leaf = ni != END;
            if (!__ballot(at_leaf)) break;   // no lane stopped at a leaf: all walks done
            if (at_leaf) {
                const uint32_t first = ((ni >> 2) & 1023u) * 4u, esc = (ni >> 12) & 0x7ffffu;
                const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
                test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a,
                      r.best, r.bi, r.limit, P.cull_abs, P.cull_rel);
                if (COUNT) n_sph += (ni & 3u) + 1u;
                ni = esc == 0x7ffffu ? END : nbase + esc * 32u;
            }
        }
        r.ni = END;
    }
#endif
}

// Escape-link walk over compact 16-B nodes (BvhNode16): one ds_read_b128 per visit; the binary16
// bounds are widened exactly to f32 (v_fma_mix_f32) and enter the one-fma slab test.
__device__ __forceinline__ float h_lo(uint32_t v) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(v & 0xffffu));
}
__device__ __forceinline__ float h_hi(uint32_t v) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(v >> 16));
}

template <bool COUNT>
__device__ __forceinline__ void walk_escape16(const rt::TraceParams& P, const uint4* __restrict__ nodes,
                                              const float4* __restrict__ leaf4,
                                              const uint32_t* __restrict__ leaf_ids, Ray& r,
                                              uint32_t& n_box, uint32_t& n_sph) {
    uint32_t ni = (P.n_nodes != 0u) ? 0u : 0xffffu;
    const RayBox q = ray_box(r.o, r.inv);
    while (ni != 0xffffu) {
        const uint4 n = nodes[ni];
        if (COUNT) n_box++;
        const float tx0 = __builtin_fmaf(h_lo(n.x), q.inv.x, -q.oi.x), tx1 = __builtin_fmaf(h_hi(n.y), q.inv.x, -q.oi.x);
        const float ty0 = __builtin_fmaf(h_hi(n.x), q.inv.y, -q.oi.y), ty1 = __builtin_fmaf(h_lo(n.z), q.inv.y, -q.oi.y);
        const float tz0 = __builtin_fmaf(h_lo(n.y), q.inv.z, -q.oi.z), tz1 = __builtin_fmaf(h_hi(n.z), q.inv.z, -q.oi.z);
        const float tnear = fmaxf(fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1)), T_MIN);
        const float tfar = fminf(fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1)), r.limit);
        const bool hit = tnear <= tfar;
        const uint32_t leaf = n.w >> 16;
        if (hit && leaf != 0u) {
            const uint32_t first = (leaf & 0x7fffu) & ~3u;   // (index << 2) = first slot
            const float4 s0 = leaf4[first], s1 = leaf4[first + 1], s2 = leaf4[first + 2], s3 = leaf4[first + 3];
            test4(s0, s1, s2, s3, [&](uint32_t k) { return leaf_ids[first + k]; }, r.o, r.d, r.inv, r.a,
                  r.best, r.bi, r.limit, P.cull_abs, P.cull_rel);
            if (COUNT) n_sph += (leaf & 3u) + 1u;
        }
        ni = (hit && leaf == 0u) ? ni + 1u : (n.w & 0xffffu);
    }
}

// Waves per SIMD the register budget is sized for. Brute force: 6 (71 VGPRs, no spills). LBVH:
// 4 (128 VGPRs): at 6 the 80-VGPR budget spilled ~34 VGPRs of path state around every walk, and
// 4 waves of the unspilled kernel measured 8 % faster.
#ifndef RT_BRUTE_WAVES_PER_SIMD
#define RT_BRUTE_WAVES_PER_SIMD 6
#endif
#ifndef RT_TRACE_WAVES_PER_SIMD
#define RT_TRACE_WAVES_PER_SIMD 4
#endif

// ---------------------------------------------------------------------------------------------
// Brute-force kernel: one segment per loop iteration for every lane (the sphere loop is
// wave-uniform, so there is no traversal divergence to manage).
// ---------------------------------------------------------------------------------------------
template <bool COUNT>
__global__ __launch_bounds__(256, RT_BRUTE_WAVES_PER_SIMD) void rt_trace_brute_kernel(const rt::TraceParams P) {
    const uint32_t lane = lane_id();
    const Camera cam = load_camera(P);
    uint32_t st = ST_NEED_PIXEL;
    Path ps{};
    V3 o = v3(0, 0, 0), d = v3(0, 0, 1);
    uint32_t n_seg = 0, n_smp = 0, n_sph = 0;
    for (;;) {
        refill(P, lane, st, ps);
        if (st == ST_NEED_SAMPLE) {
            if (start_sample(P, cam, ps, o, d)) { st = ST_TRACING; n_smp++; }
            else st = ST_NEED_PIXEL;
        }
        if (__ballot(st == ST_NEED_PIXEL)) continue;   // refill before the next trace
        if (!__ballot(st == ST_TRACING)) break;         // every lane retired
        if (st == ST_TRACING) {
            float best = T_MAX_SUCC;
            uint32_t bi = 0xffffffffu;
            const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
            closest_brute(P, o, d, inv, dot(d, d), best, bi);
            if (COUNT) n_sph += P.n_spheres;
            n_seg++;
            if (!shade(P, reinterpret_cast<const float4*>(P.geom), reinterpret_cast<const float4*>(P.mat),
                       ps, bi, best, o, d))
                st = ST_NEED_SAMPLE;
        }
    }
    atomicAdd(&P.counters->segments, (unsigned long long)n_seg);
    atomicAdd(&P.counters->samples, (unsigned long long)n_smp);
    if (COUNT) atomicAdd(&P.counters->sphere_tests, (unsigned long long)n_sph);
}

// ---------------------------------------------------------------------------------------------
// Tail compaction pool (block-local, LDS). Once the device pixel queue has run dry, lanes whose
// pixel ends stay empty, and a wave keeps paying full issue cost for a shrinking set of paths
// (the per-pixel sample stream is sequential, so the last pixels cannot be split). Waves that
// fall below RT_POOL_T active lanes donate their in-flight paths (pixel state + next ray) to a
// block-wide LDS pool and go idle; waves with empty lanes refill from it. The block's paths thus
// concentrate in few, full waves, and idle waves sleep (s_sleep) instead of issuing.
//
// Protocol (one LDS spin lock, taken by one lane per wave):
//   count   paths in the pool (LIFO stack of `cap` slots, SoA: field f of slot i at f*cap+i);
//           read and written only under the lock
//   working waves holding at least one path; changed ONLY by atomics (a wave whose last path
//           ends decrements it without the lock), increments happen under the lock
// A wave donates only while another wave is working (so someone drains the pool); an idle wave
// takes paths when at least RT_POOL_T are waiting or no wave is working; it exits when, under
// the lock, working == 0 and count == 0: no path exists any more, and none can appear.
// Capacity: every path is in exactly one lane or slot, so count <= paths in block <= cap.
// ---------------------------------------------------------------------------------------------
#ifndef RT_POOL_T
#define RT_POOL_T 32
#endif
constexpr uint32_t kPoolFields = 22;   // st, px, pixel_seed, seed, s, depth, segs, thr3, o3, d3, 3 x f64

struct PoolCtl { uint32_t lock, count, working, pad; };

__device__ __forceinline__ void pool_lock(PoolCtl* c) {
    while (atomicCAS(&c->lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
    __threadfence_block();
}
__device__ __forceinline__ void pool_unlock(PoolCtl* c) {
    __threadfence_block();
    atomicExch(&c->lock, 0u);
}
__device__ __forceinline__ uint32_t pool_peek(const PoolCtl* c, uint32_t f) {   // lock-free hint
    return __hip_atomic_load(reinterpret_cast<const uint32_t*>(c) + f, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void pool_put(uint32_t* pool, uint32_t cap, uint32_t i, uint32_t st,
                                         const Path& ps, const Ray& r) {
    const uint32_t v[kPoolFields] = {
        st, ps.px, ps.pixel_seed, ps.seed, ps.s, ps.depth, ps.segs,
        __float_as_uint(ps.thr.x), __float_as_uint(ps.thr.y), __float_as_uint(ps.thr.z),
        __float_as_uint(r.o.x), __float_as_uint(r.o.y), __float_as_uint(r.o.z),
        __float_as_uint(r.d.x), __float_as_uint(r.d.y), __float_as_uint(r.d.z),
        uint32_t(__double_as_longlong(ps.sx)), uint32_t(__double_as_longlong(ps.sx) >> 32),
        uint32_t(__double_as_longlong(ps.sy)), uint32_t(__double_as_longlong(ps.sy) >> 32),
        uint32_t(__double_as_longlong(ps.sz)), uint32_t(__double_as_longlong(ps.sz) >> 32)};
#pragma unroll
    for (uint32_t f = 0; f < kPoolFields; ++f) pool[f * cap + i] = v[f];
}

__device__ __forceinline__ void pool_get(const uint32_t* pool, uint32_t cap, uint32_t i, uint32_t& st,
                                         Path& ps, Ray& r) {
    uint32_t v[kPoolFields];
#pragma unroll
    for (uint32_t f = 0; f < kPoolFields; ++f) v[f] = pool[f * cap + i];
    st = v[0]; ps.px = v[1]; ps.pixel_seed = v[2]; ps.seed = v[3]; ps.s = v[4]; ps.depth = v[5]; ps.segs = v[6];
    ps.thr = v3(__uint_as_float(v[7]), __uint_as_float(v[8]), __uint_as_float(v[9]));
    r.o = v3(__uint_as_float(v[10]), __uint_as_float(v[11]), __uint_as_float(v[12]));
    r.d = v3(__uint_as_float(v[13]), __uint_as_float(v[14]), __uint_as_float(v[15]));
    ps.sx = __longlong_as_double((long long)(uint64_t(v[16]) | uint64_t(v[17]) << 32));
    ps.sy = __longlong_as_double((long long)(uint64_t(v[18]) | uint64_t(v[19]) << 32));
    ps.sz = __longlong_as_double((long long)(uint64_t(v[20]) | uint64_t(v[21]) << 32));
}

// Take up to `want` paths from the pool into the lanes of `vacant` (caller holds nothing; the
// leader takes the lock). `idle`: the wave holds no path yet, so it takes only when at least
// RT_POOL_T paths wait or no wave is working, and counts itself working when it takes any.
// Returns the number taken (wave-uniform).
__device__ __forceinline__ uint32_t pool_take(PoolCtl* ctl, uint32_t* pool, uint32_t cap, uint32_t lane,
                                              unsigned long long vacant, bool idle, uint32_t& st,
                                              Path& ps, Ray& r) {
    const int leader = __ffsll(vacant) - 1;
    uint32_t base = 0, k = 0;
    if (int(lane) == leader) {
        pool_lock(ctl);
        const uint32_t c = ctl->count;
        if (!idle || c >= RT_POOL_T || pool_peek(ctl, 2) == 0u) {
            k = min(c, (uint32_t)__popcll(vacant));
            base = c - k;
        }
        if (k == 0u) pool_unlock(ctl);
    }
    k = __shfl(k, leader);
    if (k == 0u) return 0u;
    base = __shfl(base, leader);
    const uint32_t rank = __popcll(vacant & ((1ull << lane) - 1ull));
    if (((vacant >> lane) & 1ull) && rank < k) pool_get(pool, cap, base + rank, st, ps, r);
    __threadfence_block();   // every lane's reads are back before the slots can be reused
    if (int(lane) == leader) {
        ctl->count = base;
        if (idle) atomicAdd(&ctl->working, 1u);
        pool_unlock(ctl);
    }
    return k;
}

// ---------------------------------------------------------------------------------------------
// LBVH kernel, classic form: one segment per lane per loop iteration; the wave's walk loop runs
// until its longest walk ends. Stamp slots: 0 refill+sample start, 1 ray setup (big spheres),
// 2 LBVH walk, 3 shading, 7 other. POOL: tail compaction through the block's LDS pool.
// Finished pixel: its chain length (traced segments) feeds the next launch's hand-out order.
__device__ __forceinline__ void record_tile_cost(const rt::TraceParams& P, const Path& ps) {
    if (!P.tile_cost) return;
    const uint32_t lx = ps.px & 0xffffu, ly = ps.px >> 16;
    uint32_t* c = &P.tile_cost[(ly >> 3) * P.tiles_x + (lx >> 3)];
    if (P.tile_cost_sum) atomicAdd(c, ps.segs); else atomicMax(c, ps.segs);
}

// ---------------------------------------------------------------------------------------------
template <bool COUNT, bool NODE16, bool POOL, int LAYOUT>
__device__ __forceinline__ void lbvh_classic(const rt::TraceParams& P, const float4* __restrict__ nodes4,
                                             const float4* __restrict__ leaf4,
                                             const uint32_t* __restrict__ leaf_ids,
                                             const float4* __restrict__ geom4,
                                             const float4* __restrict__ mat4,
                                             PoolCtl* ctl, uint32_t* pool, uint32_t cap) {
    const uint32_t lane = lane_id();
    const Camera cam = load_camera(P);
    uint32_t st = ST_NEED_PIXEL;
    Path ps{};
    Ray r{};
    uint32_t n_seg = 0, n_smp = 0, n_box = 0, n_sph = 0;
    unsigned long long wave_iters = 0;
    bool saw_dry = false;
    WaveChunk ch;
    {   // the first tiles go out by wave id, not through the counter (host starts it past them):
        // 16 Ki waves asking one address at once would queue for ~0.1 ms. Tile ranks are dealt
        // across blocks first (rank = wave-in-block * blocks + block), so the longest chains of
        // the LPT order start on different CUs (and XCDs) instead of sharing block 0's SIMDs.
        // (12 spp: -2.3 % against rank = global wave id; 100 spp: equal)
        const uint32_t wid = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
        if (wid < P.first_chunks) {
            ch.next = wid * 64u;
            ch.end = ch.next + 64u;
            ch.tile = P.tile_order ? load_now(P.tile_order + wid) : wid;
            ch.seed = tile_pixel_seed(P, ch.tile, lane);
            if (wid < P.isolate_tiles) ch.dry = ch.done = true;   // no work beyond its first tile
        }
    }
    // launch telemetry (3 atomics per wave): first start, pixel queue dry, last exit
    if (lane == 0) atomicMin(&P.counters->t_first, __builtin_amdgcn_s_memrealtime());
    STAMP_DECL;
    for (;;) {
        STAMP(0);
        if (!POOL || !saw_dry) {
            if (P.n_chunk_units) refill_chunked(P, lane, st, ps, ch STAMP_ARG);
            else refill(P, lane, st, ps);
        } else if (st == ST_NEED_PIXEL) {
            st = ST_RETIRED;   // the queue never refills once dry
        }
        if (!saw_dry && __ballot(st == ST_RETIRED)) {   // this wave saw the queue run dry
            saw_dry = true;
            if (lane == 0) atomicMin(&P.counters->t_dry, __builtin_amdgcn_s_memrealtime());
            if (POOL && st == ST_NEED_PIXEL) st = ST_RETIRED;
        }
        STAMP(4);
        if (POOL && saw_dry) {
            const unsigned long long held = __ballot(st == ST_TRACING || st == ST_NEED_SAMPLE);
            uint32_t n_held = __popcll(held);
            if (n_held != 0u && n_held < RT_POOL_T) {   // donate, if another wave keeps working
                const int leader = __ffsll(held) - 1;
                uint32_t base = 0, ok = 0;
                if (int(lane) == leader) {
                    pool_lock(ctl);
                    ok = pool_peek(ctl, 2) > 1u ? 1u : 0u;
                    base = ctl->count;
                    if (!ok) pool_unlock(ctl);
                }
                if (__shfl(ok, leader)) {
                    base = __shfl(base, leader);
                    if ((held >> lane) & 1ull) {
                        pool_put(pool, cap, base + __popcll(held & ((1ull << lane) - 1ull)), st, ps, r);
                        st = ST_RETIRED;
                    }
                    __threadfence_block();   // slots written before the count publishes them
                    if (int(lane) == leader) {
                        ctl->count = base + n_held;
                        atomicSub(&ctl->working, 1u);
                        pool_unlock(ctl);
                    }
                    n_held = 0u;
                }   // refused (the only working wave): keep the paths, top up below

            } else if (n_held == 0u) {   // idle since the last iteration: stop counting as working
                if (lane == 0) atomicSub(&ctl->working, 1u);
            }
            if (n_held == 0u) {   // idle: wait for paths, or for the block's end
                bool done = false;
                for (;;) {
                    const uint32_t c = pool_peek(ctl, 1), w = pool_peek(ctl, 2);
                    if (c >= RT_POOL_T || (c != 0u && w == 0u)) {
                        if (pool_take(ctl, pool, cap, lane, ~0ull, true, st, ps, r)) break;
                    } else if (c == 0u && w == 0u) {
                        uint32_t fin = 0;
                        if (lane == 0) {
                            pool_lock(ctl);
                            fin = (ctl->count == 0u && pool_peek(ctl, 2) == 0u) ? 1u : 0u;
                            pool_unlock(ctl);
                        }
                        if (__shfl(fin, 0)) { done = true; break; }
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
                if (done) break;
            } else if (n_held < 64u && pool_peek(ctl, 1) != 0u) {   // top up empty lanes
                pool_take(ctl, pool, cap, lane, ~held, false, st, ps, r);
            }
        }
        if (st == ST_NEED_SAMPLE) {
            if (start_sample(P, cam, ps, r.o, r.d)) {
                st = ST_TRACING;
                n_smp++;
            } else {   // pixel done (spp = 0 only: others finish at their last sample's end)
                st = ST_NEED_PIXEL;
                record_tile_cost(P, ps);
            }
        }
        if (__ballot(st == ST_NEED_PIXEL)) continue;   // refill before the next trace
        const unsigned long long tracing = __ballot(st == ST_TRACING);
        if (!tracing) {                                 // every lane retired
            if (POOL && saw_dry) continue;              // the pool stage decides idle / exit
            break;
        }
        if (COUNT && lane == 0) atomicAdd(&P.counters->lane_hist[__popcll(tracing)], 1ull);
        STAMP(1);
        const uint32_t box0 = n_box;
        if (st == ST_TRACING) setup_ray(P, r, n_sph);
        STAMP(2);
        if (st == ST_TRACING) {
            if (NODE16)
                walk_escape16<COUNT>(P, reinterpret_cast<const uint4*>(nodes4), leaf4, leaf_ids, r, n_box, n_sph);
            else
                walk_escape<COUNT, LAYOUT>(P, nodes4, leaf4, leaf_ids, r, n_box, n_sph);
        }
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
        if (st == ST_TRACING) {
            n_seg++;
            ps.segs++;
            if (!shade(P, geom4, mat4, ps, r.bi, r.best, r.o, r.d)) {
                // The sample ended. After the pixel's last one, store it here rather than at the
                // next sample start: the lane asks for a pixel at the top of the next iteration
                // directly, instead of costing its wave one extra pass of the loop head.
                if (ps.s >= P.spp) {
                    store_pixel(P, ps);
                    record_tile_cost(P, ps);
                    st = ST_NEED_PIXEL;
                } else {
                    st = ST_NEED_SAMPLE;
                }
            }
        }
    }
    STAMP_FLUSH;
    atomicAdd(&P.counters->segments, (unsigned long long)n_seg);
    atomicAdd(&P.counters->samples, (unsigned long long)n_smp);
    if (lane == 0) atomicMax(&P.counters->t_last, __builtin_amdgcn_s_memrealtime());
    if (COUNT) {
        atomicAdd(&P.counters->box_tests, (unsigned long long)n_box);
        atomicAdd(&P.counters->sphere_tests, (unsigned long long)n_sph);
        if (lane == 0) atomicAdd(&P.counters->wave_iters, wave_iters);
    }
}

#ifndef RT_LBVH_BLOCK
#define RT_LBVH_BLOCK 512
#endif
constexpr uint32_t kTopBlock = 1024;   // one block per CU shares one staged treelet

// LBVH kernel. LDS: stage the tree (nodes, leaf spheres, leaf ids) and, when SCENE_LDS, the
// per-sphere geometry + material records read by shading, once per persistent block. Blocks of
// BLOCK threads share one staged copy. Staged nodes use the AB layout (node_hit); OCT stages 8
// copies, one per ray direction octant. POOL: the tail-compaction pool (BLOCK slots x
// kPoolFields words) follows the staged data.
template <bool LDS, bool COUNT, bool NODE16, bool SCENE_LDS, bool POOL, uint32_t NOCT, uint32_t BLOCK>
__global__ __launch_bounds__(BLOCK, RT_TRACE_WAVES_PER_SIMD) void rt_trace_lbvh_kernel(const rt::TraceParams P) {
    extern __shared__ float4 lds[];
    __shared__ PoolCtl ctl;
    const float4* nodes4 = NODE16 ? reinterpret_cast<const float4*>(P.nodes16)
                                  : reinterpret_cast<const float4*>(P.nodes);
    const float4* leaf4 = reinterpret_cast<const float4*>(P.leaf_geom);
    const uint32_t* leaf_ids = P.leaf_ids;
    const float4* geom4 = reinterpret_cast<const float4*>(P.geom);
    const float4* mat4 = reinterpret_cast<const float4*>(P.mat);
    uint32_t staged4 = 0;
    if (LDS) {
        const uint32_t n_node4 = (NODE16 ? 1u : 2u * NOCT) * P.n_nodes, n_leaf4 = P.n_leaf,
                       n_id4 = (P.n_leaf + 3u) / 4u;
        if (NODE16) {
            for (uint32_t i = threadIdx.x; i < n_node4; i += BLOCK) lds[i] = nodes4[i];
        } else {
            typedef const __attribute__((address_space(3))) float4* LdsF4;
            const uint32_t lbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)lds));   // LDS address of lds[0]
            for (uint32_t oi = threadIdx.x; oi < NOCT * P.n_nodes; oi += BLOCK) {
                const uint32_t o = oi / P.n_nodes, i = oi - o * P.n_nodes;   // copy o, node i
                // BvhNode: lo.xyz escape, hi.xyz leaf. Octant copies come in their own
                // near-child-first order when the host provides one (escape links per copy).
                const float4* src = (NOCT == 8 && P.nodes_oct)
                                        ? reinterpret_cast<const float4*>(P.nodes_oct + size_t(o) * P.n_nodes)
                                        : nodes4;
                const float4 lo = src[2 * i], hi = src[2 * i + 1];
                // Links (walk_escape, AB layout): LDS address of the target node in this copy,
                // END = ~0; a hit leaf yields 0x80000000 | escape node << 12 |
                // leaf index << 2 | (count - 1), escape node = 0x7ffff for END. (Trees staged in
                // LDS have < 2^14 nodes and < 1024 leaves of <= 4 slots, checked by the host.)
                const uint32_t esc = __float_as_uint(lo.w), fc = __float_as_uint(hi.w);
                {   // bit k of o: axis k runs negative, near = hi
                    const bool nx = o & 1u, ny = o & 2u, nz = o & 4u;
                    const uint32_t cb = o * P.n_nodes;   // first node of copy o
                    const uint32_t miss = esc == END ? END : lbase + (cb + esc) * 32u;
                    // (kept as separate statements: one combined expression crashed the ROCm 7.2
                    // instruction selector)
                    const uint32_t escf = esc == END ? 0x7ffffu : cb + esc;
                    const uint32_t leafw = 0x80000000u + (escf << 12) + ((fc >> 6) << 2) + ((fc - 1u) & 3u);
                    const uint32_t hit = fc ? leafw : lbase + (cb + i + 1u) * 32u;
                    const size_t b = size_t(cb + i) * 2u;
                    lds[b] = make_float4(nx ? hi.x : lo.x, ny ? hi.y : lo.y, nx ? lo.x : hi.x, ny ? lo.y : hi.y);
                    lds[b + 1] = make_float4(nz ? hi.z : lo.z, nz ? lo.z : hi.z, __uint_as_float(miss), __uint_as_float(hit));
                }
            }
        }
        for (uint32_t i = threadIdx.x; i < n_leaf4; i += BLOCK) lds[n_node4 + i] = leaf4[i];
        const uint4* ids4 = reinterpret_cast<const uint4*>(P.leaf_ids);
        for (uint32_t i = threadIdx.x; i < n_id4; i += BLOCK) {
            const uint4 v = ids4[i];
            lds[n_node4 + n_leaf4 + i] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y),
                                                     __uint_as_float(v.z), __uint_as_float(v.w));
        }
        const uint32_t base = n_node4 + n_leaf4 + n_id4;
        staged4 = base;
        if (SCENE_LDS) {
            const uint32_t ng = P.n_spheres, nm = 2u * P.n_spheres;
            for (uint32_t i = threadIdx.x; i < ng; i += BLOCK) lds[base + i] = geom4[i];
            for (uint32_t i = threadIdx.x; i < nm; i += BLOCK) lds[base + ng + i] = mat4[i];
            geom4 = lds + base;
            mat4 = lds + base + ng;
            staged4 = base + ng + nm;
        }
        nodes4 = lds;
        leaf4 = lds + n_node4;
        leaf_ids = reinterpret_cast<const uint32_t*>(lds + n_node4 + n_leaf4);
    }
    if (POOL && threadIdx.x == 0) {
        ctl.lock = 0u;
        ctl.count = 0u;
        ctl.working = BLOCK / 64u;   // every wave enters the loop holding (or about to hold) paths
        ctl.pad = 0u;
    }
    if (LDS || POOL) __syncthreads();
    lbvh_classic<COUNT, NODE16, POOL, (LDS && !NODE16) ? (NOCT == 8 ? 2 : 1) : 0>(
        P, nodes4, leaf4, leaf_ids, geom4, mat4, &ctl, reinterpret_cast<uint32_t*>(lds + staged4), BLOCK);
}

// LBVH kernel for trees too big for LDS (ACCEL_LBVH_TOP): the treelet (rt_build.hip
// build_treelet) is staged in LDS with its rank links turned into LDS addresses; leaves,
// subtrees below the cut, geometry and materials stay in HBM/L2.
template <bool COUNT>
__global__ __launch_bounds__(kTopBlock, RT_TRACE_WAVES_PER_SIMD) void rt_trace_top_kernel(const rt::TraceParams P) {
    extern __shared__ float4 lds[];
    __shared__ PoolCtl ctl;
    typedef const __attribute__((address_space(3))) float4* LdsF4;
    const uint32_t lbase = uint32_t(reinterpret_cast<uintptr_t>((LdsF4)lds));
    const uint32_t n_top = min(*P.treelet_count, rt::kTreeletCap);
    for (uint32_t i = threadIdx.x; i < n_top; i += kTopBlock) {
        const float4* tl = reinterpret_cast<const float4*>(P.treelet);
        const float4 A = tl[2 * i], B = tl[2 * i + 1];
        const uint32_t miss = __float_as_uint(B.z), hit = __float_as_uint(B.w);
        lds[2 * i] = A;
        lds[2 * i + 1] = make_float4(B.x, B.y, __uint_as_float(miss == END ? END : lbase + miss * 32u),
                                     __uint_as_float(int32_t(hit) >= 0 ? lbase + hit * 32u : hit));
    }
    __syncthreads();
    lbvh_classic<COUNT, false, false, 3>(P, lds, reinterpret_cast<const float4*>(P.leaf_geom), P.leaf_ids,
                                         reinterpret_cast<const float4*>(P.geom),
                                         reinterpret_cast<const float4*>(P.mat), &ctl, nullptr, kTopBlock);
}

// ---------------------------------------------------------------------------------------------
// LBVH kernel, ordered walk. Dynamic LDS: [staged nodes2 | leaf spheres | leaf ids] (LDS
// variant only) followed by the per-lane stacks, stack_depth words per lane, lane-interleaved.
// ---------------------------------------------------------------------------------------------
template <bool LDS, bool COUNT, uint32_t BLOCK>
__global__ __launch_bounds__(BLOCK, RT_TRACE_WAVES_PER_SIMD) void rt_trace_lbvh2_kernel(const rt::TraceParams P) {
    extern __shared__ float4 lds[];
    const float4* nodes4 = reinterpret_cast<const float4*>(P.nodes2);
    const float4* leaf4 = reinterpret_cast<const float4*>(P.leaf_geom);
    const uint32_t* leaf_ids = P.leaf_ids;
    uint32_t staged4 = 0;
    if (LDS) {
        const uint32_t n_node4 = 4u * P.n_nodes2, n_leaf4 = P.n_leaf, n_id4 = (P.n_leaf + 3u) / 4u;
        for (uint32_t i = threadIdx.x; i < n_node4; i += BLOCK) lds[i] = nodes4[i];
        for (uint32_t i = threadIdx.x; i < n_leaf4; i += BLOCK) lds[n_node4 + i] = leaf4[i];
        const uint4* ids4 = reinterpret_cast<const uint4*>(P.leaf_ids);
        for (uint32_t i = threadIdx.x; i < n_id4; i += BLOCK) {
            const uint4 v = ids4[i];
            lds[n_node4 + n_leaf4 + i] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y),
                                                     __uint_as_float(v.z), __uint_as_float(v.w));
        }
        __syncthreads();
        nodes4 = lds;
        leaf4 = lds + n_node4;
        leaf_ids = reinterpret_cast<const uint32_t*>(lds + n_node4 + n_leaf4);
        staged4 = n_node4 + n_leaf4 + n_id4;
    }
    uint32_t* stk = reinterpret_cast<uint32_t*>(lds + staged4) + threadIdx.x;

    const uint32_t lane = lane_id();
    const Camera cam = load_camera(P);
    uint32_t st = ST_NEED_PIXEL;
    Path ps{};
    Ray r{};
    uint32_t n_seg = 0, n_smp = 0, n_box = 0, n_sph = 0;
    unsigned long long wave_iters = 0;
    STAMP_DECL;
    for (;;) {
        STAMP(0);
        refill(P, lane, st, ps);
        if (st == ST_NEED_SAMPLE) {
            if (start_sample(P, cam, ps, r.o, r.d)) { st = ST_TRACING; n_smp++; }
            else st = ST_NEED_PIXEL;
        }
        if (__ballot(st == ST_NEED_PIXEL)) continue;   // refill before the next trace
        if (!__ballot(st == ST_TRACING)) break;         // every lane retired
        STAMP(1);
        if (st == ST_TRACING) setup_ray(P, r, n_sph);
        STAMP(2);
        const uint32_t box0 = n_box;
        if (st == ST_TRACING) walk_ordered<COUNT>(P, nodes4, leaf4, leaf_ids, stk, BLOCK, r, n_box, n_sph);
        if (COUNT) {
            uint32_t m = (n_box - box0) / 2u;
            for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor(m, off));
            if (lane == 0) wave_iters += m;
        }
        STAMP(3);
        if (st == ST_TRACING) {
            n_seg++;
            if (!shade(P, reinterpret_cast<const float4*>(P.geom), reinterpret_cast<const float4*>(P.mat),
                       ps, r.bi, r.best, r.o, r.d))
                st = ST_NEED_SAMPLE;
        }
    }
    STAMP_FLUSH;
    atomicAdd(&P.counters->segments, (unsigned long long)n_seg);
    atomicAdd(&P.counters->samples, (unsigned long long)n_smp);
    if (COUNT) {
        atomicAdd(&P.counters->box_tests, (unsigned long long)n_box);
        atomicAdd(&P.counters->sphere_tests, (unsigned long long)n_sph);
        if (lane == 0) atomicAdd(&P.counters->wave_iters, wave_iters);
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

// Sum of ns accumulator slices in slice order, then the trace kernel's pixel store
// (shader.rgen:63-66) of the sum (rt_reduce_resolve / rt_resolve_rgba8). HBM-bound: ns x 16 B
// read + 16 B (acc_out) + 4 B written per texel. acc_out may alias slice 0 (same-index update).
__global__ __launch_bounds__(256) void rt_reduce_resolve_kernel(const float4* slices, uint32_t ns, uint64_t n,
                                                                float spp, float4* acc_out,
                                                                uint32_t* __restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        float4 s = slices[i];
        for (uint32_t q = 1; q < ns; ++q) {
            const float4 v = slices[uint64_t(q) * n + i];
            s.x = s.x + v.x;
            s.y = s.y + v.y;
            s.z = s.z + v.z;
        }
        if (acc_out) acc_out[i] = make_float4(s.x, s.y, s.z, 1.0f);
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
        default: r = 0.0f;
    }
    out[i] = r;
}

}  // namespace

// ---- host-callable launchers (rt_api.cpp) ---------------------------------------------------
namespace rt {

#ifndef RT_LBVH2_BLOCK
#define RT_LBVH2_BLOCK 256
#endif
constexpr uint32_t kLbvh2Block = RT_LBVH2_BLOCK;

constexpr uint32_t kLbvhBlock = RT_LBVH_BLOCK;

#ifndef RT_POOL_BLOCK
#define RT_POOL_BLOCK 1024
#endif
constexpr uint32_t kPoolBlock = RT_POOL_BLOCK;   // one block per CU: the pool spans all 16 waves

#define RT_LBVH_FN(L, C, N16, S) reinterpret_cast<const void*>(rt_trace_lbvh_kernel<L, C, N16, S, false, 1u, kLbvhBlock>)
#define RT_POOL_FN(C) reinterpret_cast<const void*>(rt_trace_lbvh_kernel<true, C, false, true, true, 1u, kPoolBlock>)
#define RT_OCT_FN(C) reinterpret_cast<const void*>(rt_trace_lbvh_kernel<true, C, false, true, false, 8u, kPoolBlock>)
static const void* pick(uint32_t accel, bool count) {
    switch (accel) {
        case ACCEL_BRUTE:
            return count ? reinterpret_cast<const void*>(rt_trace_brute_kernel<true>)
                         : reinterpret_cast<const void*>(rt_trace_brute_kernel<false>);
        case ACCEL_LBVH_LDS:
            return count ? RT_LBVH_FN(true, true, false, false) : RT_LBVH_FN(true, false, false, false);
        case ACCEL_LBVH_LDS_SCENE:
            return count ? RT_LBVH_FN(true, true, false, true) : RT_LBVH_FN(true, false, false, true);
        case ACCEL_LBVH_POOL:
            return count ? RT_POOL_FN(true) : RT_POOL_FN(false);
        case ACCEL_LBVH_OCT:
            return count ? RT_OCT_FN(true) : RT_OCT_FN(false);
        case ACCEL_LBVH_TOP:
            return count ? reinterpret_cast<const void*>(rt_trace_top_kernel<true>)
                         : reinterpret_cast<const void*>(rt_trace_top_kernel<false>);
        case ACCEL_LBVH16_LDS:
            return count ? RT_LBVH_FN(true, true, true, false) : RT_LBVH_FN(true, false, true, false);
        case ACCEL_LBVH2:
            return count ? reinterpret_cast<const void*>(rt_trace_lbvh2_kernel<false, true, kLbvh2Block>)
                         : reinterpret_cast<const void*>(rt_trace_lbvh2_kernel<false, false, kLbvh2Block>);
        case ACCEL_LBVH2_LDS:
            return count ? reinterpret_cast<const void*>(rt_trace_lbvh2_kernel<true, true, kLbvh2Block>)
                         : reinterpret_cast<const void*>(rt_trace_lbvh2_kernel<true, false, kLbvh2Block>);
        default:
            return count ? RT_LBVH_FN(false, true, false, false) : RT_LBVH_FN(false, false, false, false);
    }
}
#undef RT_LBVH_FN
#undef RT_POOL_FN
#undef RT_OCT_FN

uint32_t block_size(uint32_t accel) {
    switch (accel) {
        case ACCEL_LBVH2: case ACCEL_LBVH2_LDS: return kLbvh2Block;
        case ACCEL_BRUTE: return 256u;
        case ACCEL_LBVH_POOL: case ACCEL_LBVH_OCT: return kPoolBlock;
        case ACCEL_LBVH_TOP: return kTopBlock;
        default: return kLbvhBlock;
    }
}

hipError_t launch_trace(const TraceParams& P, uint32_t accel, bool count, int grid, size_t lds_bytes,
                        hipStream_t st) {
    void* args[] = {const_cast<TraceParams*>(&P)};
    return hipLaunchKernel(pick(accel, count), dim3(grid), dim3(block_size(accel)), args, lds_bytes, st);
}

size_t pool_bytes(uint32_t accel) {
    return accel == ACCEL_LBVH_POOL ? size_t(kPoolBlock) * kPoolFields * 4u : 0u;
}

hipError_t trace_occupancy(uint32_t accel, bool count, size_t lds_bytes, int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, pick(accel, count),
                                                        block_size(accel), lds_bytes);
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

hipError_t launch_reduce_resolve(const float* slices, uint32_t n_slices, uint64_t n_texels, uint32_t spp,
                                 float* accum_out, uint8_t* out, hipStream_t st) {
    const uint64_t need = (n_texels + 255) / 256, blocks = need < 8192 ? need : 8192;
    hipLaunchKernelGGL(rt_reduce_resolve_kernel, dim3(uint32_t(blocks)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(slices), n_slices, n_texels, float(spp),
                       reinterpret_cast<float4*>(accum_out), reinterpret_cast<uint32_t*>(out));
    return hipGetLastError();
}

hipError_t launch_debug_math(int op, const float* in, float* out, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(rt_debug_math_kernel, dim3((n + 255) / 256), dim3(256), 0, st, op, in, out, n);
    return hipGetLastError();
}

}  // namespace rt
