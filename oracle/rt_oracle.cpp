/*
 * rt_oracle.cpp — CPU ORACLE (test infrastructure, not product code).
 *
 * A scalar C++ restatement of the reference hot path, used ONLY by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, as the checker and as the
 * timed CPU baseline ("kind": "port"). The product (librt_mi355x.so) never links, loads or
 * calls anything in this directory.
 *
 * What it restates (all paths relative to the reference repo root):
 *   random.glsl:1-34                 TEA seed hash, LCG, 24-bit float, interval, unit vector
 *   shader.rgen:39-115               per-pixel seed, sample loop with double sum, depth-50
 *                                    bounce loop, viewport, camera ray, tonemap
 *   shader.rint:22-60                ray-sphere quadratic, t1-else-t2 report within [tmin, tmax]
 *   shader.rchit:38-133              normal/front face, solid+checker texture, diffuse / metal /
 *                                    dielectric scatter, Schlick
 *   shader.rmiss:13-18               constant sky
 *   scene.h:37-157                   generateRandomScene (libstdc++ mt19937 +
 *                                    uniform_real_distribution<float>, g++ 11.4 / libstdc++ 11)
 *   driver BVH traversal             closest hit by brute force over all spheres, first minimum
 *                                    by index on ties
 *
 * Pins (tests/test_oracle.py): RNG known answers and scene FNV-1a-64 b1fa62b66a87952d from
 * SURVEY.md §4, both produced from the reference's own code (random.glsl restated in C and
 * Python; scene.h compiled by g++ during the survey). Traversal and shading arithmetic have no
 * reference fixture (the reference has no tests and its GLSL cannot run here): that part of the
 * oracle is "parity unpinned" against the reference and pinned only by this restatement.
 *
 * ARITHMETIC CONTRACT — shared with the HIP kernels, each side implemented
 * independently:
 *   * IEEE binary32, round-to-nearest-even, denormals kept, no contraction except where an
 *     fma is written explicitly below (build with -ffp-contract=off).
 *   * dot(a,b)       = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
 *   * normalize(v)   = v * (1 / sqrt(dot(v,v)))           (correctly rounded sqrt and divide)
 *   * D (rint:49)    = fma(b, b, -(a*c))
 *   * hit point      = fma(t, d, o) per component        (rint:33/37)
 *   * sin (rchit:59) = rt_sinf below: 3-part Cody-Waite reduction + fdlibm float kernels
 *   * pow(x, 2.0)    = x*x (rchit:131, Q7);  pow(x, 5.0) = NaN for x < 0 else (x*x)*(x*x)*x (Q8)
 *   * everything else exactly as written in GLSL, left to right, one rounding per operator.
 */
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <thread>
#include <vector>

#include "../include/rt_abi.h"
#include "../include/rt_mi355x.h"

namespace {

// ------------------------------------------------------------------------------------
// random.glsl
// ------------------------------------------------------------------------------------

// random.glsl:1-13 getRandomSeed: 16-round TEA, returns v0.
uint32_t tea(uint32_t v0, uint32_t v1) {
    uint32_t s0 = 0;
    for (uint32_t n = 0; n < 16; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}

// random.glsl:15-18 randomInt
inline uint32_t random_int(uint32_t& seed) {
    seed = 1664525u * seed + 1013904223u;
    return seed;
}

// random.glsl:20-22 randomFloat — exact: a 24-bit integer times 2^-24.
inline float random_float(uint32_t& seed) {
    return float(random_int(seed) & 0x00FFFFFFu) / float(0x01000000u);
}

// random.glsl:24-26 randomInInterval: randomFloat * (max - min) + min (no contraction).
inline float random_in_interval(uint32_t& seed, float mn, float mx) {
    float r = random_float(seed);
    float span = mx - mn;
    float prod = r * span;
    return prod + mn;
}

struct V3 { float x, y, z; };

inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 scale(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
// Arithmetic forms (orc_render's opt->reserved[1]): L = LIT_CONTRACT is the shipped
// contract that the HIP kernels implement; LIT_RINT reads shader.rint:33-55 as
// written (D = b*b - a*c unfused, roots divided by a, hit point o + t*d unfused); LIT_ALL also
// takes every dot() unfused left to right and normalize(v) = v / length(v) (GLSL 4.60 §8.5)
// everywhere. The two literal forms exist to MEASURE the contract's distance from the GLSL as
// written; the kernels never implement them.
enum { LIT_CONTRACT = 0, LIT_RINT = 1, LIT_ALL = 2 };
template <int L = LIT_CONTRACT>
inline float dot(V3 a, V3 b) {
    if (L == LIT_ALL) {
        float xx = a.x * b.x, yy = a.y * b.y, zz = a.z * b.z;
        return (xx + yy) + zz;
    }
    return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x));
}
template <int L = LIT_CONTRACT>
inline V3 normalize(V3 v) {
    float len = std::sqrt(dot<L>(v, v));
    if (L == LIT_ALL) return v3(v.x / len, v.y / len, v.z / len);
    float inv = 1.0f / len;
    return v3(v.x * inv, v.y * inv, v.z * inv);
}
// GLSL cross, a.yzx*b.zxy - a.zxy*b.yzx, one rounding per operator.
inline V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N
template <int L = LIT_CONTRACT>
inline V3 reflect(V3 i, V3 n) {
    float k = 2.0f * dot<L>(n, i);
    return sub(i, scale(k, n));
}
// GLSL refract(I, N, eta)
template <int L = LIT_CONTRACT>
inline V3 refract(V3 i, V3 n, float eta) {
    float d = dot<L>(n, i);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return v3(0.0f, 0.0f, 0.0f);
    float s = eta * d + std::sqrt(k);
    return sub(scale(eta, i), scale(s, n));
}

// random.glsl:28-30 randomVector — GLSL evaluates constructor arguments left to right.
inline V3 random_vector(uint32_t& seed, float mn, float mx) {
    float x = random_in_interval(seed, mn, mx);
    float y = random_in_interval(seed, mn, mx);
    float z = random_in_interval(seed, mn, mx);
    return v3(x, y, z);
}
// random.glsl:32-34
template <int L = LIT_CONTRACT>
inline V3 random_unit_vector(uint32_t& seed) { return normalize<L>(random_vector(seed, -1.0f, 1.0f)); }

// ------------------------------------------------------------------------------------
// sin for the checker texture (shader.rchit:59). Deterministic: only +,-,*,fma, rint.
// ------------------------------------------------------------------------------------
float rt_sinf(float x) {
    const float two_over_pi = 0.636619772f;
    const float pio2_hi = 1.5707962513e+00f;   // 0x3fc90fda
    const float pio2_mid = 7.5497894159e-08f;  // 0x33a22168
    const float pio2_lo = 5.3903029534e-15f;   // 0x27c234c4
    float k = std::rint(x * two_over_pi);
    float r = std::fma(-k, pio2_hi, x);
    r = std::fma(-k, pio2_mid, r);
    r = std::fma(-k, pio2_lo, r);
    int q = int(k) & 3;  // |k| < 2^24 for every x the tracer passes (|x| <= 6e5)
    float r2 = r * r;
    float s, c;
    {   // fdlibm __kernel_sindf coefficients (float)
        float p = std::fma(r2, -1.9515295891e-04f, 8.3321608736e-03f);
        p = std::fma(r2, p, -1.6666654611e-01f);
        s = std::fma(r * r2, p, r);
    }
    {   // fdlibm __kernel_cosdf coefficients (float)
        float p = std::fma(r2, 2.4433157118e-05f, -1.3887316255e-03f);
        p = std::fma(r2, p, 4.1666645683e-02f);
        float r4 = r2 * r2;
        c = std::fma(r4, p, std::fma(-0.5f, r2, 1.0f));
    }
    switch (q) {
        case 0: return s;
        case 1: return c;
        case 2: return -s;
        default: return -c;
    }
}

// RT_RNG_SAMPLE_HASH: LCG start of sample s (golden-ratio spread + "lowbias32" finaliser).
inline uint32_t sample_seed_hash(uint32_t pixel_seed, uint32_t s) {
    uint32_t x = pixel_seed + 0x9E3779B9u * s;
    x ^= x >> 16;
    x *= 0x21F0AAADu;
    x ^= x >> 15;
    x *= 0x735A2D97u;
    x ^= x >> 15;
    return x;
}

// RT_RNG_SAMPLE_HASH: a colour channel as 8.24 fixed point, truncated (NaN -> 0).
inline uint64_t sample_fixed(float c) {
    float v = std::fmin(std::fmax(c, 0.0f), 1.0f) * 0x1p24f;
    return uint64_t(v);
}

inline float pow5_glsl(float x) {
    if (x < 0.0f) return std::numeric_limits<float>::quiet_NaN();
    float x2 = x * x;
    return x2 * x2 * x;
}

// ------------------------------------------------------------------------------------
// Camera and viewport, shader.rgen:29, :48-49, :92-105. Computed once per launch (uniform).
// ------------------------------------------------------------------------------------
struct Viewport {
    V3 look_from, horizontal, vertical, upper_left, cam_up, cam_right;
    float aperture;
};

template <int L = LIT_CONTRACT>
Viewport make_viewport(const RenderCallInfo& rci) {
    // shader.rgen:29 Camera(25.0f, 0.0f, 10.0f, ...), up = (0,1,0); lookFrom/lookAt from rci.
    const float fov = 25.0f, aperture = 0.0f, focus = 10.0f;
    const V3 up = v3(0.0f, 1.0f, 0.0f);
    V3 look_from = v3(rci.camera_pos.x, rci.camera_pos.y, rci.camera_pos.z);
    V3 look_at = add(look_from, v3(rci.camera_dir.x, rci.camera_dir.y, rci.camera_dir.z));
    float sx = float(rci.image_size.x), sy = float(rci.image_size.y);
    float aspect = sx / sy;  // shader.rgen:43
    float rad = fov * 0.017453292519943295f;  // radians()
    float half = rad / 2.0f;
    float th = float(std::tan(double(half)));  // tan(), rounded once to float
    float vh = th * 2.0f;
    float vw = aspect * vh;
    V3 fwd = normalize<L>(sub(look_at, look_from));
    V3 right = normalize<L>(cross(up, fwd));
    V3 cup = normalize<L>(cross(fwd, right));
    Viewport vp;
    // viewportWidth * cameraRight * focusDistance, evaluated left to right
    vp.horizontal = v3(vw * right.x * focus, vw * right.y * focus, vw * right.z * focus);
    vp.vertical = v3(vh * cup.x * focus, vh * cup.y * focus, vh * cup.z * focus);
    // lookFrom - horizontal/2 + vertical/2 + forward*focus
    V3 h2 = v3(vp.horizontal.x / 2.0f, vp.horizontal.y / 2.0f, vp.horizontal.z / 2.0f);
    V3 v2 = v3(vp.vertical.x / 2.0f, vp.vertical.y / 2.0f, vp.vertical.z / 2.0f);
    V3 ff = v3(fwd.x * focus, fwd.y * focus, fwd.z * focus);
    vp.upper_left = add(add(sub(look_from, h2), v2), ff);
    vp.look_from = look_from;
    vp.cam_up = cup;
    vp.cam_right = right;
    vp.aperture = aperture;
    return vp;
}

// ------------------------------------------------------------------------------------
// Scene access and closest hit (driver traversal + shader.rint)
// ------------------------------------------------------------------------------------
const float T_MIN = 0.001f;       // shader.rgen:75
const float T_MAX = 10000.0f;     // shader.rgen:26

struct Hit { int idx; float t; };

// Driver traversal test for one sphere's AABB (src/ray_trace.cpp:586-596: center -/+ radius),
// restated as a slab test over [T_MIN, T_MAX]: per axis t = (bound - o) * (1/d); NaN slabs
// (d == 0 and bound == o) drop out through fmin/fmax.
inline bool aabb_hit(const rt_vec4& g, V3 o, V3 inv) {
    float x0 = ((g.x - g.w) - o.x) * inv.x, x1 = ((g.x + g.w) - o.x) * inv.x;
    float y0 = ((g.y - g.w) - o.y) * inv.y, y1 = ((g.y + g.w) - o.y) * inv.y;
    float z0 = ((g.z - g.w) - o.z) * inv.z, z1 = ((g.z + g.w) - o.z) * inv.z;
    float tnear = std::fmax(std::fmax(std::fmax(std::fmin(x0, x1), std::fmin(y0, y1)), std::fmin(z0, z1)), T_MIN);
    float tfar = std::fmin(std::fmin(std::fmin(std::fmax(x0, x1), std::fmax(y0, y1)), std::fmax(z0, z1)), T_MAX);
    return tnear <= tfar;
}

// Closest hit (driver traversal + shader.rint:22-60): sphere i is a candidate when the ray
// overlaps its AABB and the quadratic reports t (t1 if t1 >= tmin, else t2) inside
// [tmin, tmax]; the closest candidate wins, the lowest index on ties.
// A report at exactly tMax is accepted (reportIntersectionEXT), hence '<' against succ(T_MAX).
template <int L>
Hit closest_hit(const Sphere* sph, uint32_t n, V3 o, V3 d, uint64_t* tests) {
    float a = dot<L>(d, d);
    float ia = 1.0f / a;
    V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float best = std::nextafter(T_MAX, std::numeric_limits<float>::infinity());
    int bi = -1;
    for (uint32_t i = 0; i < n; i++) {
        const rt_vec4& g = sph[i].geometry;
        V3 oc = sub(o, v3(g.x, g.y, g.z));
        float b = dot<L>(oc, d);
        float rr = g.w * g.w;
        float c = dot<L>(oc, oc) - rr;
        float D;
        if (L == LIT_CONTRACT) {
            D = std::fma(b, b, -(a * c));
        } else {   // shader.rint:50 as written
            float bb = b * b, ac = a * c;
            D = bb - ac;
        }
        if (D >= 0.0f) {
            float sq = std::sqrt(D);
            float t1 = L == LIT_CONTRACT ? (-b - sq) * ia : (-b - sq) / a;   // shader.rint:55-56 as written: / a
            float t2 = L == LIT_CONTRACT ? (-b + sq) * ia : (-b + sq) / a;
            float t = (t1 >= T_MIN) ? t1 : t2;   // rint:32-39 (t1 > tMax implies t2 > tMax)
            if (t >= T_MIN && t < best && aabb_hit(g, o, inv)) { best = t; bi = int(i); }
        }
    }
    *tests += n;
    return Hit{bi, best};
}

struct Payload {
    bool does_scatter;
    V3 attenuation, scatter_dir, point;
};

// shader.rchit:53-64
V3 texture_color(const Sphere& s, V3 p) {
    if (s.textureType == RT_SOLID) return v3(s.colors[0].x, s.colors[0].y, s.colors[0].z);
    if (s.textureType == RT_CHECKERED) {
        const float size = 6.0f;
        float sines = rt_sinf(size * p.x) * rt_sinf(size * p.y) * rt_sinf(size * p.z);
        const rt_vec4& c = s.colors[sines > 0.0f ? 0 : 1];
        return v3(c.x, c.y, c.z);
    }
    return v3(s.colors[0].x, s.colors[0].y, s.colors[0].z);
}

inline bool near_zero(V3 v) {  // rchit:120-123
    const float s = 1e-8f;
    return std::fabs(v.x) < s && std::fabs(v.y) < s && std::fabs(v.z) < s;
}

// shader.rchit:38-49 + 66-133
template <int L>
void closest_hit_shader(const Sphere& s, V3 p, V3 dir, uint32_t& seed, Payload& pl) {
    V3 center = v3(s.geometry.x, s.geometry.y, s.geometry.z);
    V3 outward = normalize<L>(sub(p, center));
    bool front = dot<L>(dir, outward) < 0.0f;
    V3 n = front ? outward : neg(outward);
    pl.attenuation = texture_color(s, p);
    V3 sd;
    if (s.materialType == RT_DIFFUSE) {                      // rchit:68-76
        sd = add(n, random_unit_vector<L>(seed));
        if (near_zero(sd)) sd = n;
    } else if (s.materialType == RT_METAL) {                 // rchit:78-89
        V3 refl = reflect<L>(dir, n);
        V3 fuzz = scale(s.materialSpecificAttribute, random_unit_vector<L>(seed));
        V3 sc = normalize<L>(add(refl, fuzz));
        sd = (dot<L>(sc, n) > 0.0f) ? sc : v3(0.0f, 0.0f, 0.0f);
    } else if (s.materialType == RT_REFRACTIVE) {            // rchit:91-100, 125-133
        float attr = s.materialSpecificAttribute;
        float eta = front ? (1.0f / attr) : attr;
        float cos_t = dot<L>(neg(dir), n);
        bool can_refract = eta * std::sqrt(1.0f - cos_t * cos_t) <= 1.0f;
        bool refracts = false;
        if (can_refract) {  // && short-circuit: the draw happens only here
            float q = (1.0f - eta) / (1.0f + eta);
            float r = q * q;
            float refl = r + (1.0f - r) * pow5_glsl(1.0f - cos_t);
            refracts = refl < random_float(seed);
        }
        sd = refracts ? refract<L>(dir, n, eta) : reflect<L>(dir, n);
    } else {
        sd = v3(0.0f, 0.0f, 0.0f);
    }
    pl.scatter_dir = sd;
    pl.point = p;
    pl.does_scatter = !(sd.x == 0.0f && sd.y == 0.0f && sd.z == 0.0f);  // rchit:48
}

struct Counters { uint64_t segments = 0, samples = 0, sphere_tests = 0; };

// shader.rgen:70-89 calculateRayColor
template <int L>
V3 ray_color(const Sphere* sph, uint32_t n, V3 o, V3 d, uint32_t& seed, uint32_t max_depth,
             Counters& cnt) {
    V3 reflected = v3(1.0f, 1.0f, 1.0f);
    V3 light = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t depth = 0; depth < max_depth; depth++) {
        Hit h = closest_hit<L>(sph, n, o, d, &cnt.sphere_tests);
        cnt.segments++;
        Payload pl;
        if (h.idx >= 0) {
            V3 p = L == LIT_CONTRACT
                       ? v3(std::fma(h.t, d.x, o.x), std::fma(h.t, d.y, o.y), std::fma(h.t, d.z, o.z))
                       : add(o, scale(h.t, d));   // shader.rint:33/37 as written
            closest_hit_shader<L>(sph[h.idx], p, d, seed, pl);
        } else {  // shader.rmiss:13-18
            pl.does_scatter = false;
            pl.attenuation = v3(0.7f, 0.8f, 1.0f);
        }
        if (pl.does_scatter) {
            reflected = mul(reflected, pl.attenuation);
            o = pl.point;
            d = normalize<L>(pl.scatter_dir);
        } else {
            light = pl.attenuation;
            break;
        }
    }
    return mul(reflected, light);
}

inline uint8_t to_unorm8(float x) {
    // Vulkan UNORM conversion: clamp to [0,1] (NaN -> 0), then round to nearest.
    float v = (x > 0.0f) ? ((x < 1.0f) ? x : 1.0f) : 0.0f;
    return uint8_t(std::fma(v, 255.0f, 0.5f));
}

struct RenderJob {
    const Sphere* sph;
    uint32_t n;
    const RenderCallInfo* rci;
    const uint32_t* rows;
    uint32_t band_w, band_h;
    rt_options opt;
    Viewport vp;
    float* accum;
    uint8_t* out;
};

// shader.rgen:39-67 main() for one launch-id pixel (lx, ly).
template <int L>
void render_pixel(const RenderJob& job, uint32_t lx, uint32_t ly, Counters& cnt) {
    const RenderCallInfo& rci = *job.rci;
    uint32_t gx = rci.offset.x + lx;
    uint32_t gy = job.rows ? job.rows[ly] : rci.offset.y + ly;
    uint32_t sx = (job.opt.seed_mode == RT_SEED_LAUNCH_LOCAL) ? lx : gx;
    uint32_t sy = (job.opt.seed_mode == RT_SEED_LAUNCH_LOCAL) ? ly : gy;
    uint32_t pixel_seed = tea(tea(sx, sy), rci.number);
    uint32_t seed = pixel_seed;
    float size_x = float(rci.image_size.x), size_y = float(rci.image_size.y);
    float rox = float(gx), roy = float(gy);  // render_offset (shader.rgen:45)
    const Viewport& vp = job.vp;
    uint32_t max_depth = job.opt.max_depth ? job.opt.max_depth : 50u;

    size_t texel = (size_t(ly) * job.band_w + lx) * 4;
    float* acc = job.accum + texel;
    const bool hash = job.opt.rng_mode == RT_RNG_SAMPLE_HASH;
    double sum[3] = {0.0, 0.0, 0.0};
    uint64_t q[3] = {0, 0, 0};
    if (job.opt.accumulate) { sum[0] = acc[0]; sum[1] = acc[1]; sum[2] = acc[2]; }

    for (uint32_t i = 0; i < rci.samplesPerRenderCall; i++) {
        if (job.opt.rng_mode == RT_RNG_SAMPLE_COUNTER) seed = tea(pixel_seed, job.opt.sample_base + i);
        if (hash) seed = sample_seed_hash(pixel_seed, job.opt.sample_base + i);
        // shader.rgen:57 uv (x then y)
        float ux = rox + random_float(seed);
        float uy = roy + random_float(seed);
        ux = ux / size_x;
        uy = uy / size_y;
        // shader.rgen:107-115 getCameraRay
        float lx_ = random_in_interval(seed, -1.0f, 1.0f);
        float ly_ = random_in_interval(seed, -1.0f, 1.0f);
        float l2 = L == LIT_ALL ? std::sqrt(lx_ * lx_ + ly_ * ly_) : std::sqrt(std::fma(ly_, ly_, lx_ * lx_));
        float il = 1.0f / l2;
        float half_ap = vp.aperture / 2.0f;
        float rx = half_ap * (lx_ * il), ry = half_ap * (ly_ * il);
        V3 off = add(scale(rx, vp.cam_right), scale(ry, vp.cam_up));
        V3 from = add(vp.look_from, off);
        V3 to = sub(add(vp.upper_left, scale(ux, vp.horizontal)), scale(uy, vp.vertical));
        V3 dir = normalize<L>(sub(to, from));
        cnt.samples++;
        V3 c = ray_color<L>(job.sph, job.n, from, dir, seed, max_depth, cnt);
        if (hash) {
            q[0] += sample_fixed(c.x);
            q[1] += sample_fixed(c.y);
            q[2] += sample_fixed(c.z);
        } else {
            sum[0] += double(c.x);
            sum[1] += double(c.y);
            sum[2] += double(c.z);
        }
    }
    if (hash) {   // float accumulator in + fixed-point sum, rounded once to float
        for (int k = 0; k < 3; k++)
            sum[k] = double(job.opt.accumulate ? acc[k] : 0.0f) + double(q[k]) * 0x1p-24;
    }
    float s0 = float(sum[0]), s1 = float(sum[1]), s2 = float(sum[2]);
    acc[0] = s0; acc[1] = s1; acc[2] = s2; acc[3] = 1.0f;          // shader.rgen:63
    float spp = float(rci.samplesPerRenderCall);                   // shader.rgen:65-66
    uint8_t* o8 = job.out + texel;
    o8[0] = to_unorm8(std::sqrt(s0 / spp));
    o8[1] = to_unorm8(std::sqrt(s1 / spp));
    o8[2] = to_unorm8(std::sqrt(s2 / spp));
    o8[3] = 255;
}

// ------------------------------------------------------------------------------------
// scene.h:37-157
// ------------------------------------------------------------------------------------
inline float mt_float(std::mt19937& e, float mn, float mx) {  // scene.h:37-40
    std::uniform_real_distribution<float> dist(mn, mx);
    return dist(e);
}

rt_vec4 random_color(std::mt19937& e) {  // scene.h:47-77
    float h = std::floor(mt_float(e, 0.0f, 360.0f));
    float s = 0.75f, v = 0.45f;
    float C = s * v;
    float X = C * (1.0f - std::fabs(std::fmod(h / 60.0f, 2.0f) - 1.0f));
    float m = v - C;
    float r, g, b;
    if (h >= 0 && h < 60) { r = C; g = X; b = 0; }
    else if (h >= 60 && h < 120) { r = X; g = C; b = 0; }
    else if (h >= 120 && h < 180) { r = 0; g = C; b = X; }
    else if (h >= 180 && h < 240) { r = 0; g = X; b = C; }
    else if (h >= 240 && h < 300) { r = X; g = 0; b = C; }
    else { r = C; g = 0; b = X; }
    return rt_vec4{r + m, g + m, b + m, 1.0f};
}

void set_sphere(Sphere& s, rt_vec4 g, uint32_t mat, uint32_t tex, rt_vec4 c0, rt_vec4 c1, float attr) {
    std::memset(&s, 0, sizeof(s));
    s.geometry = g; s.materialType = mat; s.textureType = tex;
    s.colors[0] = c0; s.colors[1] = c1; s.materialSpecificAttribute = attr;
}

}  // namespace

// ====================================================================================
// exported C API (ctypes)
// ====================================================================================
extern "C" {

uint32_t orc_tea(uint32_t v0, uint32_t v1) { return tea(v0, v1); }

uint32_t orc_lcg(uint32_t seed) { return random_int(seed); }

float orc_random_float(uint32_t* seed) { return random_float(*seed); }

float orc_sinf(float x) { return rt_sinf(x); }

uint32_t orc_sample_seed_hash(uint32_t pixel_seed, uint32_t s) { return sample_seed_hash(pixel_seed, s); }

uint64_t orc_sample_fixed(float c) { return sample_fixed(c); }

void orc_viewport(const RenderCallInfo* rci, float* out18) {
    Viewport vp = make_viewport<LIT_CONTRACT>(*rci);
    const V3* vs[6] = {&vp.look_from, &vp.horizontal, &vp.vertical, &vp.upper_left, &vp.cam_up,
                       &vp.cam_right};
    for (int i = 0; i < 6; i++) { out18[3 * i] = vs[i]->x; out18[3 * i + 1] = vs[i]->y; out18[3 * i + 2] = vs[i]->z; }
}

// scene.h:79-157 generateRandomScene() with explicit t and grid half extent K (11 = reference).
int orc_generate_scene(float t, uint32_t K, Sphere* out, uint32_t capacity, uint32_t* count) {
    uint32_t need = 4u + 4u * K * K;
    if (count) *count = need;
    if (!out || capacity < need) return -1;
    const rt_vec4 zero = {0, 0, 0, 0};
    // scene.h:85-116. cos() of the float argument evaluated in double, rounded to float.
    set_sphere(out[0], rt_vec4{0.0f, -1000.0f, 1.0f, 1000.0f}, RT_DIFFUSE, RT_CHECKERED,
               rt_vec4{0.05f, 0.05f, 0.05f, 1.0f}, rt_vec4{0.95f, 0.95f, 0.95f, 1.0f}, 0.0f);
    set_sphere(out[1], rt_vec4{-4.0f, 1.0f, float(std::cos(double(2 * t))), 1.0f}, RT_DIFFUSE,
               RT_SOLID, rt_vec4{0.6f, 0.3f, 0.1f, 1.0f}, zero, 0.0f);
    set_sphere(out[2], rt_vec4{4.0f, 1.0f, float(std::cos(double(3 * t))), 1.0f}, RT_METAL,
               RT_SOLID, rt_vec4{0.8f, 0.8f, 0.8f, 1.0f}, zero, 0.0f);
    set_sphere(out[3], rt_vec4{0.0f, 1.0f, float(std::cos(double(t))), 1.0f}, RT_REFRACTIVE,
               RT_SOLID, rt_vec4{1.0f, 1.0f, 1.0f, 1.0f}, zero, 1.5f);
    uint32_t idx = 4;
    std::mt19937 engine{};  // scene.h:120, default seed 5489
    int k = int(K);
    for (int a = -k; a < k; a++) {
        for (int b = -k; b < k; b++) {
            // scene.h:124-125: g++ evaluates the vec4 constructor's arguments right to left,
            // so the z draw precedes the x draw (pinned by the FNV fixture).
            float rz = mt_float(engine, 0.0f, 1.0f);
            float rx = mt_float(engine, 0.0f, 1.0f);
            rt_vec4 g = {float(a) + 0.9f * rx, 0.2f, float(b) + 0.9f * rz, 0.2f};
            float p = mt_float(engine, 0.0f, 1.0f);
            if (double(p) < 0.7) {            // float promoted to double (scene.h:129)
                rt_vec4 c = random_color(engine);
                set_sphere(out[idx], g, RT_DIFFUSE, RT_SOLID, c, zero, 0.0f);
            } else if (double(p) < 0.85) {    // scene.h:136
                // scene.h:139-140, arguments right to left: blue, green, red.
                float cb = mt_float(engine, 0.5f, 1.0f);
                float cg = mt_float(engine, 0.5f, 1.0f);
                float cr = mt_float(engine, 0.5f, 1.0f);
                set_sphere(out[idx], g, RT_METAL, RT_SOLID, rt_vec4{cr, cg, cb, 1.0f}, zero, 0.0f);
            } else {
                set_sphere(out[idx], g, RT_REFRACTIVE, RT_SOLID, rt_vec4{1.0f, 1.0f, 1.0f, 1.0f},
                           zero, 1.5f);
            }
            idx++;
        }
    }
    return 0;
}

// One frame of the hot path on `threads` CPU threads (0 = hardware concurrency).
// Band = band_w x band_h launch ids; rows (optional) maps band row -> global row.
int orc_render(const Sphere* spheres, uint32_t n, const RenderCallInfo* rci, const uint32_t* rows,
               uint32_t band_w, uint32_t band_h, const rt_options* opt, float* accum,
               uint8_t* out, uint64_t* stats3, int threads) {
    if ((!spheres && n) || !rci || !accum || !out) return -1;
    RenderJob job;
    job.sph = spheres; job.n = n; job.rci = rci; job.rows = rows;
    job.band_w = band_w; job.band_h = band_h;
    std::memset(&job.opt, 0, sizeof(job.opt));
    if (opt) job.opt = *opt;
    const uint32_t lit = job.opt.reserved[1];   // arithmetic form (LIT_*), oracle only
    if (lit > LIT_ALL) return -1;
    job.vp = lit == LIT_ALL ? make_viewport<LIT_ALL>(*rci) : make_viewport<LIT_CONTRACT>(*rci);
    job.accum = accum; job.out = out;
    if (!job.opt.accumulate) std::memset(accum, 0, size_t(band_w) * band_h * 4 * sizeof(float));
    unsigned nt = threads > 0 ? unsigned(threads) : std::max(1u, std::thread::hardware_concurrency());
    // pixels are independent: threads take runs of up to 8 pixels of a row, so narrow bands (a
    // few rows of a high-spp frame) still use every thread
    const uint32_t runs_per_row = (band_w + 7u) / 8u;
    const uint64_t n_runs = uint64_t(runs_per_row) * band_h;
    std::atomic<uint64_t> next_run{0};
    std::vector<Counters> cnts(nt);
    auto worker = [&](unsigned tid) {
        for (;;) {
            const uint64_t r = next_run.fetch_add(1);
            if (r >= n_runs) break;
            const uint32_t y = uint32_t(r / runs_per_row), x0 = uint32_t(r % runs_per_row) * 8u;
            for (uint32_t x = x0; x < std::min(band_w, x0 + 8u); x++) {
                if (lit == LIT_CONTRACT) render_pixel<LIT_CONTRACT>(job, x, y, cnts[tid]);
                else if (lit == LIT_RINT) render_pixel<LIT_RINT>(job, x, y, cnts[tid]);
                else render_pixel<LIT_ALL>(job, x, y, cnts[tid]);
            }
        }
    };
    std::vector<std::thread> pool;
    for (unsigned i = 1; i < nt; i++) pool.emplace_back(worker, i);
    worker(0);
    for (auto& th : pool) th.join();
    if (stats3) {
        stats3[0] = stats3[1] = stats3[2] = 0;
        for (auto& c : cnts) { stats3[0] += c.segments; stats3[1] += c.samples; stats3[2] += c.sphere_tests; }
    }
    return 0;
}

// Tonemap of an already summed accumulator (checker of rt_resolve_rgba8): the same conversion
// render_pixel applies to a pixel's sum (shader.rgen:65-66).
int orc_resolve(const float* acc, uint64_t n_texels, uint32_t spp, uint8_t* out) {
    if (!acc || !out || !spp) return 1;
    const float fs = float(spp);
    for (uint64_t i = 0; i < n_texels; i++) {
        for (int c = 0; c < 3; c++) out[4 * i + c] = to_unorm8(std::sqrt(acc[4 * i + c] / fs));
        out[4 * i + 3] = 255;
    }
    return 0;
}

}  // extern "C"
