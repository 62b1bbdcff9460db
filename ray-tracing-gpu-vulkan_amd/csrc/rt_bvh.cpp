// rt_bvh.cpp — LBVH over the scene's spheres (replaces the driver BLAS/TLAS built at
// src/vulkan.h:395-554 from the per-sphere AABBs of src/ray_trace.cpp:583-599).
//
// Layout (rt_internal.h BvhNode): nodes in depth-first order with escape links, so the device
// walk needs no stack: hit inner node -> index + 1, miss or leaf done -> escape.
//
// Construction (Karras-style binary radix tree over Morton codes):
//   1. "big" spheres (radius > 2 x median radius; at most 64, largest first) are kept out of the
//      tree and tested exhaustively: the reference ground sphere (r = 1000) would otherwise
//      inflate every ancestor box up to the root.
//   2. small-sphere centers quantised to 10 bits per axis inside their bounds, 30-bit Morton
//      codes, stable sort by (code, index).
//   3. recursive split at the highest differing bit of (Morton code, sorted position) — the
//      binary radix tree of Karras 2012, which rt_build.hip constructs in parallel — cut
//      at subtrees of at most kLeafMax spheres, which become leaves stored in kLeafMax slots
//      (dummy-padded) so the device issues a leaf's four loads together.
//   4. node bounds = exact float min/max of the member spheres' AABBs (center -/+ radius), so
//      every node box contains its spheres' AABBs bit-exactly (the traversal's exactness
//      argument, DESIGN.md §4.3, needs this).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_bvh.h"

namespace rt {

namespace {

constexpr uint32_t kLeafMax = 4;
#ifndef RT_BIG_FACTOR
#define RT_BIG_FACTOR 2.0f   // "big" = radius above this multiple of the median (A/B knob)
#endif

inline uint32_t expand_bits(uint32_t v) {  // 10 bits -> every third bit of 30
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

struct Prim {
    uint32_t code;
    uint32_t id;
};

// Host SAH builder knobs (A/B experiments; defaults are the measured best).
struct SahKnobs {
    bool classic = false;   // cost = area x spheres (else area x leaves needed)
    bool sweep = false;     // exact sweep over sorted centroids for ranges <= 4096 (else 32 bins)
    int order = 0;          // child order: 0 split order, 1 larger-area child first, 2 smaller first
};

struct Builder {
    const Sphere* sph;
    std::vector<Prim>& prims;
    HostBvh& out;
    bool sah;
    SahKnobs knobs;

    void bounds(uint32_t lo, uint32_t hi, float* bmin, float* bmax) const {
        bmin[0] = bmin[1] = bmin[2] = INFINITY;
        bmax[0] = bmax[1] = bmax[2] = -INFINITY;
        for (uint32_t i = lo; i < hi; i++) {
            const rt_vec4& g = sph[prims[i].id].geometry;
            const float c[3] = {g.x, g.y, g.z};
            for (int k = 0; k < 3; k++) {
                bmin[k] = std::min(bmin[k], c[k] - g.w);   // the sphere's AABB, exactly as the
                bmax[k] = std::max(bmax[k], c[k] + g.w);   // traversal test computes it
            }
        }
    }

    // Common-prefix length of the keys at sorted positions i and j, each key augmented by its
    // position (Karras 2012, duplicate codes): the GPU builder (rt_build.hip) uses the same rule,
    // so both emit the identical tree.
    int delta(uint32_t i, uint32_t j) const {
        const uint32_t a = prims[i].code, b = prims[j].code;
        return a == b ? 32 + __builtin_clz(i ^ j) : __builtin_clz(a ^ b);
    }

    uint32_t split(uint32_t lo, uint32_t hi) const {  // [lo, hi), hi - lo >= 2
        const int common = delta(lo, hi - 1);
        uint32_t s = lo, step = hi - 1 - lo;
        do {  // binary search for the last index sharing more than `common` prefix bits with lo
            step = (step + 1) >> 1;
            const uint32_t ns = s + step;
            if (ns < hi - 1 && delta(lo, ns) > common) s = ns;
        } while (step > 1);
        return s + 1;
    }

    // Exact sweep variant of split_sah (A/B knob "sweep"): every split position along each axis
    // of the centroid-sorted range.
    uint32_t split_sweep(uint32_t lo, uint32_t hi) {
        auto area = [](const float* l, const float* h) {
            const double ex = double(h[0]) - l[0], ey = double(h[1]) - l[1], ez = double(h[2]) - l[2];
            return ex * ey + ey * ez + ez * ex;
        };
        const uint32_t n = hi - lo;
        double best_cost = INFINITY;
        int best_axis = -1;
        uint32_t best_s = 0;
        std::vector<Prim> tmp(prims.begin() + lo, prims.begin() + hi);
        std::vector<double> right(n);
        for (int k = 0; k < 3; k++) {
            auto key = [&](const Prim& p) {
                const rt_vec4& g = sph[p.id].geometry;
                return k == 0 ? g.x : k == 1 ? g.y : g.z;
            };
            std::stable_sort(tmp.begin(), tmp.end(), [&](const Prim& a, const Prim& b) { return key(a) < key(b); });
            float rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (uint32_t i = n; i-- > 1;) {
                const rt_vec4& g = sph[tmp[i].id].geometry;
                const float c[3] = {g.x, g.y, g.z};
                for (int j = 0; j < 3; j++) { rl[j] = std::min(rl[j], c[j] - g.w); rh[j] = std::max(rh[j], c[j] + g.w); }
                right[i] = area(rl, rh);
            }
            float ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (uint32_t i = 0; i + 1 < n; i++) {   // left = [0, i], right = [i + 1, n)
                const rt_vec4& g = sph[tmp[i].id].geometry;
                const float c[3] = {g.x, g.y, g.z};
                for (int j = 0; j < 3; j++) { ll[j] = std::min(ll[j], c[j] - g.w); lh[j] = std::max(lh[j], c[j] + g.w); }
                const uint32_t nl = i + 1, nr = n - nl;
                const double cost = knobs.classic ? area(ll, lh) * nl + right[i + 1] * nr
                                                  : area(ll, lh) * ((nl + kLeafMax - 1) / kLeafMax) +
                                                        right[i + 1] * ((nr + kLeafMax - 1) / kLeafMax);
                if (cost < best_cost) { best_cost = cost; best_axis = k; best_s = nl; }
            }
        }
        if (best_axis < 0) return (lo + hi) / 2;
        auto key = [&](const Prim& p) {
            const rt_vec4& g = sph[p.id].geometry;
            return best_axis == 0 ? g.x : best_axis == 1 ? g.y : g.z;
        };
        std::stable_sort(prims.begin() + lo, prims.begin() + hi, [&](const Prim& a, const Prim& b) { return key(a) < key(b); });
        return lo + best_s;
    }

    // Binned surface-area split of [lo, hi) (hi - lo > kLeafMax): 32 centroid bins per axis, cost
    // = sum over both sides of area x leaves needed (a leaf costs the same for 1..4 spheres, the
    // device always tests four slots). Reorders prims[lo, hi) and returns the split index;
    // coincident centroids fall back to a split by count.
    uint32_t split_sah(uint32_t lo, uint32_t hi) {
        if (knobs.sweep && hi - lo <= 4096) return split_sweep(lo, hi);
        constexpr int kBins = 32;
        float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = lo; i < hi; i++) {
            const rt_vec4& g = sph[prims[i].id].geometry;
            const float c[3] = {g.x, g.y, g.z};
            for (int k = 0; k < 3; k++) { cmin[k] = std::min(cmin[k], c[k]); cmax[k] = std::max(cmax[k], c[k]); }
        }
        auto area = [](const float* l, const float* h) {
            const double ex = double(h[0]) - l[0], ey = double(h[1]) - l[1], ez = double(h[2]) - l[2];
            return ex * ey + ey * ez + ez * ex;
        };
        auto bin_of = [&](int k, float c) {
            const float ext = cmax[k] - cmin[k];
            int b = int(double(c - cmin[k]) / ext * kBins);
            return std::min(std::max(b, 0), kBins - 1);
        };
        double best_cost = INFINITY;
        int best_axis = -1, best_plane = 0;
        for (int k = 0; k < 3; k++) {
            if (!(cmax[k] > cmin[k])) continue;
            float bl[kBins][3], bh[kBins][3];
            uint32_t cnt[kBins] = {};
            for (int b = 0; b < kBins; b++)
                for (int j = 0; j < 3; j++) { bl[b][j] = INFINITY; bh[b][j] = -INFINITY; }
            for (uint32_t i = lo; i < hi; i++) {
                const rt_vec4& g = sph[prims[i].id].geometry;
                const float c[3] = {g.x, g.y, g.z};
                const int b = bin_of(k, c[k]);
                cnt[b]++;
                for (int j = 0; j < 3; j++) {
                    bl[b][j] = std::min(bl[b][j], c[j] - g.w);
                    bh[b][j] = std::max(bh[b][j], c[j] + g.w);
                }
            }
            double right_area[kBins];
            uint32_t right_cnt[kBins];
            float rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t rc = 0;
            for (int b = kBins - 1; b > 0; b--) {
                rc += cnt[b];
                for (int j = 0; j < 3; j++) { rl[j] = std::min(rl[j], bl[b][j]); rh[j] = std::max(rh[j], bh[b][j]); }
                right_area[b] = rc ? area(rl, rh) : 0.0;
                right_cnt[b] = rc;
            }
            float ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t lc = 0;
            for (int b = 0; b + 1 < kBins; b++) {   // plane between bin b and b + 1
                lc += cnt[b];
                for (int j = 0; j < 3; j++) { ll[j] = std::min(ll[j], bl[b][j]); lh[j] = std::max(lh[j], bh[b][j]); }
                const uint32_t rcnt = right_cnt[b + 1];
                if (lc == 0 || rcnt == 0) continue;
                const double cost = knobs.classic
                                         ? area(ll, lh) * lc + right_area[b + 1] * rcnt
                                         : area(ll, lh) * ((lc + kLeafMax - 1) / kLeafMax) +
                                               right_area[b + 1] * ((rcnt + kLeafMax - 1) / kLeafMax);
                if (cost < best_cost) { best_cost = cost; best_axis = k; best_plane = b; }
            }
        }
        if (best_axis < 0) {   // all centroids coincide on every axis: split by count
            return (lo + hi) / 2;
        }
        const auto mid = std::stable_partition(prims.begin() + lo, prims.begin() + hi, [&](const Prim& p) {
            const rt_vec4& g = sph[p.id].geometry;
            const float c = best_axis == 0 ? g.x : best_axis == 1 ? g.y : g.z;
            return bin_of(best_axis, c) <= best_plane;
        });
        return uint32_t(mid - prims.begin());
    }

    // Emits the subtree [lo, hi) as escape-link nodes in depth-first order.
    void build(uint32_t lo, uint32_t hi) {
        const uint32_t me = uint32_t(out.nodes.size());
        out.nodes.push_back(BvhNode{});
        float bmin[3], bmax[3];
        bounds(lo, hi, bmin, bmax);
        BvhNode n;
        n.lox = bmin[0]; n.loy = bmin[1]; n.loz = bmin[2];
        n.hix = bmax[0]; n.hiy = bmax[1]; n.hiz = bmax[2];
        if (hi - lo <= kLeafMax) {
            const uint32_t first = uint32_t(out.leaf_geom.size());
            for (uint32_t i = lo; i < lo + kLeafMax; i++) {
                if (i < hi) {
                    const rt_vec4& g = sph[prims[i].id].geometry;
                    out.leaf_geom.push_back(GeomRec{g.x, g.y, g.z, g.w});   // radius, not r^2
                    out.leaf_ids.push_back(prims[i].id);
                } else {   // dummy: 1e19 below the scene, radius 0 -> never reports
                    out.leaf_geom.push_back(GeomRec{0.0f, -1e19f, 0.0f, 0.0f});
                    out.leaf_ids.push_back(0xffffffffu);
                }
            }
            n.first_count = (first << 4) | (hi - lo);
        } else {
            uint32_t s = sah ? split_sah(lo, hi) : split(lo, hi);
            if (knobs.order) {   // put the larger (order 1) / smaller (order 2) child first
                float la[3], ha[3], lb[3], hb[3];
                bounds(lo, s, la, ha);
                bounds(s, hi, lb, hb);
                auto area = [](const float* l, const float* h) {
                    const double ex = double(h[0]) - l[0], ey = double(h[1]) - l[1], ez = double(h[2]) - l[2];
                    return ex * ey + ey * ez + ez * ex;
                };
                const double a0 = area(la, ha), a1 = area(lb, hb);
                if ((knobs.order == 1 && a1 > a0) || (knobs.order == 2 && a1 < a0)) {
                    std::rotate(prims.begin() + lo, prims.begin() + s, prims.begin() + hi);
                    s = lo + (hi - s);
                }
            }
            build(lo, s);
            build(s, hi);
            n.first_count = 0;
        }
        n.escape = uint32_t(out.nodes.size());  // first node after this subtree
        out.nodes[me] = n;
    }
};

}  // namespace

void build_lbvh_host(const Sphere* sph, uint32_t n, HostBvh& out, bool sah, uint32_t sah_knobs) {
    out = HostBvh{};
    if (n == 0) return;
    if (n >= (1u << 27)) return;   // leaf references hold 28-bit slot indices
    // 1. big spheres
    std::vector<float> radii(n);
    for (uint32_t i = 0; i < n; i++) radii[i] = sph[i].geometry.w;
    std::vector<float> sorted = radii;
    std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
    const float median = sorted[n / 2];
    std::vector<uint32_t> big;
    for (uint32_t i = 0; i < n; i++)
        if (radii[i] > RT_BIG_FACTOR * median) big.push_back(i);
    if (big.size() > kBigMax) {
        std::stable_sort(big.begin(), big.end(), [&](uint32_t a, uint32_t b) { return radii[a] > radii[b]; });
        big.resize(kBigMax);
    }
    std::sort(big.begin(), big.end());
    out.big_ids = big;
    std::vector<char> is_big(n, 0);
    for (uint32_t i : big) is_big[i] = 1;
    // 2. Morton codes of the small spheres
    std::vector<Prim> prims;
    prims.reserve(n - big.size());
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < n; i++) {
        if (is_big[i]) continue;
        const float c[3] = {sph[i].geometry.x, sph[i].geometry.y, sph[i].geometry.z};
        for (int k = 0; k < 3; k++) { cmin[k] = std::min(cmin[k], c[k]); cmax[k] = std::max(cmax[k], c[k]); }
        out.small_rmax = std::max(out.small_rmax, radii[i]);
        out.small_rmin = std::min(out.small_rmin, radii[i]);   // NaN radii keep INFINITY: slack off
        prims.push_back(Prim{0, i});
    }
    if (prims.empty()) return;
    for (Prim& p : prims) {
        const float c[3] = {sph[p.id].geometry.x, sph[p.id].geometry.y, sph[p.id].geometry.z};
        uint32_t q[3];
        for (int k = 0; k < 3; k++) {
            const float ext = cmax[k] - cmin[k];
            float f = ext > 0.0f ? (c[k] - cmin[k]) / ext : 0.5f;
            f = std::min(std::max(f, 0.0f), 1.0f);
            q[k] = std::min(1023u, uint32_t(f * 1024.0f));
        }
        p.code = (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
    }
    std::stable_sort(prims.begin(), prims.end(), [](const Prim& a, const Prim& b) { return a.code < b.code; });
    // 3-4. hierarchy in depth-first order
    out.nodes.reserve(2 * prims.size());
    SahKnobs knobs;
    knobs.classic = (sah_knobs & 1u) != 0;
    knobs.sweep = (sah_knobs & 2u) != 0;
    knobs.order = int((sah_knobs >> 2) & 3u);
    Builder b{sph, prims, out, sah, knobs};
    b.build(0, uint32_t(prims.size()));
    for (BvhNode& nd : out.nodes)
        if (nd.escape >= out.nodes.size()) nd.escape = 0xffffffffu;
}

}  // namespace rt
