// rt_build.hip — parallel LBVH build / refit on the GPU (gfx950).
//
// Replaces the reference's per-frame acceleration-structure rebuild (src/vulkan.h:395-554 BLAS +
// TLAS from the per-sphere AABBs of src/ray_trace.cpp:583-599, rebuilt every frame at
// src/vulkan.h:1020-1059). It emits exactly the tree the host builder (rt_bvh.cpp, Morton form)
// emits from the same spheres, so tests compare the two array for array:
//
//   prep      Sphere (80-B std140, HBM) -> GeomRec / radius / MatRec records, brute-force pad
//             records, scene radius R (max |center| + |r|, exact max via ordered-int atomics)
//   sort 1    radii, descending, stable (hipCUB radix sort): median and the 64 largest "big"
//             spheres with the host's tie order (stable_sort by radius over index order)
//   select    one wave: threshold 2 x median, big ids ascending, is_big flags
//   reduce    centroid bounds and largest radius of the small spheres
//   morton    30-bit codes with the host's float ops; big spheres get key 0xffffffff, so one
//             stable sort of all n puts the small spheres first in (code, index) order and no
//             count has to come back to the host
//   sort 2    (key, index) pairs, stable (hipCUB)
//   karras    binary radix tree over the keys augmented by their position (Karras 2012,
//             "Maximizing parallelism in the construction of BVHs, octrees, and k-d trees"):
//             one thread per inner node finds its range and split by binary search
//   bottomup  one thread per leaf climbs to the root; the second arrival at a node (agent-scope
//             acq_rel counter: the 8 XCD L2s are not coherent) unions its children's boxes
//             (exact float min/max) and counts emitted nodes / leaves of the cut tree (subtrees of
//             <= 4 spheres become leaves)
//   emit      one thread per radix-tree node that survives the cut: depth-first position and leaf
//             index by climbing to the root, then the padded + raw 32-B node (escape link) and
//             its 4 dummy-padded leaf slots
//
// Refit (per-frame animation, src/scene.h:94-111 moves spheres with t): prep + reduce +
// bottomup + emit over the stored order and topology.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "rt_build.h"

namespace rt {

namespace {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kPrim = 0x80000000u;   // radix-tree reference: leaf (sorted position)
constexpr uint32_t kLeafMax = 4;
constexpr uint32_t kEnd = 0xffffffffu;
constexpr uint32_t kMaxDepth = 128;   // loop bound: the radix tree is at most 59 levels deep

__device__ __forceinline__ uint32_t f2o(float f) {   // order-preserving float -> uint
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, s));
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, s));
    return v;
}

__global__ void k_init(BuildSummary* S, bool refit) {
    if (threadIdx.x) return;
    if (!refit) {
        S->n_big = 0; S->n_small = 0; S->n_nodes = 0; S->n_leaf_slots = 0;
        for (int k = 0; k < 3; k++) { S->cmin_o[k] = f2o(INFINITY); S->cmax_o[k] = f2o(-INFINITY); }
    }
    S->rmax_o = f2o(0.0f);
    S->rmin_o = f2o(INFINITY);
    S->colour_out_of_range = 0u;
    S->R_o = f2o(0.0f);
}

// Records (rt_api.cpp conventions: rr = r * r rounded once, shader.rint:48), sort keys, R.
__global__ void __launch_bounds__(kBlock) k_prep(const Sphere* __restrict__ sph, uint32_t n, uint32_t n_geom,
                                                 GeomRec* geom, float* radius, MatRec* mat, float* rkeys,
                                                 uint32_t* ids, BuildSummary* S) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    uint32_t Ro = f2o(0.0f);
    if (i < n) {
        const Sphere s = sph[i];
        const float x = s.geometry.x, y = s.geometry.y, z = s.geometry.z, r = s.geometry.w;
        geom[i] = GeomRec{x, y, z, r * r};
        radius[i] = r;
        mat[i] = make_mat(s.colors[0].x, s.colors[0].y, s.colors[0].z, s.materialSpecificAttribute,
                          s.colors[1].x, s.colors[1].y, s.colors[1].z, s.materialType, s.textureType);
        if (rkeys) { rkeys[i] = r; ids[i] = i; }
        if (!colours_in_unit(s)) atomicOr(&S->colour_out_of_range, 1u);
        Ro = f2o(__builtin_sqrtf(x * x + y * y + z * z) + __builtin_fabsf(r));
    } else if (i < n_geom) {   // brute-force pad record: never hit (rt_api.cpp)
        geom[i] = GeomRec{0.0f, 1e19f, 0.0f, -1e38f};
    }
    Ro = wave_max(Ro);
    if (__lane_id() == 0) atomicMax(&S->R_o, Ro);
}

// One wave: threshold and the big set from the descending radius order.
__global__ void k_select(const float* __restrict__ rdesc, const uint32_t* __restrict__ idesc, uint32_t n,
                         uint32_t* big_ids, uint8_t* is_big, BuildSummary* S) {
    const uint32_t lane = threadIdx.x;   // 64 lanes
    const float median = rdesc[n - 1 - n / 2];   // ascending[n / 2] (host nth_element)
    const float thr = 2.0f * median;
    const bool big = lane < n && lane < kBigMax && rdesc[lane] > thr;
    const uint64_t mask = __ballot(big);
    const uint32_t nb = __popcll(mask);   // descending order: the big ones are a prefix
    const uint32_t id = big ? idesc[lane] : kEnd;
    uint32_t rank = 0;
    for (uint32_t j = 0; j < nb; j++) {
        const uint32_t other = (uint32_t)__shfl((int)id, (int)j);
        rank += other < id ? 1u : 0u;
    }
    if (big) {
        big_ids[rank] = id;
        is_big[id] = 1;
    }
    if (lane == 0) {
        S->n_big = nb;
        S->n_small = n - nb;
    }
}

// Centroid bounds (Morton frame) and largest radius of the spheres in the tree.
__global__ void __launch_bounds__(kBlock) k_reduce(const Sphere* __restrict__ sph, uint32_t n,
                                                   const uint8_t* __restrict__ is_big, bool refit,
                                                   BuildSummary* S) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const bool small = i < n && !is_big[i];
    float c[3] = {0.0f, 0.0f, 0.0f};
    float r = 0.0f;
    if (small) {
        const rt_vec4 g = sph[i].geometry;
        c[0] = g.x; c[1] = g.y; c[2] = g.z; r = g.w;
    }
    const uint32_t ro = wave_max(small ? f2o(r) : f2o(0.0f));
    if (__lane_id() == 0) atomicMax(&S->rmax_o, ro);
    const uint32_t rmo = wave_min(small ? f2o(r) : f2o(INFINITY));
    if (__lane_id() == 0) atomicMin(&S->rmin_o, rmo);
    if (refit) return;   // the Morton frame belongs to the stored topology
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t mn = wave_min(small ? f2o(c[k]) : f2o(INFINITY));
        const uint32_t mx = wave_max(small ? f2o(c[k]) : f2o(-INFINITY));
        if (__lane_id() == 0) {
            atomicMin(&S->cmin_o[k], mn);
            atomicMax(&S->cmax_o[k], mx);
        }
    }
}

__device__ __forceinline__ float o2f(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// rt_bvh.cpp step 2, the same float operations (division correctly rounded, no contraction).
__global__ void __launch_bounds__(kBlock) k_morton(const Sphere* __restrict__ sph, uint32_t n,
                                                   const uint8_t* __restrict__ is_big,
                                                   const BuildSummary* __restrict__ S, uint32_t* keys,
                                                   uint32_t* ids) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    ids[i] = i;
    if (is_big[i]) { keys[i] = kEnd; return; }
    const rt_vec4 g = sph[i].geometry;
    const float c[3] = {g.x, g.y, g.z};
    uint32_t q[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float cmin = o2f(S->cmin_o[k]), cmax = o2f(S->cmax_o[k]);
        const float ext = cmax - cmin;
        float f = ext > 0.0f ? (c[k] - cmin) / ext : 0.5f;
        f = fminf(fmaxf(f, 0.0f), 1.0f);
        q[k] = min(1023u, (uint32_t)(f * 1024.0f));
    }
    keys[i] = (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
}

// Common prefix of the position-augmented keys at i and j (-1 outside [0, m)).
__device__ __forceinline__ int kdelta(const uint32_t* __restrict__ keys, int m, int i, int j) {
    if (j < 0 || j >= m) return -1;
    const uint32_t a = keys[i], b = keys[j];
    return a == b ? 32 + __clz(i ^ j) : __clz((int)(a ^ b));
}

// Karras 2012, Fig. 4: inner node i of the radix tree over m sorted keys.
__global__ void __launch_bounds__(kBlock) k_karras(const uint32_t* __restrict__ keys, const BuildSummary* S,
                                                   uint32_t* par_i, uint32_t* par_l, uint32_t* left,
                                                   uint32_t* right, uint32_t* lo_out, uint32_t* hi_out) {
    const int m = (int)S->n_small;
    const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
    if (i >= m - 1) return;
    const int d = kdelta(keys, m, i, i + 1) - kdelta(keys, m, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = kdelta(keys, m, i, i - d);
    int lmax = 2;
    while (kdelta(keys, m, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (kdelta(keys, m, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = kdelta(keys, m, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (kdelta(keys, m, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    const uint32_t L = (lo == gamma) ? (kPrim | (uint32_t)gamma) : (uint32_t)gamma;
    const uint32_t R = (hi == gamma + 1) ? (kPrim | (uint32_t)(gamma + 1)) : (uint32_t)(gamma + 1);
    left[i] = L;
    right[i] = R;
    lo_out[i] = (uint32_t)lo;
    hi_out[i] = (uint32_t)hi;
    if (L & kPrim) par_l[L & ~kPrim] = (uint32_t)i; else par_i[L] = (uint32_t)i;
    if (R & kPrim) par_l[R & ~kPrim] = (uint32_t)i; else par_i[R] = (uint32_t)i;
}

__device__ __forceinline__ void prim_box(const Sphere* __restrict__ sph, uint32_t id, float* b) {
    const rt_vec4 g = sph[id].geometry;
    b[0] = g.x - g.w; b[1] = g.y - g.w; b[2] = g.z - g.w;   // the sphere's AABB as the
    b[3] = g.x + g.w; b[4] = g.y + g.w; b[5] = g.z + g.w;   // traversal's gate computes it
}

__global__ void __launch_bounds__(kBlock) k_bottomup(const Sphere* __restrict__ sph,
                                                     const uint32_t* __restrict__ sids, const BuildSummary* S,
                                                     const uint32_t* __restrict__ par_i,
                                                     const uint32_t* __restrict__ par_l,
                                                     const uint32_t* __restrict__ left,
                                                     const uint32_t* __restrict__ right,
                                                     const uint32_t* __restrict__ lo,
                                                     const uint32_t* __restrict__ hi, uint32_t* flags,
                                                     float4* bnd, uint32_t* cnt, uint32_t* lcnt) {
    const uint32_t m = S->n_small;
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (m < 2 || p >= m) return;
    uint32_t node = par_l[p];
    for (uint32_t guard = 0; guard < kMaxDepth; guard++) {   // radix-tree depth <= 32 + 27
        // Release this thread's writes (the child it finished) and acquire the sibling's.
        const uint32_t old = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == 0u) return;
        float b[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
        uint32_t c = 1u, lc = 0u;
        const uint32_t ch[2] = {left[node], right[node]};
#pragma unroll
        for (int k = 0; k < 2; k++) {
            float cb[6];
            uint32_t cc, cl;
            if (ch[k] & kPrim) {
                prim_box(sph, sids[ch[k] & ~kPrim], cb);
                cc = 1u; cl = 1u;
            } else {
                const float4 a = bnd[2 * ch[k]], e = bnd[2 * ch[k] + 1];
                cb[0] = a.x; cb[1] = a.y; cb[2] = a.z; cb[3] = e.x; cb[4] = e.y; cb[5] = e.z;
                cc = cnt[ch[k]]; cl = lcnt[ch[k]];
            }
            for (int q = 0; q < 3; q++) { b[q] = fminf(b[q], cb[q]); b[q + 3] = fmaxf(b[q + 3], cb[q + 3]); }
            c += cc; lc += cl;
        }
        const bool leafy = hi[node] - lo[node] + 1u <= kLeafMax;
        bnd[2 * node] = make_float4(b[0], b[1], b[2], 0.0f);
        bnd[2 * node + 1] = make_float4(b[3], b[4], b[5], 0.0f);
        cnt[node] = leafy ? 1u : c;
        lcnt[node] = leafy ? 1u : lc;
        if (node == 0u) return;
        node = par_i[node];
    }
}

__global__ void __launch_bounds__(kBlock) k_emit(const Sphere* __restrict__ sph, const uint32_t* __restrict__ sids,
                                                 BuildSummary* S, const uint32_t* __restrict__ par_i,
                                                 const uint32_t* __restrict__ par_l,
                                                 const uint32_t* __restrict__ left,
                                                 const uint32_t* __restrict__ lo,
                                                 const uint32_t* __restrict__ hi,
                                                 const float4* __restrict__ bnd,
                                                 const uint32_t* __restrict__ cnt,
                                                 const uint32_t* __restrict__ lcnt, BvhNode* nodes,
                                                 BvhNode* nodes_raw, GeomRec* leaf_geom, uint32_t* leaf_ids) {
    const uint32_t m = S->n_small;
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (m == 0u || t >= 2u * m - 1u) return;
    const uint32_t ref = t < m - 1u ? t : (kPrim | (t - (m - 1u)));
    const uint32_t root = m == 1u ? kPrim : 0u;
    auto size_of = [&](uint32_t r) { return (r & kPrim) ? 1u : hi[r] - lo[r] + 1u; };
    auto parent_of = [&](uint32_t r) { return (r & kPrim) ? par_l[r & ~kPrim] : par_i[r]; };
    auto cnt_of = [&](uint32_t r) { return (r & kPrim) ? 1u : cnt[r]; };
    auto lcnt_of = [&](uint32_t r) { return (r & kPrim) ? 1u : lcnt[r]; };
    if (ref != root && size_of(parent_of(ref)) <= kLeafMax) return;   // inside a leaf
    uint32_t pos = 0u, lidx = 0u;
    uint32_t guard = 0;
    for (uint32_t c = ref; c != root && guard < kMaxDepth; guard++) {
        const uint32_t p = parent_of(c);
        pos += 1u;
        const uint32_t l = left[p];
        if (l != c) { pos += cnt_of(l); lidx += lcnt_of(l); }
        c = p;
    }
    const uint32_t total = cnt_of(root);
    if (t == 0u) {
        S->n_nodes = total;
        S->n_leaf_slots = kLeafMax * lcnt_of(root);
    }
    float b[6];
    if (ref & kPrim) {
        prim_box(sph, sids[ref & ~kPrim], b);
    } else {
        const float4 a = bnd[2 * ref], e = bnd[2 * ref + 1];
        b[0] = a.x; b[1] = a.y; b[2] = a.z; b[3] = e.x; b[4] = e.y; b[5] = e.z;
    }
    const uint32_t sz = size_of(ref);
    const bool leafy = sz <= kLeafMax;
    const uint32_t esc = pos + cnt_of(ref);
    BvhNode nd;
    nd.lox = b[0]; nd.loy = b[1]; nd.loz = b[2];
    nd.hix = b[3]; nd.hiy = b[4]; nd.hiz = b[5];
    nd.escape = esc >= total ? kEnd : esc;
    nd.first_count = leafy ? (((kLeafMax * lidx) << 4) | sz) : 0u;
    nodes_raw[pos] = nd;
    if (pos == 0u) {   // the root: the grid's bounds (read back with the summary)
        for (int k = 0; k < 3; k++) { S->root_lo[k] = b[k]; S->root_hi[k] = b[k + 3]; }
    }
    // padding for origins within the scene radius and a nearby camera (rt_api.cpp pad_for)
    const float pad_radius = o2f(S->R_o) * 1.01f + 100.0f;
    const float pad = 18.0f * 5.9604645e-8f * pad_radius;
    nd.lox -= pad; nd.loy -= pad; nd.loz -= pad;
    nd.hix += pad; nd.hiy += pad; nd.hiz += pad;
    nodes[pos] = nd;
    if (leafy) {
        const uint32_t first = (ref & kPrim) ? (ref & ~kPrim) : lo[ref];
        for (uint32_t k = 0; k < kLeafMax; k++) {
            const uint32_t slot = kLeafMax * lidx + k;
            if (k < sz) {
                const uint32_t id = sids[first + k];
                const rt_vec4 g = sph[id].geometry;
                leaf_geom[slot] = GeomRec{g.x, g.y, g.z, g.w};   // radius, not r^2
                leaf_ids[slot] = id;
            } else {   // dummy: 1e19 below the scene, radius 0 -> never reports
                leaf_geom[slot] = GeomRec{0.0f, -1e19f, 0.0f, 0.0f};
                leaf_ids[slot] = kEnd;
            }
        }
    }
}

__global__ void __launch_bounds__(kBlock) k_repad(const BvhNode* __restrict__ raw, BvhNode* nodes,
                                                  uint32_t n, float pad) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    BvhNode nd = raw[i];
    nd.lox -= pad; nd.loy -= pad; nd.loz -= pad;
    nd.hix += pad; nd.hiy += pad; nd.hiz += pad;
    nodes[i] = nd;
}

// Top treelet (ACCEL_LBVH_TOP, layout in rt_internal.h) of an escape-link tree in depth-first
// order: one block gathers the nodes of depth <= kTreeletDepth level by level (children of inner
// node i: i + 1 and the escape of i + 1), sorts them by node index (bitonic, in LDS) so they keep
// the tree's depth-first order, and writes each in AB layout with its links as treelet ranks (the
// escape of a node is never deeper than the node, so it is in the treelet too).
constexpr uint32_t kTreeletThreads = 1024;
__global__ void __launch_bounds__(kTreeletThreads) k_treelet(const BvhNode* __restrict__ nodes, uint32_t n_nodes,
                                                             float4* __restrict__ out, uint32_t* out_count) {
    constexpr uint32_t kSort = 4096;   // >= kTreeletCap, a power of two
    static_assert(kSort >= kTreeletCap, "treelet sort capacity");
    __shared__ unsigned long long key[kSort];   // node index << 8 | depth
    __shared__ uint32_t count;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        count = n_nodes ? 1u : 0u;
        key[0] = 0ull;
    }
    __syncthreads();
    uint32_t lb = 0, le = count;
    for (uint32_t d = 0; d < kTreeletDepth && lb < le; ++d) {
        for (uint32_t t = lb + tid; t < le; t += kTreeletThreads) {
            const uint32_t i = uint32_t(key[t] >> 8);
            if (nodes[i].first_count == 0u) {   // inner: both children, one level deeper
                const uint32_t s = atomicAdd(&count, 2u);
                key[s] = (uint64_t(i + 1u) << 8) | (d + 1u);
                key[s + 1] = (uint64_t(nodes[i + 1].escape) << 8) | (d + 1u);
            }
        }
        __syncthreads();
        lb = le;
        le = count;
        __syncthreads();
    }
    const uint32_t n = count;
    for (uint32_t t = n + tid; t < kSort; t += kTreeletThreads) key[t] = ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= kSort; k <<= 1) {   // bitonic sort, ascending
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = tid; t < kSort; t += kTreeletThreads) {
                const uint32_t p = t ^ j;
                if (p > t) {
                    const unsigned long long a = key[t], b = key[p];
                    if (((t & k) == 0) == (a > b)) { key[t] = b; key[p] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t t = tid; t < n; t += kTreeletThreads) {
        const uint32_t i = uint32_t(key[t] >> 8), dep = uint32_t(key[t] & 255u);
        const BvhNode nd = nodes[i];
        uint32_t miss = kEnd;
        if (nd.escape != kEnd) {   // rank of the escape: binary search over the sorted indices
            uint32_t lo = 0, hi = n;
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (uint32_t(key[m] >> 8) < nd.escape) lo = m + 1; else hi = m;
            }
            if (lo < n && uint32_t(key[lo] >> 8) == nd.escape) miss = lo;
        }
        const uint32_t hit = nd.first_count ? (0x80000000u | nd.first_count)
                                            : (dep == kTreeletDepth ? (0xC0000000u | i) : t + 1u);
        out[2 * t] = make_float4(nd.lox, nd.loy, nd.hix, nd.hiy);
        out[2 * t + 1] = make_float4(nd.loz, nd.hiz, __uint_as_float(miss), __uint_as_float(hit));
    }
    if (tid == 0) *out_count = n;
}

// Uniform grid (rt_grid.h) over the small spheres of a device build: the cell range of sphere i's
// AABB widened by the margin (the host builder's arithmetic), counted, then filled through a scan.
__device__ __forceinline__ void grid_range(const GridInfo& g, int k, float c, float r, uint32_t& a, uint32_t& b) {
    const double x0 = (double(c - r) - g.margin - g.gmin[k]) / g.cs[k];
    const double x1 = (double(c + r) + g.margin - g.gmin[k]) / g.cs[k];
    a = uint32_t(fmin(double(g.n[k] - 1), fmax(0.0, floor(x0))));
    b = uint32_t(fmin(double(g.n[k] - 1), fmax(0.0, floor(x1))));
}

template <bool FILL>
__global__ void __launch_bounds__(kBlock) k_grid_refs(const Sphere* __restrict__ sph, uint32_t n,
                                                      const uint8_t* __restrict__ is_big, const GridInfo g,
                                                      uint32_t* __restrict__ cnt, GeomRec* __restrict__ rec,
                                                      uint32_t* __restrict__ ids) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || is_big[i]) return;
    const rt_vec4 s = sph[i].geometry;
    uint32_t a[3], b[3];
    grid_range(g, 0, s.x, s.w, a[0], b[0]);
    grid_range(g, 1, s.y, s.w, a[1], b[1]);
    grid_range(g, 2, s.z, s.w, a[2], b[2]);
    for (uint32_t z = a[2]; z <= b[2]; z++)
        for (uint32_t y = a[1]; y <= b[1]; y++)
            for (uint32_t x = a[0]; x <= b[0]; x++) {
                const uint32_t c = (z * g.n[1] + y) * g.n[0] + x;
                const uint32_t j = atomicAdd(&cnt[c], 1u);   // FILL: cnt holds each cell's next slot
                if (FILL) {
                    rec[j] = GeomRec{s.x, s.y, s.z, s.w * s.w};   // r^2 (rt_grid.h)
                    ids[j] = i;
                }
            }
}

__global__ void __launch_bounds__(kBlock) k_iota(uint32_t* v, uint32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) v[i] = i;
}

inline uint32_t blocks(uint32_t n) { return (n + kBlock - 1) / kBlock; }

template <typename T>
hipError_t alloc(T** p, size_t count) {
    return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T) + 16);
}

}  // namespace

float summary_float(uint32_t o) {
    const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

void build_release(BuildWorkspace& ws) {
    void* ptrs[] = {ws.rkeys, ws.rkeys_s, ws.ids, ws.ids_s, ws.keys, ws.keys_s, ws.sids, ws.is_big,
                    ws.par_i, ws.par_l, ws.left, ws.right, ws.lo, ws.hi, ws.flags, ws.cnt, ws.lcnt,
                    ws.bnd, ws.tmp, ws.S};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    ws = BuildWorkspace{};
}

hipError_t build_reserve(BuildWorkspace& ws, uint32_t n) {
    if (n <= ws.cap && ws.S) return hipSuccess;
    build_release(ws);
    const uint32_t c = n < 64u ? 64u : n;
    hipError_t e = hipSuccess;
#define RT_ALLOC(p, k) if (e == hipSuccess) e = alloc(&ws.p, k)
    RT_ALLOC(rkeys, c); RT_ALLOC(rkeys_s, c); RT_ALLOC(ids, c); RT_ALLOC(ids_s, c);
    RT_ALLOC(keys, c); RT_ALLOC(keys_s, c); RT_ALLOC(sids, c); RT_ALLOC(is_big, c);
    RT_ALLOC(par_i, c); RT_ALLOC(par_l, c); RT_ALLOC(left, c); RT_ALLOC(right, c);
    RT_ALLOC(lo, c); RT_ALLOC(hi, c); RT_ALLOC(flags, c); RT_ALLOC(cnt, c); RT_ALLOC(lcnt, c);
    RT_ALLOC(bnd, 2 * size_t(c)); RT_ALLOC(S, 1);
#undef RT_ALLOC
    if (e == hipSuccess) {
        size_t b1 = 0, b2 = 0;
        e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, b1, ws.rkeys, ws.rkeys_s, ws.ids, ws.ids_s,
                                                         int(c), 0, 32);
        if (e == hipSuccess)
            e = hipcub::DeviceRadixSort::SortPairs(nullptr, b2, ws.keys, ws.keys_s, ws.ids, ws.sids, int(c), 0, 32);
        ws.tmp_bytes = b1 > b2 ? b1 : b2;
        if (e == hipSuccess) e = hipMalloc(&ws.tmp, ws.tmp_bytes + 16);
    }
    if (e != hipSuccess) {
        build_release(ws);
        return e;
    }
    ws.cap = c;
    return hipSuccess;
}

hipError_t build_scene_gpu(BuildWorkspace& ws, const Sphere* sph, uint32_t n, const BuildOutputs& o,
                           bool refit, hipStream_t st, BuildSummary* out) {
    if (refit && ws.topo_n != n) return hipErrorInvalidValue;
    if (!refit) {
        if (hipError_t e = build_reserve(ws, n)) return e;
        ws.topo_n = 0;
    }
    const uint32_t n_geom = (n + 7u) & ~7u;
    k_init<<<1, 64, 0, st>>>(ws.S, refit);
    if (n_geom) {
        k_prep<<<blocks(n_geom), kBlock, 0, st>>>(sph, n, n_geom, o.geom, o.radius, o.mat,
                                                 refit ? nullptr : ws.rkeys, ws.ids, ws.S);
    }
    if (n) {
        if (!refit) {
            size_t tb = ws.tmp_bytes;
            if (hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(ws.tmp, tb, ws.rkeys, ws.rkeys_s, ws.ids,
                                                                            ws.ids_s, int(n), 0, 32, st))
                return e;
            if (hipError_t e = hipMemsetAsync(ws.is_big, 0, n, st)) return e;
            k_select<<<1, 64, 0, st>>>(ws.rkeys_s, ws.ids_s, n, o.big_ids, ws.is_big, ws.S);
        }
        k_reduce<<<blocks(n), kBlock, 0, st>>>(sph, n, ws.is_big, refit, ws.S);
        if (!refit) {
            k_morton<<<blocks(n), kBlock, 0, st>>>(sph, n, ws.is_big, ws.S, ws.keys, ws.ids);
            size_t tb = ws.tmp_bytes;
            if (hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws.tmp, tb, ws.keys, ws.keys_s, ws.ids, ws.sids,
                                                                  int(n), 0, 32, st))
                return e;
            k_karras<<<blocks(n), kBlock, 0, st>>>(ws.keys_s, ws.S, ws.par_i, ws.par_l, ws.left, ws.right, ws.lo,
                                                  ws.hi);
        }
        if (hipError_t e = hipMemsetAsync(ws.flags, 0, size_t(n) * 4, st)) return e;
        k_bottomup<<<blocks(n), kBlock, 0, st>>>(sph, ws.sids, ws.S, ws.par_i, ws.par_l, ws.left, ws.right, ws.lo,
                                                ws.hi, ws.flags, ws.bnd, ws.cnt, ws.lcnt);
        k_emit<<<blocks(2 * n), kBlock, 0, st>>>(sph, ws.sids, ws.S, ws.par_i, ws.par_l, ws.left, ws.lo, ws.hi,
                                                ws.bnd, ws.cnt, ws.lcnt, o.nodes, o.nodes_raw, o.leaf_geom,
                                                o.leaf_ids);
    }
    if (hipError_t e = hipGetLastError()) return e;
    if (hipError_t e = hipMemcpyAsync(out, ws.S, sizeof(BuildSummary), hipMemcpyDeviceToHost, st)) return e;
    if (!refit) ws.topo_n = n;
    return hipSuccess;
}

void schedule_release(TileSchedule& s) {
    void* ptrs[] = {s.cost[0], s.cost[1], s.order, s.keys, s.iota, s.norm, s.tmp};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    s = TileSchedule{};
}

hipError_t schedule_reserve(TileSchedule& s, uint32_t n, hipStream_t st) {
    if (s.n == n && s.cost[0]) return hipSuccess;
    schedule_release(s);
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = alloc(&s.cost[0], n);
    if (e == hipSuccess) e = alloc(&s.cost[1], n);
    if (e == hipSuccess) e = alloc(&s.order, n);
    if (e == hipSuccess) e = alloc(&s.keys, n);
    if (e == hipSuccess) e = alloc(&s.iota, n);
    if (e == hipSuccess) e = alloc(&s.norm, n);
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, s.tmp_bytes, s.cost[0], s.keys, s.iota, s.order,
                                                         int(n), 0, 16);
    if (e == hipSuccess) e = hipMalloc(&s.tmp, s.tmp_bytes + 16);
    if (e == hipSuccess) e = hipMemsetAsync(s.cost[0], 0, size_t(n) * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(s.cost[1], 0, size_t(n) * 4, st);
    if (e == hipSuccess) {
        k_iota<<<blocks(n), kBlock, 0, st>>>(s.iota, n);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        schedule_release(s);
        return e;
    }
    s.n = n;
    return hipSuccess;
}

// The sort key of tile order[r]: its recorded cost x the chunk count of rank r in the launch that
// recorded it (head_tiles 0: x 1), as the top 16 bits of its binary32 value (8 exponent + 7
// mantissa bits: monotonic in the cost, 2 radix passes instead of 4; the order is a scheduling
// heuristic, any order renders the same image). Written beside the recorded costs, never over
// them: schedule_order may run again on the same record (a launch that fails after it).
__global__ void k_cost_norm(const uint32_t* __restrict__ cost, const uint32_t* __restrict__ order, uint32_t n,
                            uint32_t head_tiles, uint32_t head_chunks, uint32_t chunks, uint32_t* __restrict__ norm) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint32_t t = head_tiles ? order[r] : r;
    const float v = float(cost[t]) * float(head_tiles ? (r < head_tiles ? head_chunks : chunks) : 1u);
    norm[t] = __float_as_uint(v) >> 16;
}

hipError_t schedule_order(TileSchedule& s, hipStream_t st) {
    const int last = s.cur ^ 1;
    // head_tiles != 0: `order` still holds the ranks that launch handed out
    k_cost_norm<<<blocks(s.n), kBlock, 0, st>>>(s.cost[last], s.order, s.n, s.rec_head_tiles[last],
                                               s.rec_head_chunks[last], s.rec_chunks[last], s.norm);
    if (hipError_t e = hipGetLastError()) return e;
    size_t tb = s.tmp_bytes;
    return hipcub::DeviceRadixSort::SortPairsDescending(s.tmp, tb, s.norm, s.keys, s.iota, s.order,
                                                        int(s.n), 0, 16, st);
}

hipError_t build_treelet(const BvhNode* nodes, uint32_t n_nodes, float* out, uint32_t* out_count, hipStream_t st) {
    k_treelet<<<1, kTreeletThreads, 0, st>>>(nodes, n_nodes, reinterpret_cast<float4*>(out), out_count);
    return hipGetLastError();
}

hipError_t build_grid_gpu(const BuildWorkspace& ws, const Sphere* sph, uint32_t n, const GridInfo& g,
                          uint32_t* cursor, uint32_t* cell_start, GeomRec* rec, uint32_t* ids, void* tmp,
                          size_t tmp_bytes, hipStream_t st) {
    if (!n) return hipSuccess;
    if (hipError_t e = hipMemsetAsync(cursor, 0, (size_t(g.n_cells) + 1) * 4, st)) return e;
    k_grid_refs<false><<<blocks(n), kBlock, 0, st>>>(sph, n, ws.is_big, g, cursor, nullptr, nullptr);
    size_t tb = tmp_bytes;
    if (hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cursor, cell_start, int(g.n_cells + 1), st)) return e;
    if (hipError_t e = hipMemcpyAsync(cursor, cell_start, size_t(g.n_cells) * 4, hipMemcpyDeviceToDevice, st)) return e;
    k_grid_refs<true><<<blocks(n), kBlock, 0, st>>>(sph, n, ws.is_big, g, cursor, rec, ids);
    return hipGetLastError();
}

size_t grid_scan_bytes(uint32_t n_cells) {
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, static_cast<uint32_t*>(nullptr),
                                           static_cast<uint32_t*>(nullptr), int(n_cells + 1));
    return tb;
}

hipError_t repad_nodes_gpu(const BvhNode* raw, BvhNode* nodes, uint32_t n_nodes, float pad, hipStream_t st) {
    if (!n_nodes) return hipSuccess;
    k_repad<<<blocks(n_nodes), kBlock, 0, st>>>(raw, nodes, n_nodes, pad);
    return hipGetLastError();
}

}  // namespace rt
