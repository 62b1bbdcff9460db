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
//   boxes     an inner node covers the sorted range [lo, hi], so its box is the union (exact
//             float min / max) of the range's sphere boxes: a pyramid of unions over 64-sphere
//             groups (leafbox + level), then 8 lanes per node read at most 2 x 63 entries per
//             pyramid level. The cut tree (subtrees of <= 4 spheres become leaves) is counted the
//             same way: each cut leaf marks its first sphere, a node's leaves are the marks in its
//             range and its emitted nodes 2 leaves - 1. No atomics: the climb with an agent-scope
//             counter per node it replaced paid an L2 writeback + invalidate per level (364 us at
//             99 860 spheres; now 41 us: leafbox 6, levels 3 x 5, nodebox 20)
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

// Block-wide max / min (kBlock threads, every thread calls): wave results through LDS, so a block
// makes one device-scope atomic per summary field instead of one per wave. The summary fields are
// single addresses every block updates; memory-side atomics on one address serialise (99 860
// spheres: 1 560 waves x 8 fields took 143 us).
template <bool MAX>
__device__ __forceinline__ uint32_t block_reduce(uint32_t v) {
    __shared__ uint32_t part[kBlock / 64];
    v = MAX ? wave_max(v) : wave_min(v);
    __syncthreads();   // part[] may still be read by the previous call
    if (__lane_id() == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    v = part[0];
#pragma unroll
    for (uint32_t w = 1; w < kBlock / 64; w++) v = MAX ? max(v, part[w]) : min(v, part[w]);
    return v;
}
__device__ __forceinline__ uint32_t block_max(uint32_t v) { return block_reduce<true>(v); }
__device__ __forceinline__ uint32_t block_min(uint32_t v) { return block_reduce<false>(v); }

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
    Ro = block_max(Ro);
    if (threadIdx.x == 0) atomicMax(&S->R_o, Ro);
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

// Centroid bounds (Morton frame) and largest / smallest radius of the spheres in the tree: a
// grid-stride loop over kReduceBlocks blocks, block reductions, one atomic per field per block.
constexpr uint32_t kReduceBlocks = 96;
__global__ void __launch_bounds__(kBlock) k_reduce(const Sphere* __restrict__ sph, uint32_t n,
                                                   const uint8_t* __restrict__ is_big, bool refit,
                                                   BuildSummary* S) {
    uint32_t rmax = f2o(0.0f), rmin = f2o(INFINITY);
    uint32_t cmin[3], cmax[3];
#pragma unroll
    for (int k = 0; k < 3; k++) { cmin[k] = f2o(INFINITY); cmax[k] = f2o(-INFINITY); }
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        if (is_big[i]) continue;
        const rt_vec4 g = sph[i].geometry;
        rmax = max(rmax, f2o(g.w));
        rmin = min(rmin, f2o(g.w));
        const float c[3] = {g.x, g.y, g.z};
#pragma unroll
        for (int k = 0; k < 3; k++) { cmin[k] = min(cmin[k], f2o(c[k])); cmax[k] = max(cmax[k], f2o(c[k])); }
    }
    rmax = block_max(rmax);
    rmin = block_min(rmin);
    if (threadIdx.x == 0) { atomicMax(&S->rmax_o, rmax); atomicMin(&S->rmin_o, rmin); }
    if (refit) return;   // the Morton frame belongs to the stored topology
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t mn = block_min(cmin[k]), mx = block_max(cmax[k]);
        if (threadIdx.x == 0) { atomicMin(&S->cmin_o[k], mn); atomicMax(&S->cmax_o[k], mx); }
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

// Box pyramid over the m sorted spheres: level 0 = each sphere's box (lo.w = 1 when the sphere is
// the first of its cut leaf, as uint bits), level k + 1 entry j = union of level-k entries
// [64 j, 64 j + 64) (lo.w = their marks summed). kLevels levels hold up to 64^kLevels ... spheres
// per top entry; a node reads the top level whole.
constexpr uint32_t kLevels = 4;
__host__ __device__ __forceinline__ uint32_t level_size(uint32_t n, uint32_t k) {
    for (uint32_t i = 0; i < k; i++) n = (n + 63u) / 64u;
    return n;
}
__host__ __device__ __forceinline__ size_t level_offset(uint32_t cap, uint32_t k) {   // in PBox (2 float4)
    size_t off = 0;
    for (uint32_t i = 0; i < k; i++) off += level_size(cap, i);
    return off;
}

__global__ void __launch_bounds__(kBlock) k_leafbox(const Sphere* __restrict__ sph,
                                                    const uint32_t* __restrict__ sids, const BuildSummary* S,
                                                    const uint32_t* __restrict__ par_i,
                                                    const uint32_t* __restrict__ par_l,
                                                    const uint32_t* __restrict__ lo,
                                                    const uint32_t* __restrict__ hi, float4* pyr) {
    const uint32_t m = S->n_small;
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (m < 2 || p >= m) return;
    float b[6];
    prim_box(sph, sids[p], b);
    // the cut leaf holding sphere p: its highest ancestor of <= kLeafMax spheres (the root has none)
    uint32_t c = kPrim | p;
    for (uint32_t guard = 0; guard < kMaxDepth; guard++) {
        const uint32_t up = (c & kPrim) ? par_l[c & ~kPrim] : par_i[c];
        if (hi[up] - lo[up] + 1u > kLeafMax) break;
        c = up;
        if (c == 0u) break;
    }
    const uint32_t first = (c & kPrim) ? (c & ~kPrim) : lo[c];
    pyr[2 * size_t(p)] = make_float4(b[0], b[1], b[2], __uint_as_float(first == p ? 1u : 0u));
    pyr[2 * size_t(p) + 1] = make_float4(b[3], b[4], b[5], 0.0f);
}

struct BoxAcc {
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t marks = 0;
    __device__ __forceinline__ void add(const float4* __restrict__ e) {
        const float4 a = e[0], z = e[1];
        mn[0] = fminf(mn[0], a.x); mn[1] = fminf(mn[1], a.y); mn[2] = fminf(mn[2], a.z);
        mx[0] = fmaxf(mx[0], z.x); mx[1] = fmaxf(mx[1], z.y); mx[2] = fmaxf(mx[2], z.z);
        marks += __float_as_uint(a.w);
    }
    template <int LANES = 64>   // over aligned groups of LANES lanes
    __device__ __forceinline__ void wave_reduce() {
#pragma unroll
        for (int s = LANES / 2; s >= 1; s >>= 1) {
#pragma unroll
            for (int k = 0; k < 3; k++) {
                mn[k] = fminf(mn[k], __shfl_xor(mn[k], s));
                mx[k] = fmaxf(mx[k], __shfl_xor(mx[k], s));
            }
            marks += (uint32_t)__shfl_xor((int)marks, s);
        }
    }
};

// Level k + 1 of the pyramid from level k: one wave per entry.
__global__ void __launch_bounds__(kBlock) k_level(const BuildSummary* S, uint32_t cap, uint32_t k, float4* pyr) {
    const uint32_t m = S->n_small;
    const uint32_t j = (blockIdx.x * kBlock + threadIdx.x) >> 6, lane = __lane_id();
    if (m < 2 || j >= level_size(m, k + 1)) return;   // wave-uniform
    const float4* src = pyr + 2 * level_offset(cap, k);
    const uint32_t n_src = level_size(m, k), e = 64u * j + lane;
    BoxAcc acc;
    if (e < n_src) acc.add(src + 2 * size_t(e));
    acc.wave_reduce();
    if (lane == 0) {
        float4* dst = pyr + 2 * (level_offset(cap, k + 1) + j);
        dst[0] = make_float4(acc.mn[0], acc.mn[1], acc.mn[2], __uint_as_float(acc.marks));
        dst[1] = make_float4(acc.mx[0], acc.mx[1], acc.mx[2], 0.0f);
    }
}

// Inner node i (kNodeLanes lanes): box = union over its sorted range, cut-tree counts from the
// marks. The range [a, b) at level L splits into the entries before the next multiple of 64 and
// after the last one (read here) and the 64-aligned middle, which is [a / 64, b / 64) at level
// L + 1; at most 2 x 63 entries per level, the top level read whole. Most nodes span a few spheres:
// 8 lanes per node (a wave per node took 104 us at 99 860 spheres, mostly idle lanes).
constexpr uint32_t kNodeLanes = 8;
__global__ void __launch_bounds__(kBlock) k_nodebox(const BuildSummary* S, uint32_t cap,
                                                    const uint32_t* __restrict__ lo,
                                                    const uint32_t* __restrict__ hi,
                                                    const float4* __restrict__ pyr, float4* bnd, uint32_t* cnt,
                                                    uint32_t* lcnt) {
    const uint32_t m = S->n_small;
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t i = t / kNodeLanes, sub = t % kNodeLanes;
    const bool live = m >= 2 && i < m - 1u;
    BoxAcc acc;
    uint32_t l0 = 0, h0 = 0;
    if (live) {
        l0 = lo[i];
        h0 = hi[i];
        uint32_t a = l0, b = h0 + 1u;
        for (uint32_t L = 0; L < kLevels; L++) {
            const float4* P = pyr + 2 * level_offset(cap, L);
            if (b - a <= 128u || L + 1 == kLevels) {
                for (uint32_t e = a + sub; e < b; e += kNodeLanes) acc.add(P + 2 * size_t(e));
                break;
            }
            const uint32_t a1 = (a + 63u) & ~63u, b1 = b & ~63u;   // a1 < b1: b - a > 128
            for (uint32_t e = a + sub; e < a1; e += kNodeLanes) acc.add(P + 2 * size_t(e));
            for (uint32_t e = b1 + sub; e < b; e += kNodeLanes) acc.add(P + 2 * size_t(e));
            a = a1 >> 6;
            b = b1 >> 6;
        }
    }
    acc.wave_reduce<kNodeLanes>();   // every lane: the groups' shuffles stay inside the group
    if (live && sub == 0) {
        const bool leafy = h0 - l0 + 1u <= kLeafMax;
        bnd[2 * size_t(i)] = make_float4(acc.mn[0], acc.mn[1], acc.mn[2], 0.0f);
        bnd[2 * size_t(i) + 1] = make_float4(acc.mx[0], acc.mx[1], acc.mx[2], 0.0f);
        cnt[i] = leafy ? 1u : 2u * acc.marks - 1u;   // the cut subtree is a full binary tree
        lcnt[i] = leafy ? 1u : acc.marks;
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
                    ws.par_i, ws.par_l, ws.left, ws.right, ws.lo, ws.hi, ws.cnt, ws.lcnt,
                    ws.bnd, ws.pyr, ws.tmp, ws.S};
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
    RT_ALLOC(lo, c); RT_ALLOC(hi, c); RT_ALLOC(cnt, c); RT_ALLOC(lcnt, c);
    RT_ALLOC(bnd, 2 * size_t(c)); RT_ALLOC(pyr, 2 * level_offset(c, kLevels)); RT_ALLOC(S, 1);
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
        k_reduce<<<std::min(blocks(n), kReduceBlocks), kBlock, 0, st>>>(sph, n, ws.is_big, refit, ws.S);
        if (!refit) {
            k_morton<<<blocks(n), kBlock, 0, st>>>(sph, n, ws.is_big, ws.S, ws.keys, ws.ids);
            size_t tb = ws.tmp_bytes;
            if (hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws.tmp, tb, ws.keys, ws.keys_s, ws.ids, ws.sids,
                                                                  int(n), 0, 32, st))
                return e;
            k_karras<<<blocks(n), kBlock, 0, st>>>(ws.keys_s, ws.S, ws.par_i, ws.par_l, ws.left, ws.right, ws.lo,
                                                  ws.hi);
        }
        // node boxes and cut-tree counts (kernels read the small count from the summary; grids
        // sized for n, the excess exits)
        k_leafbox<<<blocks(n), kBlock, 0, st>>>(sph, ws.sids, ws.S, ws.par_i, ws.par_l, ws.lo, ws.hi, ws.pyr);
        constexpr uint32_t kWaves = kBlock / 64u;   // one wave per entry / node
        for (uint32_t k = 0; k + 1 < kLevels; k++)
            k_level<<<(level_size(n, k + 1) + kWaves - 1) / kWaves, kBlock, 0, st>>>(ws.S, ws.cap, k, ws.pyr);
        k_nodebox<<<(uint64_t(n) * kNodeLanes + kBlock - 1) / kBlock, kBlock, 0, st>>>(ws.S, ws.cap, ws.lo, ws.hi,
                                                                                      ws.pyr, ws.bnd, ws.cnt, ws.lcnt);
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

// The last launch's record carried over to a new tile count (a band that gained or lost rows at its
// end, rt_multi's balancer): tile t < min(old, new) keeps its cost x the chunk count its rank ran
// with (the normalisation k_cost_norm would apply), tiles beyond the old count start at 0 (they
// are handed out last). The carried record is then marked as one chunk count (rec_* = 1).
__global__ void k_cost_resize(const uint32_t* __restrict__ old_cost, const uint32_t* __restrict__ old_order,
                              uint32_t n_old, uint32_t head_tiles, uint32_t head_chunks, uint32_t chunks,
                              uint32_t* __restrict__ new_cost, uint32_t n_new) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_old) {
        const uint32_t t = head_tiles ? old_order[i] : i;
        if (t < n_new) {
            const uint64_t v = uint64_t(old_cost[t]) * (head_tiles ? (i < head_tiles ? head_chunks : chunks) : 1u);
            new_cost[t] = v > 0xffffffffull ? 0xffffffffu : uint32_t(v);
        }
    } else if (i < n_new) {
        new_cost[i] = 0u;
    }
}

hipError_t schedule_reserve(TileSchedule& s, uint32_t n, hipStream_t st) {
    if (s.n == n && s.cost[0]) return hipSuccess;
    TileSchedule old = s;   // released after its record is carried over
    const bool carry = old.valid && old.cost[0] && old.n && n;
    s = TileSchedule{};
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
    if (e == hipSuccess && carry) {   // the last launch's costs keep ordering the band's tiles
        const int last = old.cur ^ 1;
        k_cost_resize<<<blocks(std::max(old.n, n)), kBlock, 0, st>>>(
            old.cost[last], old.order, old.n, old.rec_head_tiles[last], old.rec_head_chunks[last],
            old.rec_chunks[last], s.cost[last], n);
        e = hipGetLastError();
        if (e == hipSuccess) {
            s.cur = old.cur;
            s.valid = true;
            s.rec_head_tiles[last] = 0;
            s.rec_head_chunks[last] = s.rec_chunks[last] = 1;
        }
    }
    schedule_release(old);
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
