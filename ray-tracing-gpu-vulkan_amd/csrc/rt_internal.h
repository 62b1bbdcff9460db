// rt_internal.h — device data layout and launch parameters shared by the HIP kernels
// (rt_kernels.hip) and the host runtime (rt_api.cpp). Not part of the public C-ABI.
#pragma once

#include <stdint.h>

namespace rt {

// Per-sphere geometry record read by the closest-hit search (shader.rint:28-30):
// center.xyz and radius^2 (rounded once, as shader.rint:48 computes radius * radius).
struct alignas(16) GeomRec {
    float cx, cy, cz, rr;
};

// Per-sphere material record read once per hit (shader.rchit:39): 32 B instead of the
// reference's 80-B std140 Sphere, so one hit costs two 16-B loads.
struct alignas(16) MatRec {
    float c0x, c0y, c0z, attr;   // colors[0].rgb, materialSpecificAttribute
    float c1x, c1y, c1z;         // colors[1].rgb (checker)
    uint32_t type_tex;           // materialType | textureType << 8
};

// LBVH node, 32 B. Stackless "escape-link" layout: nodes are stored in depth-first order, so a
// hit on an inner node continues at index+1 and a miss (or a finished leaf) jumps to `escape`.
//   inner node: lo/hi = bounds of the subtree, count = 0
//   leaf:       lo/hi = bounds, first = first slot in the leaf-sphere permutation, count >= 1
struct alignas(16) BvhNode {
    float lox, loy, loz;
    uint32_t escape;             // next node index when the box is missed / leaf done; ~0u = end
    float hix, hiy, hiz;
    uint32_t first_count;        // leaf: first << 4 | count (count 1..15); inner: 0
};

// Two-wide LBVH node for the ordered (stack) walk, 64 B: both children's boxes, so one visit
// tests two boxes and descends into the nearer hit child first (the farther one is pushed).
// Child reference: bit 31 set = leaf, (first slot << 3) | count in the low bits; else the index
// of an inner node.
struct alignas(16) Bvh2Node {
    float l0x, l0y, l0z; uint32_t c0;   // child 0: box lo, reference
    float h0x, h0y, h0z; uint32_t pad0; // child 0: box hi
    float l1x, l1y, l1z; uint32_t c1;   // child 1: box lo, reference
    float h1x, h1y, h1z; uint32_t pad1; // child 1: box hi
};
constexpr uint32_t kLeafFlag = 0x80000000u;

// Compact escape-link node, 16 B (one ds_read_b128 per visit): the padded box rounded OUTWARD to
// binary16 (so it still contains every member sphere's AABB: the walk stays conservative and
// exact), the escape index and the leaf field in 16 bits each. Used when the tree has fewer than
// 65535 nodes and 8192 leaves (the LDS-staged case).
//   x = lo.x | lo.y << 16, y = lo.z | hi.x << 16, z = hi.y | hi.z << 16  (binary16 bit patterns)
//   w = escape | leaf << 16, escape 0xffff = end, leaf 0 = inner else 0x8000 | index << 2 | (count - 1)
struct alignas(16) BvhNode16 {
    uint32_t x, y, z, w;
};

// Scene as resident in HBM (one allocation per context, rebuilt by rt_set_scene).
struct DeviceScene {
    uint32_t n_spheres = 0;
    GeomRec* geom = nullptr;       // n_spheres, original sphere order (brute force + shading)
    float* radius = nullptr;       // n_spheres, for the AABB test (center -/+ radius)
    MatRec* mat = nullptr;         // n_spheres
    // LBVH over the "small" spheres; "big" spheres (radius above a scene-relative threshold,
    // e.g. the ground sphere r = 1000) are tested exhaustively before the tree walk.
    uint32_t n_big = 0;
    uint32_t* big_ids = nullptr;   // n_big sphere indices, ascending
    uint32_t n_nodes = 0;
    BvhNode* nodes = nullptr;      // 2 * n_leaf_spheres - 1 at most
    BvhNode* nodes_raw = nullptr;  // device-built trees: unpadded boxes (far-camera re-pad)
    GeomRec* leaf_geom = nullptr;  // spheres permuted into leaf order (contiguous per leaf)
    uint32_t* leaf_ids = nullptr;  // original index of each leaf slot
    uint32_t n_leaf = 0;
    BvhNode16* nodes16 = nullptr;  // compact escape-link nodes (null when the tree is too big)
    BvhNode* nodes_oct = nullptr;  // host-built trees: 8 x n_nodes, one near-child-first order per
                                   // ray octant (null: every octant copy uses `nodes`' order)
    float* treelet = nullptr;      // device-built trees: kTreeletCap x 8 floats (ACCEL_LBVH_TOP)
    uint32_t* treelet_count = nullptr;   // device word: nodes in the treelet
    Bvh2Node* nodes2 = nullptr;    // ordered-walk layout (same leaves)
    uint32_t n_nodes2 = 0;
    uint32_t root2 = 0;            // root reference (inner index or leaf reference)
    uint32_t depth2 = 0;           // inner nodes on the longest root-to-leaf path (stack bound)
    float small_rmax = 0.0f;       // largest radius in the tree
};

enum : uint32_t { ACCEL_BRUTE = 1, ACCEL_LBVH = 2, ACCEL_LBVH_LDS = 3, ACCEL_LBVH2 = 4, ACCEL_LBVH2_LDS = 5, ACCEL_LBVH16_LDS = 6, ACCEL_LBVH_LDS_SCENE = 7,
       ACCEL_LBVH_POOL = 8 /* LBVH_LDS_SCENE + tail-compaction pool, 1024-thread blocks */,
       ACCEL_LBVH_OCT = 9  /* LBVH_LDS_SCENE with 8 octant-specialised node copies, 1024-thread blocks */,
       ACCEL_LBVH_TOP = 10 /* tree too big for LDS: its top levels (treelet) in LDS, the rest from L2 */ };

// Top treelet of a tree too big for LDS (ACCEL_LBVH_TOP): the nodes of depth <= kTreeletDepth in
// the tree's depth-first order, 2 float4 each, AB layout: A = (lo.x, lo.y, hi.x, hi.y),
// B = (lo.z, hi.z, miss, hit). miss = treelet rank of the escape (END = ~0); hit = rank of the
// next node (inner node above the cut), or a word with bit 31 set: 0x80000000 | first_count
// (leaf) or 0xC0000000 | global node index (inner node at the cut: walk its subtree from L2).
constexpr uint32_t kTreeletDepth = 11;
constexpr uint32_t kTreeletCap = (2u << kTreeletDepth) - 1u;   // 4095 nodes, 128 KiB

// Counters block (device memory, zeroed before each launch by the host).
struct Counters {
    uint32_t work_head;            // next unit (pixel) to hand out; chunked refill: next 64-unit chunk
    uint32_t work_tail;            // chunked refill: next unit past n_chunk_units (per-lane hand-out)
    unsigned long long segments;
    unsigned long long samples;
    unsigned long long box_tests;
    unsigned long long sphere_tests;
    unsigned long long wave_iters; // COUNT builds: sum over waves of walk-loop iterations
    unsigned long long walk_hist[2][64];  // COUNT builds: box tests per segment, [miss, hit]
    unsigned long long lane_hist[65];     // COUNT builds: segment-loop iterations by tracing lanes
    unsigned long long t_first, t_dry, t_last;   // LBVH kernel: s_memrealtime of the first wave's
                                                 // start, of the pixel queue running dry, of the last exit
    unsigned long long stamp[8];   // diagnostic builds only (-DRT_STAMPS): cycles per phase
};

// Kernel launch parameters (passed by value as the kernel argument).
struct TraceParams {
    // Camera / viewport (shader.rgen:92-115), computed once per launch on the host.
    float lf[3], hor[3], ver[3], ulc[3], cup[3], crt[3];
    float half_aperture;
    float size_x, size_y;          // full image size as float (shader.rgen:42)
    uint32_t number, spp, max_depth;
    uint32_t seed_local;           // 1: seed from launch-local ids (shader.rgen:40 verbatim)
    uint32_t rng_counter;          // 1: RT_RNG_SAMPLE_COUNTER
    uint32_t sample_base;
    uint32_t accumulate;
    uint32_t off_x, off_y;         // band offset (rows == nullptr)
    uint32_t band_w, band_h;
    uint32_t tiles_x;              // ceil(band_w / 8)
    uint32_t n_units;              // tiles_x * ceil(band_h / 8) * 64
    uint32_t n_chunk_units;        // LBVH kernels: units [0, n_chunk_units) go out as whole 8x8 tiles
                                   // (one atomic per 64 pixels per wave), the rest pixel by pixel
    uint32_t first_chunks;         // tiles [0, first_chunks) start on wave id = tile rank (no atomic)
    uint32_t isolate_tiles;        // waves of the first LPT tiles take no further work
    const uint32_t* rows;          // optional global row per band row
    const uint32_t* tile_order;    // optional: hand-out rank -> 8x8 tile index (null: row-major)
    uint32_t* tile_cost;           // optional: per 8x8 tile, traced segments of its most expensive
                                   // pixel (zeroed by the host)
    uint32_t tile_cost_sum;        // A/B only: record the tile's total instead
    // scene
    uint32_t n_spheres;
    const GeomRec* geom;
    const float* radius;
    const MatRec* mat;
    uint32_t n_big;
    const uint32_t* big_ids;
    const BvhNode* nodes;
    uint32_t n_nodes;
    const BvhNode16* nodes16;
    const BvhNode* nodes_oct;      // optional, see DeviceScene
    const float* treelet;          // ACCEL_LBVH_TOP, see DeviceScene (2 float4 per node)
    const uint32_t* treelet_count;
    const Bvh2Node* nodes2;
    uint32_t n_nodes2, root2, stack_depth;
    uint32_t n_leaf;               // spheres in the tree (leaf slots)
    const GeomRec* leaf_geom;
    const uint32_t* leaf_ids;
    float cull_abs;                // LBVH node-cull slack: best + cull_abs + cull_rel * best
    float cull_rel;
    // outputs
    float* accum;                  // band_w * band_h * 4 floats
    uint32_t* out;                 // band_w * band_h packed rgba8
    Counters* counters;
};

}  // namespace rt
