// rt_internal.h — device data layout and launch parameters shared by the HIP kernels
// (rt_kernels.hip) and the host runtime (rt_api.cpp). Not part of the public C-ABI.
#pragma once

#include <stdint.h>

#include "../../include/rt_abi.h"

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
    float c1x, c1y, c1z;         // colors[1].rgb (checker); solid dielectrics: kMatDielConst
    uint32_t type_tex;           // materialType | textureType << 8 | flags
};
// Solid dielectric (colors[1] unused): c1 = {1 / attr, r0(front), r0(back)}, the per-sphere
// constants of shader.rchit:94 and :131 (eta = 1/ior on a front face, ior on a back face;
// r0 = ((1 - eta) / (1 + eta))^2, Q7), computed with the kernel's own binary32 operations.
constexpr uint32_t kMatDielConst = 1u << 16;

// Every colour a sphere can return as attenuation (shader.rchit:53-64: colors[0], and colors[1]
// of a checkered texture) lies in [0, 1] (NaN fails): then every sample colour does too, which
// RT_RNG_SAMPLE_HASH's 8.24 fixed-point sums require (rt_render_device refuses other scenes).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline bool colours_in_unit(const Sphere& s) {
    auto in = [](float v) { return v >= 0.0f && v <= 1.0f; };
    bool ok = in(s.colors[0].x) && in(s.colors[0].y) && in(s.colors[0].z);
    if (s.textureType == 1u) ok = ok && in(s.colors[1].x) && in(s.colors[1].y) && in(s.colors[1].z);
    return ok;
}

// Fills a material record (host and device builds alike).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline MatRec make_mat(float c0x, float c0y, float c0z, float attr, float c1x, float c1y, float c1z,
                       uint32_t mtype, uint32_t ttype) {
    MatRec m;
    m.c0x = c0x; m.c0y = c0y; m.c0z = c0z; m.attr = attr;
    m.c1x = c1x; m.c1y = c1y; m.c1z = c1z;
    m.type_tex = (mtype & 0xffu) | ((ttype & 0xffu) << 8);
    if (mtype == 2u && ttype != 1u) {
        const float ef = 1.0f / attr, eb = attr;
        const float qf = (1.0f - ef) / (1.0f + ef), qb = (1.0f - eb) / (1.0f + eb);
        m.c1x = ef;
        m.c1y = qf * qf;
        m.c1z = qb * qb;
        m.type_tex |= kMatDielConst;
    }
    return m;
}

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

// Uniform grid over the small spheres (rt_grid.h): cell (x, y, z) is index (z * n[1] + y) * n[0] + x,
// its references cell_start[c] .. cell_start[c + 1] into grid_rec / grid_ids.
struct GridInfo {
    float gmin[3];      // min corner
    float gmax[3];      // max corner (gmin + n * cs)
    float cs[3];        // cell size per axis
    float inv_cs[3];    // 1 / cs (cell of the entry point)
    float margin;       // registration margin (the entry box is widened by it too)
    float lo_m[3];      // entry box: gmin - margin, gmax + margin (one binary32 subtraction / addition,
    float hi_m[3];      // on the host: kernel operands from SGPRs instead of loop-invariant VGPRs)
    uint32_t n[3];      // cells per axis
    uint32_t n_cells, n_refs;
};

#ifndef RT_TRACE_BLOCK
#define RT_TRACE_BLOCK 768   // threads per block of the tree / grid kernels (rt_kernels.hip kTraceBlock)
#endif
// Static LDS of the grid kernels beside their dynamic LDS: per-thread 64-bit unit sums of the
// counter-based stream (rt_kernels.hip s_lane_sum).
constexpr unsigned kLaneSumLdsBytes = 3u * 8u * RT_TRACE_BLOCK;
// Wave-cooperative grid walk (ACCEL_GRID_COOP): per thread a ray (2 float4), a key (u64) and a
// pass marker (u32) in LDS.
constexpr unsigned kCoopLdsBytes = (2u * 16u + 8u + 4u) * RT_TRACE_BLOCK;
// Wave-wide candidate queue (ACCEL_GRID_CQ / ACCEL_GRID_REC_CQ): 128 queue entries (u32) and a
// count per wave, a key (u64) per thread.
constexpr unsigned kCqLdsBytes = (128u * 4u + 4u) * (RT_TRACE_BLOCK / 64u) + 8u * RT_TRACE_BLOCK;

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
    BvhNode* nodes_oct = nullptr;  // host-built trees: 8 x n_nodes, one near-child-first order per
                                   // ray octant (null: every octant copy uses `nodes`' order)
    float* treelet = nullptr;      // device-built trees: kTreeletCap x 8 floats (ACCEL_LBVH_TOP)
    uint32_t* treelet_count = nullptr;   // device word: nodes in the treelet
    float small_rmax = 0.0f;       // largest radius in the tree
    float small_rmin = 0.0f;       // smallest (<= 0 or NaN: the grid keeps the full cull slack)
    GridInfo grid{};               // host-built scenes that suit a grid (n_refs = 0: none)
    uint32_t* cell_start = nullptr;
    GeomRec* grid_rec = nullptr;
    uint32_t* grid_ids = nullptr;
};

// Trace kernel forms (rt_kernels.hip pick()). Production: BRUTE (BASELINE config 2), OCT (trees
// whose 8 octant node copies + scene records fit LDS: the canonical scene), LDS (one node copy +
// scene records in LDS), TOP (bigger trees: LDS treelet + L2 subtrees). GLOBAL (every node from
// L2) is the A/B reference of TOP (options.reserved[1] = 10).
enum : uint32_t { ACCEL_BRUTE = 1, ACCEL_LBVH_GLOBAL = 2, ACCEL_LBVH_LDS = 3, ACCEL_LBVH_OCT = 4,
                  ACCEL_LBVH_TOP = 5, ACCEL_GRID = 6, ACCEL_GRID_GLOBAL = 7, ACCEL_GRID_COOP = 8,
                  ACCEL_GRID_GLOBAL_COOP = 9, ACCEL_GRID_REC = 10, ACCEL_GRID_CQ = 11, ACCEL_GRID_REC_CQ = 12,
                  ACCEL_COUNT = 13 };

// Random stream layout of a launch (template parameter of the trace kernels).
//   STREAM: the reference's per-pixel LCG stream (random.glsl), or with rng_counter the TEA
//           counter restart per sample (RT_RNG_SAMPLE_COUNTER); dvec3 sum per pixel
//           (shader.rgen:55), one lane runs all samples of a pixel.
//   HASH:   RT_RNG_SAMPLE_HASH: sample s restarts the LCG at sample_seed(pixel_seed, s); per-sample
//           colours summed as 8.24 fixed point with integer atomics, so a pixel's samples may be
//           split into chunks on any lanes / GPUs in any order and the sum is the same bits.
enum : int { MODE_STREAM = 0, MODE_HASH = 1 };

// Top treelet of a tree too big for LDS (ACCEL_LBVH_TOP): the nodes of depth <= kTreeletDepth in
// the tree's depth-first order, 2 float4 each, AB layout: A = (lo.x, lo.y, hi.x, hi.y),
// B = (lo.z, hi.z, miss, hit). miss = treelet rank of the escape (END = ~0); hit = rank of the
// next node (inner node above the cut), or a word with bit 31 set: 0x80000000 | first_count
// (leaf) or 0xC0000000 | global node index (inner node at the cut: walk its subtree from L2).
#ifndef RT_TREELET_DEPTH
#define RT_TREELET_DEPTH 10
#endif
constexpr uint32_t kTreeletDepth = RT_TREELET_DEPTH;
constexpr uint32_t kTreeletCap = (2u << kTreeletDepth) - 1u;   // 2047 nodes, 64 KiB: two blocks per CU

// Counters block (device memory, zeroed before each launch by the host).
struct Counters {
    uint32_t work_head;            // next unit to hand out; block refill: next 64-unit block
    uint32_t work_tail;            // block refill: next unit past n_block_units (per-lane hand-out)
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
    unsigned long long util[2 * 16];   // diagnostic builds only (-DRT_UTIL): per code point k, wave
                                       // passes [2k] and active lanes summed over them [2k + 1]
    unsigned long long steals;     // counter-based stream: tail steals (rt_kernels.hip steal_tail)
    unsigned long long cells_empty;     // COUNT builds, grid walks: visited cells without references
    unsigned long long walk_split[4];   // COUNT builds: walk work (cells + references) per segment
                                        // pass, max over the wave's tracing lanes [0], over its bounce
                                        // lanes only [1]; primary lanes' summed work [2], count [3]
};

// Kernel launch parameters (passed by value as the kernel argument).
//
// Work units: unit u = (8x8 tile, sample chunk, pixel of the tile). Block b = u / 64 covers one
// chunk of one tile's 64 pixels; tile rank = b / n, chunk = b % n for the n = head_chunks chunks
// of the head ranks, then likewise over the remaining blocks with n = chunks; the tile is
// tile_order[rank] (LPT hand-out) or the rank itself. Chunk c of n runs samples
// [c * spp / n, (c + 1) * spp / n). STREAM launches have one chunk.
struct TraceParams {
    // Camera / viewport (shader.rgen:92-115), computed once per launch on the host.
    float lf[3], hor[3], ver[3], ulc[3], cup[3], crt[3];
    float half_aperture;
    uint32_t pinhole_lf;           // 1: half_aperture = 0, lf has no zero component and crt / cup are
                                   // finite, so the ray origin lf + rx crt + ry cup (rx, ry = +-0, or
                                   // NaN when the disk sample is (0, 0)) is lf itself or NaN
    float size_x, size_y;          // full image size as float (shader.rgen:42)
    double inv_size_x, inv_size_y; // 1 / size, rounded to double (camera division, rt_kernels.hip)
    uint32_t number, spp, max_depth;
    uint32_t seed_local;           // 1: seed from launch-local ids (shader.rgen:40 verbatim)
    uint32_t rng_counter;          // STREAM only, 1: RT_RNG_SAMPLE_COUNTER
    uint32_t sample_base;
    uint32_t accumulate;           // STREAM: the pixel sum starts from accum (HASH: the resolve adds it)
    uint32_t off_x, off_y;         // band offset (rows == nullptr)
    uint32_t band_w, band_h;
    uint32_t tiles_x;              // ceil(band_w / 8)
    uint32_t chunks;               // sample chunks per pixel (>= 1)
    uint32_t head_tiles;           // hand-out ranks [0, head_tiles) (the head of the LPT order, the
    uint32_t head_chunks;          // longest tiles) split a pixel into head_chunks chunks, the
                                   // other ranks into `chunks`; 0 tiles: no head
    uint32_t n_units;              // 64 * (head_tiles * head_chunks + (tiles - head_tiles) * chunks)
    uint32_t n_block_units;        // units [0, n_block_units) go out as whole 64-unit blocks (one
                                   // atomic per block per wave), the rest unit by unit
    uint32_t first_blocks;         // blocks [0, first_blocks) start on wave id = block (no atomic)
    uint32_t isolate_blocks;       // waves of the first LPT blocks take no further work
    uint32_t force_regate;         // test only: every segment's winner recomputed by the gated brute force
    const uint32_t* rows;          // optional global row per band row
    uint32_t rows_lds;             // rows staged in dynamic LDS at this byte offset by the walk
                                   // kernels' prologue (kNoRowsLds: read from global memory)
    const uint32_t* tile_order;    // optional: hand-out rank -> 8x8 tile index (null: row-major)
    uint32_t* tile_cost;           // optional: per 8x8 tile, traced segments of its longest unit
                                   // (zeroed by the host)
    // scene
    uint32_t n_spheres;
    const GeomRec* geom;
    const float* radius;
    const MatRec* mat;
    uint32_t n_big;
    const uint32_t* big_ids;
    const BvhNode* nodes;
    uint32_t n_nodes;
    const BvhNode* nodes_oct;      // optional, see DeviceScene
    const float* treelet;          // ACCEL_LBVH_TOP, see DeviceScene (2 float4 per node)
    const uint32_t* treelet_count;
    uint32_t n_leaf;               // spheres in the tree (leaf slots)
    const GeomRec* leaf_geom;
    const uint32_t* leaf_ids;
    float cull_abs;                // LBVH node-cull slack: best + cull_abs + cull_rel * best
    float cull_rel;
    float cull_near_t, cull_near_abs;   // grid walks: best <= cull_near_t uses cull_near_abs instead
    GridInfo grid;                 // ACCEL_GRID
    const uint32_t* cell_start;
    const GeomRec* grid_rec;
    const uint32_t* grid_ids;
    // outputs
    float* accum;                  // STREAM: band_w * band_h * 4 floats
    uint32_t* out;                 // STREAM: band_w * band_h packed rgba8
    unsigned long long* fixed;     // HASH: 3 planes of band_w * band_h u64 (r, g, b), zero on entry
    Counters* counters;
    const float* big_tab;          // the big spheres as kBigMax records {cx, cy, cz, r} (padded to a
                                   // multiple of 4 by repeating the last) + kBigMax ids, filled per
                                   // launch (rt_big_table_kernel), read through the scalar cache
};

// HASH mode fixed point: a sample colour channel c in [0, 1] (every colour and the sky are <= 1,
// so is every product of them) adds trunc(c * 2^24) (rt_kernels.hip sample_fixed). A lane sums its
// samples in 32 bits and adds the partial to the pixel's 64-bit sum whenever its next sample index
// is a multiple of kFixedFlush, and at the end of its unit: a partial holds <= 128 * 2^24 = 2^31.
constexpr int kFixedFracBits = 24;
constexpr uint32_t kFixedFlush = 128;

// "Big" spheres (radius above a scene-relative threshold, e.g. the ground sphere) are tested by
// every segment before the tree walk; at most kBigMax of them. A one-wave kernel writes their
// records (center, radius) and ids into TraceParams::big_tab before each launch; the walk kernels
// read them through the scalar cache (rt_kernels.hip setup_ray).
constexpr uint32_t kBigMax = 64;
constexpr uint32_t kRecStatic = 512;   // spheres of the REC grid kernels' static LDS record table
constexpr uint32_t kNoRowsLds = 0xffffffffu;
constexpr uint32_t kHashMaxSpp = 1u << 19;

}  // namespace rt
