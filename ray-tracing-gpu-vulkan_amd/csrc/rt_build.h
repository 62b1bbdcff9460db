// rt_build.h — device-side scene build and refit (rt_build.hip). Replaces the per-frame
// BLAS/TLAS rebuild of the reference (src/vulkan.h:395-554, :1020-1059) and its AABB fill
// (src/ray_trace.cpp:583-599) with a parallel LBVH build over the spheres in HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_abi.h"
#include "rt_internal.h"

namespace rt {

// Build results read back by the host (one small copy per build / refit).
struct BuildSummary {
    uint32_t n_big, n_small, n_nodes, n_leaf_slots;
    uint32_t rmax_o, R_o;            // order-preserving bit patterns of small_rmax and R
    uint32_t rmin_o;                 // ... and of the smallest small radius
    uint32_t cmin_o[3], cmax_o[3];   // centroid bounds of the small spheres (Morton frame)
    uint32_t colour_out_of_range;    // != 0: some sphere colour leaves [0, 1] (colours_in_unit)
    float root_lo[3], root_hi[3];    // unpadded root box (the small spheres' AABB union): the grid's
                                     // bounds, so the host needs no second read-back
};
float summary_float(uint32_t ordered);

// Destination arrays (DeviceScene), sized for n spheres:
//   geom round_up(n, 8), radius n, mat n, big_ids 64, nodes / nodes_raw max(1, 2n),
//   leaf_geom / leaf_ids 4n.
struct BuildOutputs {
    GeomRec* geom;
    float* radius;
    MatRec* mat;
    uint32_t* big_ids;
    BvhNode* nodes;       // padded for pad(R) (the traversal's copy)
    BvhNode* nodes_raw;   // exact unions (re-padded for far cameras)
    GeomRec* leaf_geom;
    uint32_t* leaf_ids;
};

// Scratch that persists between a build and later refits (sorted order, radix-tree topology).
struct BuildWorkspace {
    uint32_t cap = 0;        // spheres the buffers hold
    uint32_t topo_n = 0;     // sphere count of the topology a refit may reuse (0: none)
    float* rkeys = nullptr;  float* rkeys_s = nullptr;
    uint32_t* ids = nullptr; uint32_t* ids_s = nullptr;
    uint32_t* keys = nullptr; uint32_t* keys_s = nullptr; uint32_t* sids = nullptr;
    uint8_t* is_big = nullptr;
    uint32_t* par_i = nullptr; uint32_t* par_l = nullptr;
    uint32_t* left = nullptr;  uint32_t* right = nullptr;
    uint32_t* lo = nullptr;    uint32_t* hi = nullptr;
    uint32_t* cnt = nullptr; uint32_t* lcnt = nullptr;
    float4* bnd = nullptr;   // 2 per inner node: lo.xyz, hi.xyz
    float4* pyr = nullptr;   // box pyramid over the sorted spheres (rt_build.hip k_leafbox / k_level)
    void* tmp = nullptr;     size_t tmp_bytes = 0;
    BuildSummary* S = nullptr;
};

hipError_t build_reserve(BuildWorkspace& ws, uint32_t n);
void build_release(BuildWorkspace& ws);

// Full build (refit = false) or refit of the previous topology (refit = true: same n, same big
// set and leaf assignment; boxes, records, radii bounds and padding recomputed). Asynchronous on
// `st`, the summary included: it is copied into *out (pinned host memory), valid once `st` has
// reached that point (the caller records an event after this call).
hipError_t build_scene_gpu(BuildWorkspace& ws, const Sphere* d_spheres, uint32_t n,
                           const BuildOutputs& o, bool refit, hipStream_t st, BuildSummary* out);

// Pixel hand-out order of the persistent trace kernel (longest-processing-time first). A lane
// runs one pixel's samples as one sequential chain (the per-pixel LCG stream), so the frame ends
// with every lane finishing its last pixel alone, and the frame ends with the longest chain still
// running. Tiles are handed out in descending order of their most expensive pixel (traced
// segments) in the previous launch over the same band geometry, recorded by the kernel itself
// (one atomicMax per finished pixel), so long chains start early and the last ones are short.
struct TileSchedule {
    uint32_t n = 0;                // tiles of the geometry the tables belong to
    uint32_t* cost[2] = {nullptr, nullptr};   // ping-pong: the launch being recorded, the last one
    uint32_t* order = nullptr;     // hand-out rank -> tile
    uint32_t* keys = nullptr;      // sort scratch
    uint32_t* iota = nullptr;
    uint32_t* norm = nullptr;      // costs scaled by their chunk counts (schedule_order's sort keys)
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int cur = 0;                   // table the next launch records into
    bool valid = false;            // cost[cur ^ 1] holds a completed launch of this geometry
    // the head / tail chunk split of the launch that recorded cost[k] (TraceParams head_tiles,
    // head_chunks, chunks; head_tiles = 0: one chunk count): its unit chains are per chunk, so
    // schedule_order scales each tile's cost by its chunk count before sorting (a per-pixel chain
    // estimate, comparable between head and tail tiles)
    uint32_t rec_head_tiles[2] = {0, 0}, rec_head_chunks[2] = {1, 1}, rec_chunks[2] = {1, 1};
};
// (Re)allocates for n tiles when the geometry changes. A valid record of the last launch is carried
// over (tiles below both counts keep their chunk-normalised cost, new tiles cost 0), so a band that
// gains or loses rows at its end keeps its LPT order; without one the tables are zeroed.
hipError_t schedule_reserve(TileSchedule& s, uint32_t n, hipStream_t st);
void schedule_release(TileSchedule& s);
// order = tiles by descending cost of the last launch (stable: ties in tile order).
hipError_t schedule_order(TileSchedule& s, hipStream_t st);

// nodes[i] = nodes_raw[i] grown by `pad` on every side (far-camera re-pad).
hipError_t repad_nodes_gpu(const BvhNode* raw, BvhNode* nodes, uint32_t n_nodes, float pad, hipStream_t st);
// Top treelet of the padded tree for ACCEL_LBVH_TOP (layout in rt_internal.h): out holds
// kTreeletCap x 8 floats, *out_count receives the node count. Asynchronous on `st`.
hipError_t build_treelet(const BvhNode* nodes, uint32_t n_nodes, float* out, uint32_t* out_count, hipStream_t st);

// Uniform grid over the small spheres of the last build_scene_gpu (its big flags), layout g from
// rt_grid.h grid_layout: cell_start (n_cells + 1), references rec / ids (cell-major; order within a
// cell unspecified), cursor scratch (n_cells + 1), tmp: grid_scan_bytes(n_cells).
hipError_t build_grid_gpu(const BuildWorkspace& ws, const Sphere* d_spheres, uint32_t n, const GridInfo& g,
                          uint32_t* cursor, uint32_t* cell_start, GeomRec* rec, uint32_t* ids, void* tmp,
                          size_t tmp_bytes, hipStream_t st);
size_t grid_scan_bytes(uint32_t n_cells);

}  // namespace rt
