// rt_grid.h — uniform grid over the scene's small spheres (host build, rt_grid.cpp): the closest-hit
// structure of the trace kernels for scenes of similar-size spheres, traversed by a 3D DDA
// (rt_kernels.hip grid_walk). Replaces the driver BVH of src/vulkan.h:395-554 like the LBVH does.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/rt_abi.h"
#include "rt_internal.h"

namespace rt {

struct HostGrid {
    GridInfo info{};
    std::vector<uint32_t> cell_start;   // n_cells + 1 offsets into the reference lists
    std::vector<GeomRec> rec;           // per reference: center, r^2 (cell-major, index order; r*r in binary32, test1)
    std::vector<uint32_t> ids;          // per reference: sphere index
};

// Builds the grid over the spheres not in `big` (tested exhaustively by the kernels). Every sphere
// is referenced by each cell its AABB, widened by `margin` + 1e-3 cell, overlaps (info.margin).
// Returns false when the scene does not suit a grid: no small spheres, radii spread over more than
// a factor 8, non-finite spheres, or more than `max_refs` references.
bool build_grid_host(const Sphere* spheres, uint32_t n, const std::vector<uint32_t>& big, float margin,
                     float cell_scale, uint32_t max_refs, HostGrid& out);

// The grid's layout for m small spheres of radius <= rmax whose AABBs span [lo, hi] (shared by the
// host build and the device build, rt_build.hip build_grid_gpu). Returns false when the cell count
// would exceed 2^24. *ref_bound = references at most (each sphere's widened AABB spans at most
// ceil((2 rmax + 2 margin) / cs) + 1 cells per axis).
// Cells sized for about kGridCellScale^3 small spheres per cell volume. Measured at config 3 / 5
// (scripts/scale_ab.py, images bit-identical): 1.5 / 1.7 / 1.9 / 2.2 / 2.6 / 3.0 ->
// 138.4 / 137.8 / 138.4 / 139.3 / 141.9 / 147.0 ms and 15.31 / 15.17 / 15.28 / 15.39 / 15.49 / 15.88 ms.
constexpr float kGridCellScale = 1.7f;
// Host-built grids (<= 1 024 spheres: staged in LDS, where a cell step costs an LDS read instead of
// an L2 round trip) take slightly smaller cells. Round 5, the one-layer walk, config 3 at 10 000 spp
// (scripts/grid_scale_ab.py): 1.55 / 1.6 / 1.65 / 1.7 -> 1 127.8 / 1 114.6 / 1 114.3 / 1 124.7 ms
// (19 cells a side at 1.6-1.65 against 18 at 1.7); config 5's device-built L2 grid keeps 1.7
// (1.65: +0.6 %).
constexpr float kGridCellScaleHost = 1.65f;

// Spare part of the registration margin, in cells (rt_api.cpp: it bounds the near cull slack).
#ifndef RT_GRID_SPARE
#define RT_GRID_SPARE 4e-3
#endif
bool grid_layout(const float lo[3], const float hi[3], uint32_t m, float rmax, float margin, float cell_scale,
                 GridInfo& gi, uint64_t* ref_bound);

}  // namespace rt
