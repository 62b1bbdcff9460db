// rt_bvh.h — host-side LBVH build interface (rt_bvh.cpp).
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/rt_abi.h"
#include "rt_internal.h"

namespace rt {

struct HostBvh {
    std::vector<uint32_t> big_ids;    // spheres tested exhaustively, ascending index
    std::vector<BvhNode> nodes;       // depth-first, escape links
    std::vector<GeomRec> leaf_geom;   // small spheres in leaf order: center, RADIUS (4 per leaf)
    std::vector<uint32_t> leaf_ids;   // original index per leaf slot
    float small_rmax = 0.0f;          // largest radius inside the tree (traversal slack)
    float small_rmin = INFINITY;      // smallest one (grid cull slack, rt_api.cpp)
};

// sah: binned surface-area splits (the default tree for small scenes); else the Morton radix
// split that rt_build.hip reproduces on the device. sah_knobs (A/B only, rt_debug_tune "sah_knobs";
// 0 = the measured best): bit 0 classic cost (area x spheres), bit 1 exact sweep, bits 2-3 child
// order (1 larger-area child first, 2 smaller first).
void build_lbvh_host(const Sphere* spheres, uint32_t n, HostBvh& out, bool sah, uint32_t sah_knobs = 0);

}  // namespace rt
