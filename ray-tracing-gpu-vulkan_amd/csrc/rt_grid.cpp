// rt_grid.cpp — host build of the uniform grid (rt_grid.h).
//
// Cells are sized for about `cell_scale`^3 small spheres per cell volume (cube root of the bounds'
// volume per sphere); each axis gets ceil(extent / size) cells spanning the small spheres' AABB
// bounds exactly. A sphere is referenced by every cell its AABB (center -/+ radius, the box the
// kernels' AABB gate uses) overlaps after widening by `margin`: the DDA may attribute a stretch of
// ray within rounding distance of a cell boundary to a neighbouring cell, and the margin keeps every
// sphere near that boundary in both. References of a cell are in sphere-index
// order and carry the sphere's record, so a cell's spheres are one contiguous run.
#include "rt_grid.h"

#include <algorithm>
#include <cmath>

namespace rt {

bool grid_layout(const float lo[3], const float hi[3], uint32_t m, float rmax, float margin, float cell_scale,
                 GridInfo& gi, uint64_t* ref_bound) {
    gi = GridInfo{};
    double ext[3], vol = 1.0;
    for (int k = 0; k < 3; k++) {
        ext[k] = std::max(double(hi[k]) - lo[k], 1e-6);
        vol *= std::max(ext[k], 2.0 * rmax);   // a flat layer counts one sphere diameter thick
    }
    const double size = cell_scale * std::cbrt(vol / std::max(1u, m));
    uint64_t cells = 1, span = 1;
    for (int k = 0; k < 3; k++) {
        const uint32_t nk = uint32_t(std::min(4096.0, std::max(1.0, std::ceil(ext[k] / size))));
        gi.n[k] = nk;
        gi.gmin[k] = lo[k];
        gi.gmax[k] = hi[k];
        gi.cs[k] = float(ext[k] / nk);
        gi.inv_cs[k] = 1.0f / gi.cs[k];
        cells *= nk;
    }
    if (cells > (1u << 24)) return false;
    gi.n_cells = uint32_t(cells);
    gi.margin = margin + float(RT_GRID_SPARE) * std::min(gi.cs[0], std::min(gi.cs[1], gi.cs[2]));
    for (int k = 0; k < 3; k++) {
        gi.lo_m[k] = gi.gmin[k] - gi.margin;
        gi.hi_m[k] = gi.gmax[k] + gi.margin;
    }
    for (int k = 0; k < 3; k++)
        span *= std::min<uint64_t>(gi.n[k], uint64_t(std::ceil((2.0 * rmax + 2.0 * gi.margin) / gi.cs[k])) + 1u);
    if (ref_bound) *ref_bound = span * m;
    return true;
}

bool build_grid_host(const Sphere* sph, uint32_t n, const std::vector<uint32_t>& big, float margin,
                     float cell_scale, uint32_t max_refs, HostGrid& out) {
    out = HostGrid{};
    std::vector<char> is_big(n, 0);
    for (uint32_t i : big) is_big[i] = 1;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float rmin = INFINITY, rmax = 0.0f;
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (is_big[i]) continue;
        const rt_vec4& g = sph[i].geometry;
        const float c[3] = {g.x, g.y, g.z};
        if (!std::isfinite(g.x) || !std::isfinite(g.y) || !std::isfinite(g.z) || !std::isfinite(g.w)) return false;
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], c[k] - g.w);
            hi[k] = std::max(hi[k], c[k] + g.w);
        }
        rmin = std::min(rmin, std::fabs(g.w));
        rmax = std::max(rmax, std::fabs(g.w));
        m++;
    }
    if (m == 0 || !(rmax > 0.0f) || rmax > 8.0f * rmin) return false;
    GridInfo& gi = out.info;
    if (!grid_layout(lo, hi, m, rmax, margin, cell_scale, gi, nullptr)) return false;
    margin = gi.margin;
    // cell range of a sphere's widened AABB on axis k (clamped to the grid)
    auto range = [&](int k, float c, float r, uint32_t& a, uint32_t& b) {
        const double x0 = (double(c - r) - margin - gi.gmin[k]) / gi.cs[k];
        const double x1 = (double(c + r) + margin - gi.gmin[k]) / gi.cs[k];
        a = uint32_t(std::min<double>(gi.n[k] - 1, std::max(0.0, std::floor(x0))));
        b = uint32_t(std::min<double>(gi.n[k] - 1, std::max(0.0, std::floor(x1))));
    };
    std::vector<uint32_t> count(gi.n_cells + 1, 0);
    uint64_t refs = 0;
    for (int pass = 0; pass < 2; pass++) {
        std::vector<uint32_t> fill;
        if (pass == 1) {
            out.cell_start.assign(gi.n_cells + 1, 0);
            for (uint32_t c = 0; c < gi.n_cells; c++) out.cell_start[c + 1] = out.cell_start[c] + count[c];
            out.rec.resize(refs);
            out.ids.resize(refs);
            fill.assign(out.cell_start.begin(), out.cell_start.end() - 1);
        }
        for (uint32_t i = 0; i < n; i++) {   // index order: each cell's references sorted by index
            if (is_big[i]) continue;
            const rt_vec4& g = sph[i].geometry;
            uint32_t a[3], b[3];
            range(0, g.x, g.w, a[0], b[0]);
            range(1, g.y, g.w, a[1], b[1]);
            range(2, g.z, g.w, a[2], b[2]);
            for (uint32_t z = a[2]; z <= b[2]; z++)
                for (uint32_t y = a[1]; y <= b[1]; y++)
                    for (uint32_t x = a[0]; x <= b[0]; x++) {
                        const uint32_t c = (z * gi.n[1] + y) * gi.n[0] + x;
                        if (pass == 0) {
                            count[c]++;
                            if (++refs > max_refs) return false;
                        } else {
                            const uint32_t j = fill[c]++;
                            out.rec[j] = GeomRec{g.x, g.y, g.z, g.w * g.w};   // r^2 (rt_grid.h)
                            out.ids[j] = i;
                        }
                    }
        }
    }
    gi.n_refs = uint32_t(refs);
    return true;
}

}  // namespace rt
