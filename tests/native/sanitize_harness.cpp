// sanitize_harness.cpp — the path's host C++ under AddressSanitizer + UndefinedBehaviorSanitizer
// (race detection / sanitizers row: the reference runs with its validation layers
// off, src/vulkan.h:51). Test infrastructure: built and run by tests/native/Makefile `sanitize`
// (tests/test_sanitize.py), never shipped.
//
// Driven here, with the scenes of configs 3 and 5 and the edge scenes of
// tests/test_gpu_build.py::test_device_tree_edge_cases:
//   * the host SAH and Morton LBVH builders (csrc/rt_bvh.cpp) and the host uniform grid
//     (csrc/rt_grid.cpp) — what rt_set_scene runs for scenes of up to 1 024 spheres;
//   * the grid layout of the device build (grid_layout, config 5's bounds);
//   * the multi-device partition, balancer and frame plan (csrc/rt_plan.cpp): every device count
//     1-9 over the image heights of the configs and small odd ones, random partitions, random
//     device times and row weights, malformed inputs;
//   * the CPU oracle (oracle/rt_oracle.cpp): scenes, small frames in both streams, with a rows map
//     and accumulation, the tonemap.
// Every structural property is checked; the process exits non-zero on the first violation (and
// the sanitizers abort on the first error).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/rt_abi.h"
#include "../../include/rt_mi355x.h"
#include "../../ray-tracing-gpu-vulkan_amd/csrc/rt_bvh.h"
#include "../../ray-tracing-gpu-vulkan_amd/csrc/rt_grid.h"
#include "../../ray-tracing-gpu-vulkan_amd/csrc/rt_plan.h"

extern "C" {
int orc_generate_scene(float t, uint32_t K, Sphere* out, uint32_t capacity, uint32_t* count);
int orc_render(const Sphere* spheres, uint32_t n, const RenderCallInfo* rci, const uint32_t* rows, uint32_t band_w,
               uint32_t band_h, const rt_options* opt, float* accum, uint8_t* out, uint64_t* stats3, int threads);
int orc_resolve(const float* acc, uint64_t n_texels, uint32_t spp, uint8_t* out);
}

namespace {

int g_checks = 0;
#define CHECK(cond)                                                                          \
    do {                                                                                     \
        g_checks++;                                                                          \
        if (!(cond)) {                                                                       \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond);   \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

std::vector<Sphere> scene(float t, uint32_t K) {
    uint32_t n = 0;
    orc_generate_scene(t, K, nullptr, 0, &n);
    std::vector<Sphere> s(n);
    CHECK(orc_generate_scene(t, K, s.data(), n, &n) == 0);
    return s;
}

std::vector<Sphere> spheres_at(const std::vector<float>& c, const std::vector<float>& r) {
    const std::vector<Sphere> base = scene(0.0f, 11);
    std::vector<Sphere> s(r.size());
    for (size_t i = 0; i < r.size(); i++) {
        s[i] = base[i % base.size()];
        s[i].geometry = rt_vec4{c[3 * i], c[3 * i + 1], c[3 * i + 2], r[i]};
    }
    return s;
}

// The edge scenes of tests/test_gpu_build.py::test_device_tree_edge_cases.
std::vector<std::vector<Sphere>> edge_scenes() {
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(0.0f, 1.0f);
    auto uni = [&](float a, float b) { return a + (b - a) * u(g); };
    std::vector<std::vector<Sphere>> out;
    out.push_back(spheres_at({0, -1000, 1}, {1000}));                                     // one
    out.push_back(spheres_at({0, -1000, 1, 1, 0.2f, 1}, {1000, 0.2f}));                   // two
    {   // five
        std::vector<float> c, r;
        for (int i = 0; i < 5; i++) { c.insert(c.end(), {uni(-3, 3), uni(-3, 3), uni(-3, 3)}); r.push_back(0.2f); }
        out.push_back(spheres_at(c, r));
    }
    {   // dups: coincident centres
        std::vector<float> c, r;
        for (int i = 0; i < 37; i++) {
            const float x = uni(-5, 5), y = uni(-5, 5), z = uni(-5, 5);
            for (int k = 0; k < 7; k++) { c.insert(c.end(), {x, y, z}); r.push_back(uni(0.1f, 0.3f)); }
        }
        out.push_back(spheres_at(c, r));
    }
    out.push_back(spheres_at(std::vector<float>(33 * 3, 0.0f), std::vector<float>(33, 0.5f)));   // all equal
    {   // many big, tied radii
        std::vector<float> c, r;
        for (int i = 0; i < 300; i++) {
            c.insert(c.end(), {uni(-50, 50), uni(-50, 50), uni(-50, 50)});
            r.push_back(i < 200 ? 0.2f : float(3 + (i % 3)));
        }
        out.push_back(spheres_at(c, r));
    }
    {   // flat line
        std::vector<float> c, r;
        for (int i = 0; i < 129; i++) { c.insert(c.end(), {-10.0f + 20.0f * float(i) / 128.0f, 0.0f, 0.0f}); r.push_back(0.05f); }
        out.push_back(spheres_at(c, r));
    }
    return out;
}

void check_tree(const std::vector<Sphere>& s, bool sah) {
    rt::HostBvh b;
    rt::build_lbvh_host(s.data(), uint32_t(s.size()), b, sah);
    CHECK(!b.nodes.empty() || s.empty());
    CHECK(b.leaf_geom.size() == b.leaf_ids.size());
    std::vector<int> seen(s.size(), 0);
    for (uint32_t id : b.big_ids) {
        CHECK(id < s.size());
        seen[id]++;
    }
    for (size_t k = 0; k < b.leaf_ids.size(); k++) {
        // leaf slots hold the small spheres once each (padding slots repeat an id with radius 0 or
        // sit outside the count; count only slots whose record is the sphere's)
        const uint32_t id = b.leaf_ids[k];
        CHECK(id < s.size() || b.leaf_geom[k].rr <= 0.0f);
        if (id < s.size() && b.leaf_geom[k].cx == s[id].geometry.x && b.leaf_geom[k].cy == s[id].geometry.y &&
            b.leaf_geom[k].cz == s[id].geometry.z && b.leaf_geom[k].rr == s[id].geometry.w)
            seen[id]++;
    }
    for (size_t i = 0; i < s.size(); i++) CHECK(seen[i] >= 1);
    rt::HostGrid grid;
    if (rt::build_grid_host(s.data(), uint32_t(s.size()), b.big_ids, 64.0f * 0x1p-24f * 1100.0f, rt::kGridCellScaleHost,
                            1u << 22, grid)) {
        CHECK(grid.cell_start.size() == size_t(grid.info.n_cells) + 1);
        for (size_t c = 0; c + 1 < grid.cell_start.size(); c++) CHECK(grid.cell_start[c] <= grid.cell_start[c + 1]);
        CHECK(grid.cell_start.back() == grid.ids.size() && grid.ids.size() == grid.rec.size());
        for (uint32_t id : grid.ids) CHECK(id < s.size());
    }
}

void check_plans() {
    using namespace rt::plan;
    std::mt19937 g(2024);
    const uint32_t heights[] = {1, 5, 7, 8, 27, 64, 1080, 2160};
    for (uint32_t n = 1; n <= 9; n++) {
        for (uint32_t H : heights) {
            Parts parts = strip_parts(n, H);
            std::vector<int> seen(H, 0);
            size_t mn = H, mx = 0;
            for (auto& p : parts) {
                for (uint32_t y : p.second) {
                    CHECK(y < H);
                    seen[y]++;
                }
                mn = std::min(mn, p.second.size());
                mx = std::max(mx, p.second.size());
            }
            for (uint32_t y = 0; y < H; y++) CHECK(seen[y] == 1);
            CHECK(mx - mn <= 1);
            for (int acc = 0; acc < 2; acc++) {
                Parts cp = parts;
                const FramePlan p = make_plan(1920, H, std::move(cp), acc != 0);
                const std::vector<uint32_t> v = serialize(p);
                CHECK(v.size() >= 2 && v[0] == p.parts.size() && v[1] == p.steps.size());
            }
            // balancing: random row costs, random device times and weights, a few rounds
            std::vector<double> cost(H, 0.0);
            std::uniform_real_distribution<float> u(0.5f, 2.0f);
            for (int round = 0; round < 4; round++) {
                std::vector<float> ms(n);
                std::vector<std::vector<double>> w(n);
                for (uint32_t d = 0; d < n; d++) {
                    ms[d] = u(g) * float(parts[d].second.size());
                    if (round % 2) for (size_t k = 0; k < parts[d].second.size(); k++) w[d].push_back(u(g));
                }
                update_costs(parts, ms.data(), cost, round % 2 ? &w : nullptr);
                std::vector<double> loads;
                const double before = imbalance(parts, cost);
                rebalance(parts, cost, 0.0, &loads);
                CHECK(imbalance(parts, cost) <= before + 1e-12);
                std::vector<int> seen2(H, 0);
                for (auto& p : parts)
                    for (uint32_t y : p.second) seen2[y]++;
                for (uint32_t y = 0; y < H; y++) CHECK(seen2[y] == 1);
                std::vector<uint32_t> rows, counts;
                for (auto& p : parts) {
                    counts.push_back(uint32_t(p.second.size()));
                    rows.insert(rows.end(), p.second.begin(), p.second.end());
                }
                CHECK(!row_parts(n, H, rows.data(), counts.data()).empty());
                Parts cp = parts;
                const FramePlan fp = make_plan(64, H, std::move(cp), true);
                CHECK(!fp.steps.empty());
            }
        }
    }
    // malformed partitions and bands are refused, not read out of bounds
    const uint32_t rows_dup[] = {0, 1, 1, 3}, counts2[] = {2, 2};
    CHECK(row_parts(2, 4, rows_dup, counts2).empty());
    const uint32_t rows_big[] = {0, 1, 2, 9};
    CHECK(row_parts(2, 4, rows_big, counts2).empty());
    const uint32_t short_counts[] = {1, 2};
    CHECK(row_parts(2, 4, rows_big, short_counts).empty());
    const uint32_t bad_start[] = {3, 5}, bad_order[] = {0, 7, 5};
    CHECK(band_parts(2, 10, bad_start, 2).empty());
    CHECK(band_parts(2, 10, bad_order, 3).empty());
}

void check_oracle() {
    const std::vector<Sphere> s = scene(0.0f, 11);
    const uint32_t W = 32, H = 18;
    RenderCallInfo rci;
    std::memset(&rci, 0, sizeof(rci));
    rci.samplesPerRenderCall = 2;
    rci.image_size = rt_uvec2{W, H};
    rci.camera_pos = rt_vec4{13.0f, 11.0f, -3.0f, 0.0f};
    rci.camera_dir = rt_vec4{-13.0f, -11.0f, 3.0f, 0.0f};
    for (uint32_t mode : {0u, 1u, 2u}) {
        rt_options o;
        std::memset(&o, 0, sizeof(o));
        o.rng_mode = mode;
        std::vector<float> acc(size_t(W) * H * 4);
        std::vector<uint8_t> out(size_t(W) * H * 4);
        uint64_t st[3] = {0, 0, 0};
        CHECK(orc_render(s.data(), uint32_t(s.size()), &rci, nullptr, W, H, &o, acc.data(), out.data(), st, 4) == 0);
        CHECK(st[1] == uint64_t(W) * H * 2 && st[0] >= st[1]);
        // a rows map (every third row, reversed) and accumulation on top
        std::vector<uint32_t> rows;
        for (int y = int(H) - 1; y >= 0; y -= 3) rows.push_back(uint32_t(y));
        std::vector<float> bacc(rows.size() * W * 4);
        std::vector<uint8_t> bout(rows.size() * W * 4);
        CHECK(orc_render(s.data(), uint32_t(s.size()), &rci, rows.data(), W, uint32_t(rows.size()), &o, bacc.data(),
                         bout.data(), nullptr, 3) == 0);
        for (size_t i = 0; i < rows.size(); i++)
            CHECK(std::memcmp(&bacc[i * W * 4], &acc[size_t(rows[i]) * W * 4], W * 16) == 0);
        o.accumulate = 1;
        o.sample_base = mode ? 2 : 0;
        CHECK(orc_render(s.data(), uint32_t(s.size()), &rci, nullptr, W, H, &o, acc.data(), out.data(), nullptr, 2) == 0);
        std::vector<uint8_t> res(out.size());
        CHECK(orc_resolve(acc.data(), uint64_t(W) * H, 4, res.data()) == 0);
    }
}

}  // namespace

int main() {
    const float ts[] = {0.0f, 1.3f};
    for (float t : ts) {
        const std::vector<Sphere> s = scene(t, 11);
        CHECK(s.size() == 488);
        check_tree(s, true);
        check_tree(s, false);
    }
    for (uint32_t K : {1u, 2u, 40u}) {
        const std::vector<Sphere> s = scene(0.5f, K);
        check_tree(s, true);
        check_tree(s, false);
    }
    for (const auto& s : edge_scenes()) {
        check_tree(s, true);
        check_tree(s, false);
    }
    {   // config 5: 99 860 spheres, the Morton tree (the device build's host twin) and the grid layout
        const std::vector<Sphere> s = scene(0.0f, 158);
        CHECK(s.size() == 99860);
        check_tree(s, false);
        const float lo[3] = {-158.0f, 0.0f, -158.0f}, hi[3] = {158.0f, 0.4f, 158.0f};
        rt::GridInfo gi;
        uint64_t bound = 0;
        CHECK(rt::grid_layout(lo, hi, 99856, 0.2f, 64.0f * 0x1p-24f * 330.0f, rt::kGridCellScale, gi, &bound));
        CHECK(gi.n_cells > 0 && bound >= 99856);
    }
    check_plans();
    check_oracle();
    std::printf("sanitize harness: %d checks passed (ASan + UBSan)\n", g_checks);
    return 0;
}
