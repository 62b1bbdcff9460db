// rt_plan.cpp — row partitions, the multi-device frame plan and the cross-device balancer
// (rt_plan.h). Host-only C++, no HIP.
#include "rt_plan.h"

#include <algorithm>
#include <cmath>

namespace rt {
namespace plan {

Parts strip_parts(uint32_t n, uint32_t H) {
    Parts parts(n);
    for (uint32_t d = 0; d < n; d++) parts[d].first = d;
    if (n == 0) return parts;
    const uint64_t round = uint64_t(kStrip) * n;
    const uint32_t y0 = uint32_t((H / round) * round);   // rows of the full rounds of strips
    for (uint32_t y = 0; y < y0; y++) parts[(y / kStrip) % n].second.push_back(y);
    // the rest (< 8 n rows): n contiguous runs, the first (rest % n) one row longer
    const uint32_t rest = H - y0, base = rest / n, extra = rest % n;
    uint32_t y = y0;
    for (uint32_t d = 0; d < n; d++)
        for (uint32_t k = 0; k < base + (d < extra ? 1u : 0u); k++) parts[d].second.push_back(y++);
    return parts;
}

Parts band_parts(uint32_t n, uint32_t H, const uint32_t* start, uint32_t n_bands) {
    Parts parts(n_bands);
    for (uint32_t i = 0; i < n_bands; i++) {
        const uint32_t y0 = start[i], y1 = i + 1 < n_bands ? start[i + 1] : H;
        if (y1 < y0 || y1 > H || (i == 0 && y0 != 0)) return Parts{};
        parts[i].first = i % n;
        for (uint32_t y = y0; y < y1; y++) parts[i].second.push_back(y);
    }
    return parts;
}

Parts row_parts(uint32_t n, uint32_t H, const uint32_t* rows, const uint32_t* counts) {
    Parts parts(n);
    std::vector<uint8_t> seen(H, 0);
    uint64_t at = 0;
    for (uint32_t d = 0; d < n; d++) {
        parts[d].first = d;
        for (uint32_t k = 0; k < counts[d]; k++, at++) {
            const uint32_t y = rows[at];
            if (y >= H || seen[y]) return Parts{};
            seen[y] = 1;
            parts[d].second.push_back(y);
        }
    }
    return at == H ? parts : Parts{};
}

// accumulate: every part starts from its rows of the caller's accumulator (rt_render_device's
// accumulate semantics for the whole image, at any device count): device 0 loads them into its
// own bands and into the stages of the other devices' parts, and sends those in one group. Then
// every part renders; one group brings the other devices' accumulator bands to device 0's stages;
// device 0 stores every band in place and tonemaps the whole image. A part of device 0 never goes
// through RCCL; a `whole` part renders into the caller's buffers and needs nothing else (the
// one-device frame).
FramePlan make_plan(uint32_t W, uint32_t H, Parts&& parts, bool accumulate) {
    FramePlan p;
    for (auto& pr : parts) {
        PlanPart q;
        q.dev = pr.first;
        q.rows = std::move(pr.second);
        q.whole = q.dev == 0 && q.rows.size() == H;
        for (uint32_t y = 0; q.whole && y < H; y++) q.whole = q.rows[y] == y;
        p.parts.push_back(std::move(q));
    }
    const uint32_t np = uint32_t(p.parts.size());
    auto live = [&](uint32_t i) { return !p.parts[i].rows.empty(); };
    auto floats = [&](uint32_t i) { return uint64_t(p.parts[i].rows.size()) * W * 4u; };
    auto add = [&](uint32_t op, uint32_t dev, uint32_t peer, uint32_t part, uint32_t flags, uint64_t count) {
        p.steps.push_back(PlanStep{op, dev, peer, part, flags, count});
    };
    bool whole = false, remote = false;
    for (uint32_t i = 0; i < np; i++) {
        whole |= live(i) && p.parts[i].whole;
        remote |= live(i) && p.parts[i].dev != 0;
    }
    if (accumulate && !whole) {
        for (uint32_t i = 0; i < np; i++)
            if (live(i)) add(OP_LOAD_ROWS, 0, 0, i, 0, floats(i));
        if (remote) {
            add(OP_GROUP_START, 0, 0, 0, 0, 0);
            for (uint32_t i = 0; i < np; i++) {
                if (!live(i) || p.parts[i].dev == 0) continue;
                add(OP_SEND, 0, p.parts[i].dev, i, 0, floats(i));
                add(OP_RECV, p.parts[i].dev, 0, i, 0, floats(i));
            }
            add(OP_GROUP_END, 0, 0, 0, 0, 0);
        }
    }
    for (uint32_t i = 0; i < np; i++)
        if (live(i)) add(OP_RENDER, p.parts[i].dev, p.parts[i].dev, i, p.parts[i].whole ? kDirect : 0u, 0);
    if (whole) return p;
    if (remote) {
        add(OP_GROUP_START, 0, 0, 0, 0, 0);
        for (uint32_t i = 0; i < np; i++) {
            if (!live(i) || p.parts[i].dev == 0) continue;
            add(OP_SEND, p.parts[i].dev, 0, i, 0, floats(i));
            add(OP_RECV, 0, p.parts[i].dev, i, 0, floats(i));
        }
        add(OP_GROUP_END, 0, 0, 0, 0, 0);
    }
    for (uint32_t i = 0; i < np; i++)
        if (live(i)) add(OP_STORE_ROWS, 0, 0, i, 0, floats(i));
    add(OP_RESOLVE, 0, 0, 0, 0, uint64_t(W) * H);
    return p;
}

std::vector<uint32_t> serialize(const FramePlan& p) {
    std::vector<uint32_t> v{uint32_t(p.parts.size()), uint32_t(p.steps.size())};
    for (const PlanPart& q : p.parts) {
        v.push_back(q.dev);
        v.push_back(q.whole ? 1u : 0u);
        v.push_back(uint32_t(q.rows.size()));
        v.insert(v.end(), q.rows.begin(), q.rows.end());
    }
    for (const PlanStep& s : p.steps) {
        const uint32_t w[7] = {s.op, s.dev, s.peer, s.part, s.flags, uint32_t(s.count), uint32_t(s.count >> 32)};
        v.insert(v.end(), w, w + 7);
    }
    return v;
}

void update_costs(const Parts& measured, const float* device_ms, std::vector<double>& cost,
                  const std::vector<std::vector<double>>* weights, double blend) {
    const double keep = blend >= 1.0 || !(blend > 0.0) ? 0.0 : 1.0 - blend;
    auto set = [&](uint32_t y, double v) { cost[y] = cost[y] > 0.0 && keep > 0.0 ? keep * cost[y] + (1.0 - keep) * v : v; };
    for (size_t i = 0; i < measured.size(); i++) {
        const std::vector<uint32_t>& rows = measured[i].second;
        const double t = double(device_ms[i]);
        if (rows.empty() || !(t > 0.0) || !std::isfinite(t)) continue;
        if (weights && i < weights->size() && (*weights)[i].size() == rows.size()) {
            const std::vector<double>& w = (*weights)[i];
            double sw = 0.0;
            for (double v : w) sw += std::isfinite(v) && v > 0.0 ? v : 0.0;
            if (sw > 0.0) {
                // a row of weight 0 (a tile row that traced nothing) still costs its share of the
                // launch's fixed work: floor each row at 1 % of the mean
                const double floor_w = 0.01 * sw / double(rows.size());
                double sf = 0.0;
                for (double v : w) sf += std::max(floor_w, std::isfinite(v) ? v : 0.0);
                for (size_t k = 0; k < rows.size(); k++)
                    if (rows[k] < cost.size()) set(rows[k], t * std::max(floor_w, std::isfinite(w[k]) ? w[k] : 0.0) / sf);
                continue;
            }
        }
        double known = 0.0;
        size_t n_known = 0;
        for (uint32_t y : rows)
            if (y < cost.size() && cost[y] > 0.0) {
                known += cost[y];
                n_known++;
            }
        // unknown rows at the mean of the known ones (all unknown: the time spread evenly)
        const double fill = n_known ? known / double(n_known) : 1.0;
        const double est = known + fill * double(rows.size() - n_known);
        const double scale = t / est;
        for (uint32_t y : rows) {   // (the time alone: the rescale is the estimate, no average)
            if (y >= cost.size()) continue;
            cost[y] = (cost[y] > 0.0 ? cost[y] : fill) * scale;
        }
    }
}

namespace {
std::vector<double> part_loads(const Parts& parts, const std::vector<double>& cost) {
    std::vector<double> L(parts.size(), 0.0);
    for (size_t i = 0; i < parts.size(); i++)
        for (uint32_t y : parts[i].second) L[i] += y < cost.size() ? std::max(0.0, cost[y]) : 0.0;
    return L;
}
}  // namespace

double imbalance(const Parts& parts, const std::vector<double>& cost) {
    const std::vector<double> L = part_loads(parts, cost);
    if (L.empty()) return 1.0;
    double sum = 0.0, mx = 0.0;
    for (double v : L) {
        sum += v;
        mx = std::max(mx, v);
    }
    return sum > 0.0 ? mx / (sum / double(L.size())) : 1.0;
}

uint32_t rebalance(Parts& parts, const std::vector<double>& cost, double tolerance, std::vector<double>* loads_out) {
    std::vector<double> L = part_loads(parts, cost);
    const size_t np = parts.size();
    uint32_t moved = 0;
    if (np > 1) {
        double sum = 0.0;
        for (double v : L) sum += v;
        const double mean = sum / double(np);
        auto c = [&](uint32_t y) { return y < cost.size() ? std::max(0.0, cost[y]) : 0.0; };
        auto tail = [](const std::vector<uint32_t>& v) { return v.size() > kStrip ? v.size() - kStrip : size_t(0); };
        // each exchange strictly lowers the sum of squared loads, so this ends; the cap is a guard
        for (size_t guard = 0; guard < 4 * cost.size() + 16; guard++) {
            size_t hi = 0;
            for (size_t i = 1; i < np; i++)
                if (L[i] > L[hi]) hi = i;
            if (!(L[hi] > mean * (1.0 + tolerance))) break;
            std::vector<uint32_t>& src = parts[hi].second;
            // the exchange with any other device that leaves the larger of the pair's loads lowest
            size_t best_j = np, best_a = 0, best_b = 0;   // best_b == rows of j: a move
            double best_max = L[hi] - std::max(tolerance * mean, L[hi] * 1e-12);
            for (size_t j = 0; j < np; j++) {
                if (j == hi) continue;
                const std::vector<uint32_t>& dst = parts[j].second;
                for (size_t a = tail(src); a < src.size(); a++) {
                    const double wa = c(src[a]);
                    const double m = std::max(L[hi] - wa, L[j] + wa);
                    if (m < best_max) {
                        best_max = m;
                        best_j = j;
                        best_a = a;
                        best_b = dst.size();
                    }
                    for (size_t b = tail(dst); b < dst.size(); b++) {
                        const double d = wa - c(dst[b]);
                        if (!(d > 0.0)) continue;
                        const double ms = std::max(L[hi] - d, L[j] + d);
                        if (ms < best_max) {
                            best_max = ms;
                            best_j = j;
                            best_a = a;
                            best_b = b;
                        }
                    }
                }
            }
            if (best_j == np) break;
            std::vector<uint32_t>& dst = parts[best_j].second;
            const uint32_t ya = src[best_a];
            src.erase(src.begin() + std::ptrdiff_t(best_a));
            if (best_b != dst.size()) {   // swap: the receiver's row goes to the end of the donor's band
                const uint32_t yb = dst[best_b];
                dst.erase(dst.begin() + std::ptrdiff_t(best_b));
                src.push_back(yb);
                L[hi] += c(yb);
                L[best_j] -= c(yb);
                moved++;
            }
            dst.push_back(ya);
            L[hi] -= c(ya);
            L[best_j] += c(ya);
            moved++;
        }
    }
    if (loads_out) *loads_out = L;
    return moved;
}

}  // namespace plan
}  // namespace rt
