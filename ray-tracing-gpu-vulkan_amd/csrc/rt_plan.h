// rt_plan.h — the multi-device frame as host data (no HIP): the row partition over the devices
// and the ordered steps rt_multi executes for one frame. Plain C++ so the CPU tests
// (rt_debug_multi_plan*, rt_partition_*) and the sanitizer build (oracle/Makefile `sanitize`)
// exercise exactly the code rt_multi runs.
//
// Reference: the per-GPU row bands of src/ray_trace.cpp:74-93 (first band takes the remainder)
// and the tuner that moves rows between GPUs from their measured frame times
// (src/workload_tuner.hpp:38-104, fed at src/ray_trace.cpp:750-775). Here the initial split is
// row-exact interleaved strips, and the re-deal is a deterministic greedy move of band-end rows
// from the slowest device to the fastest, driven by per-row cost estimates that every measured
// frame rescales to the device times (no teardown: only rows maps change).
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

namespace rt {
namespace plan {

constexpr uint32_t kStrip = 8;   // rows per strip: one 8x8 pixel tile high, the kernel's wave tile

// A partition: for each part, its device and its global rows in band order.
using Parts = std::vector<std::pair<uint32_t, std::vector<uint32_t>>>;

// Row-exact interleaved strips over n devices (rtvk.dist.strip_rows): the rows below
// R = floor(H / (8 n)) full rounds are 8-row strips dealt round robin (strip k on device k % n);
// the H - 8 n R rows left are cut into n contiguous runs, the first (H - 8 n R) % n one row
// longer, run d on device d. Every device holds floor(H / n) or ceil(H / n) rows.
Parts strip_parts(uint32_t n, uint32_t H);

// The reference's contiguous bands: band i = rows [start[i], start[i+1]) (the last to H), on
// device i % n. Empty when the starts do not tile [0, H) top to bottom.
Parts band_parts(uint32_t n, uint32_t H, const uint32_t* start, uint32_t n_bands);

// An explicit partition of n devices (device d: rows[off_d .. off_d + counts[d]), band order).
// Empty unless every row of [0, H) appears exactly once.
Parts row_parts(uint32_t n, uint32_t H, const uint32_t* rows, const uint32_t* counts);

// ---- the frame plan --------------------------------------------------------------------
// Buffers a step names: the caller's accumulator / rgba8 image on device 0 (W x H), each part's
// band on its device (rows x W), and each remote part's stage on device 0 (rows x W float4).
enum PlanOp : uint32_t {
    OP_LOAD_ROWS = 1,   // device 0: the part's rows of the caller's accumulator -> its band (a part
                        // of device 0) or its stage (accumulating frames: the running sums)
    OP_GROUP_START = 2, // ncclGroupStart
    OP_SEND = 3,        // dev -> peer: `count` floats of the part's band (dev != 0) or stage (dev 0)
    OP_RECV = 4,        // dev <- peer: `count` floats into the part's band (dev != 0) or stage (dev 0)
    OP_GROUP_END = 5,   // ncclGroupEnd
    OP_RENDER = 6,      // dev renders the part; flags bit 0: straight into the caller's buffers
    OP_STORE_ROWS = 7,  // device 0: the part's band (device 0) or stage -> its rows of the accumulator
    OP_RESOLVE = 8,     // device 0: rgba8 of the whole accumulator (`count` texels)
};
constexpr uint32_t kDirect = 1u;

struct PlanPart {
    uint32_t dev = 0;
    std::vector<uint32_t> rows;   // global rows, band order
    bool whole = false;           // device 0, every row in order: renders into the caller's buffers
};
struct PlanStep {
    uint32_t op, dev, peer, part, flags;
    uint64_t count;
};
struct FramePlan {
    std::vector<PlanPart> parts;
    std::vector<PlanStep> steps;
};

// The steps of one frame over `parts` (W x H), with or without accumulation (rt_multi.cpp).
FramePlan make_plan(uint32_t W, uint32_t H, Parts&& parts, bool accumulate);

// Flat form (rt_debug_multi_plan): {n_parts, n_steps}, per part {dev, whole, n_rows, rows...},
// per step {op, dev, peer, part, flags, count low, count high}.
std::vector<uint32_t> serialize(const FramePlan& p);

// ---- cross-device balancing ------------------------------------------------------------
// Per-row cost estimates (same unit as the measured device times; <= 0: unknown). With weights
// (per part, one per band row of the measured frame, e.g. rt_launch_row_weights; an empty or
// all-zero vector: none), a measured part's rows get its time split in proportion to them.
// Without, they are rescaled so that they sum to its time, a row never measured taking the mean
// of its part's known rows (all unknown: the time spread evenly). blend < 1: a known row keeps
// (1 - blend) of its previous estimate (an exponential average over frames: per-frame kernel times
// vary by a few tenths of a percent, which a re-deal should not chase).
void update_costs(const Parts& measured, const float* device_ms, std::vector<double>& cost,
                  const std::vector<std::vector<double>>* weights = nullptr, double blend = 1.0);

// While the most loaded device is more than (1 + tolerance) x the mean load, applies the exchange
// with another device that leaves the larger of the pair's loads lowest, if it is below the most
// loaded device's load (so every step lowers the sum of squared loads): a MOVE
// of one of the donor's last min(8, rows) band rows (its last tile row, so the band's other tiles
// keep their index and their LPT cost record) to the end of the receiver's band, or a SWAP of one
// such row with one of the receiver's last rows (finer than one row), when it lowers the most
// loaded device's load by more than tolerance x the mean load. Deterministic (ties to the lowest
// index). Returns the rows moved (a swap moves two); loads_out (optional, per part)
// receives the predicted loads afterwards.
uint32_t rebalance(Parts& parts, const std::vector<double>& cost, double tolerance, std::vector<double>* loads_out);

// max / mean of the parts' loads under `cost` (1 when every load is 0).
double imbalance(const Parts& parts, const std::vector<double>& cost);

}  // namespace plan
}  // namespace rt
