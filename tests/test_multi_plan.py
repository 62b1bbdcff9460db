"""The multi-GPU frame plan of rt_multi (csrc/rt_multi.cpp make_plan), checked on the CPU for the
device counts and heights config 4 and its neighbours use: the plan is the exact list of steps
rt_multi_render / rt_render execute (rt_debug_multi_plan serialises the same FramePlan), so these
tests cover the N > 1 logic that a one-GPU box never runs.

Reference: the bands of src/ray_trace.cpp:74-93 (rt_render) and the per-GPU row split the
reference records per benchmark window (:750-760) and re-deals (src/workload_tuner.hpp:38-104);
here row-exact interleaved strips (rtvk.dist.strip_rows, rt_partition_strips) re-dealt by
rt_partition_rebalance (rt_multi_render, rtvk.dist)."""
import numpy as np
import pytest

from rtvk.dist import strip_rows

NS = [1, 2, 3, 4, 8]
HS = [7, 27, 1080, 2160]


@pytest.fixture(scope="module")
def rtvk():
    import rtvk as m
    m.load_library()
    return m


def groups(steps):
    """Send / receive steps per RCCL group, in order."""
    out, cur = [], None
    for s in steps:
        if s["op"] == "group_start":
            assert cur is None, "nested group"
            cur = []
        elif s["op"] == "group_end":
            assert cur is not None, "group end without start"
            out.append(cur)
            cur = None
        elif s["op"] in ("send", "recv"):
            assert cur is not None, "send / receive outside a group"
            cur.append(s)
        else:
            assert cur is None, f"{s['op']} inside an RCCL group"
    assert cur is None, "unterminated group"
    return out


def simulate(plan, W, H, n, accumulate, acc_in, frame):
    """Executes a plan on per-device numpy buffers. A render adds `frame` (the rows' new samples)
    to its band when accumulating, else stores it; returns the caller's (accumulator, resolved)
    after the frame, or raises on a step that reads a buffer nobody wrote."""
    parts = plan["parts"]
    acc = acc_in.copy()
    resolved = np.zeros(H, bool)
    band = {}    # part -> band on its device
    stage = {}   # part -> stage on device 0
    direct_rows = None
    for g in groups(plan["steps"]):   # every send has one receive in its group: pair them
        sends = [(s["dev"], s["peer"], s["part"], s["count"]) for s in g if s["op"] == "send"]
        recvs = [(s["peer"], s["dev"], s["part"], s["count"]) for s in g if s["op"] == "recv"]
        assert sorted(sends) == sorted(recvs), "unmatched send / receive"
    pending = {}   # (src, dst, part) -> data in flight in the current group
    for s in plan["steps"]:
        op, p = s["op"], s["part"]
        dev, rows = parts[p][0], parts[p][2]
        if op == "load_rows":
            assert s["dev"] == 0
            (band if dev == 0 else stage)[p] = acc[rows].copy()
        elif op == "send":
            assert s["dev"] != s["peer"], "a device sends to itself"
            buf = stage[p] if s["dev"] == 0 else band[p]
            assert buf.size == s["count"], "count differs from the buffer"
            pending[(s["dev"], s["peer"], p)] = buf.copy()
        elif op == "recv":
            data = pending.pop((s["peer"], s["dev"], p))
            assert data.size == s["count"]
            if s["dev"] == 0:
                stage[p] = data
            else:
                band[p] = data
        elif op == "render":
            assert s["dev"] == dev
            if s["flags"] & 1:   # straight into the caller's buffers
                assert parts[p][1] and dev == 0 and np.array_equal(rows, np.arange(H))
                acc = acc + frame if accumulate else frame.copy()
                direct_rows = rows
            else:
                new = frame[rows]
                band[p] = band[p] + new if accumulate else new.copy()
        elif op == "store_rows":
            assert s["dev"] == 0
            acc[rows] = band[p] if dev == 0 else stage[p]
        elif op == "resolve":
            assert s["dev"] == 0 and s["count"] == W * H
            resolved[:] = True
    assert not pending
    if direct_rows is not None:
        resolved[:] = True   # the kernel stored rgba8 itself
    return acc, resolved


@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("H", HS)
@pytest.mark.parametrize("accumulate", [False, True])
def test_strip_plan(rtvk, n, H, accumulate):
    W = 1920
    plan = rtvk.multi_plan(n, W, H, accumulate=accumulate)
    parts = plan["parts"]
    # one part per device, its rows exactly rtvk.dist.strip_rows (the per-process path's split)
    assert [p[0] for p in parts] == list(range(n))
    for d, (dev, whole, rows) in enumerate(parts):
        np.testing.assert_array_equal(rows, strip_rows(d, n, H))
        assert whole == (len(rows) == H)   # one device holds every row (n = 1, or H <= 8)
    allrows = np.concatenate([p[2] for p in parts])
    assert sorted(allrows.tolist()) == list(range(H)), "every row exactly once"
    steps = plan["steps"]
    live = [i for i, p in enumerate(parts) if len(p[2])]
    # renders: one per part that holds rows, on its own device
    assert sorted(s["part"] for s in steps if s["op"] == "render") == live
    sends = [s for s in steps if s["op"] == "send"]
    assert all(s["dev"] != s["peer"] for s in sends), "device 0 never sends to itself"
    assert all(s["count"] == len(parts[s["part"]][2]) * W * 4 for s in sends)
    # gather: every remote part's accumulator exactly once to device 0 (no rgba8 travels)
    gathered = sorted(s["part"] for s in sends if s["peer"] == 0)
    assert gathered == [i for i in live if parts[i][0] != 0]
    # distribution before the frame only when accumulating
    scattered = sorted(s["part"] for s in sends if s["dev"] == 0)
    assert scattered == ([i for i in live if parts[i][0] != 0] if accumulate else [])
    if len(parts[0][2]) == H:   # one device: renders straight into the caller's buffers, nothing else
        assert [s["op"] for s in steps] == ["render"] and steps[0]["flags"] == 1
    else:
        assert sum(s["op"] == "resolve" for s in steps) == 1 and steps[-1]["op"] == "resolve"
        stores = sorted(s["part"] for s in steps if s["op"] == "store_rows")
        assert stores == live
    # executing it gives every row the frame's samples (+ the caller's running sums)
    rng = np.random.default_rng(n * 10000 + H)
    acc0 = rng.integers(0, 1000, (H, 1, 4)).astype(np.float64) if accumulate else np.full((H, 1, 4), np.nan)
    frame = rng.integers(0, 1000, (H, 1, 4)).astype(np.float64)
    plan_w1 = rtvk.multi_plan(n, 1, H, accumulate=accumulate)   # same plan at width 1 (counts scale)
    acc, resolved = simulate(plan_w1, 1, H, n, accumulate, acc0, frame)
    np.testing.assert_array_equal(acc, acc0 + frame if accumulate else frame)
    assert resolved.all()


def test_step_order(rtvk):
    """Per remote part: receive its running sums, render, send, then device 0 stores it and
    resolves once after every store."""
    plan = rtvk.multi_plan(8, 64, 1080, accumulate=True)
    steps = plan["steps"]
    idx = {}
    for i, s in enumerate(steps):
        idx.setdefault((s["op"], s["dev"], s["part"]), []).append(i)
    resolve = idx[("resolve", 0, 0)][0]
    for p, (dev, _, rows) in enumerate(plan["parts"]):
        if dev == 0:
            assert idx[("load_rows", 0, p)][0] < idx[("render", 0, p)][0] < idx[("store_rows", 0, p)][0] < resolve
            continue
        load, = idx[("load_rows", 0, p)]
        send0, = idx[("send", 0, p)]
        recv_d, = idx[("recv", dev, p)]
        render, = idx[("render", dev, p)]
        send_d, = idx[("send", dev, p)]
        recv0, = idx[("recv", 0, p)]
        store, = idx[("store_rows", 0, p)]
        assert load < send0 and recv_d < render < send_d and recv0 < store < resolve


@pytest.mark.parametrize("n,starts,H", [(1, [0, 7, 13], 20), (2, [0, 7, 13], 20), (3, [0, 360, 720], 1080),
                                          (8, [0, 135, 270, 405, 540, 675, 810, 945], 1080), (2, [0], 5)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_band_plan(rtvk, n, starts, H, accumulate):
    """rt_render's contiguous bands (src/ray_trace.cpp:74-93): band i on device i % n."""
    plan = rtvk.multi_plan(n, 1, H, band_starts=starts, accumulate=accumulate)
    parts = plan["parts"]
    assert len(parts) == len(starts)
    for i, (dev, whole, rows) in enumerate(parts):
        y1 = starts[i + 1] if i + 1 < len(starts) else H
        np.testing.assert_array_equal(rows, np.arange(starts[i], y1))
        assert dev == i % n
        assert whole == (len(starts) == 1)
    rng = np.random.default_rng(len(starts) * 100 + n)
    acc0 = rng.integers(0, 1000, (H, 1, 4)).astype(np.float64) if accumulate else np.full((H, 1, 4), np.nan)
    frame = rng.integers(0, 1000, (H, 1, 4)).astype(np.float64)
    acc, resolved = simulate(plan, 1, H, n, accumulate, acc0, frame)
    np.testing.assert_array_equal(acc, acc0 + frame if accumulate else frame)
    assert resolved.all()


def test_plan_rejects_bad_bands(rtvk):
    with pytest.raises(rtvk.RtError):
        rtvk.multi_plan(2, 8, 10, band_starts=[3, 5])   # does not start at row 0
    with pytest.raises(rtvk.RtError):
        rtvk.multi_plan(2, 8, 10, band_starts=[0, 7, 5])   # not top to bottom
    with pytest.raises(rtvk.RtError):
        rtvk.multi_plan(0, 8, 10)


def test_gather_bytes_config4(rtvk):
    """Config 4 (1920x1080 on 8 GPUs): the gather moves only the float4 accumulators of the 7
    remote devices, 7/8 of 33.2 MB (round 4 also sent the rgba8 bands: 20 % more bytes, twice the
    RCCL operations)."""
    plan = rtvk.multi_plan(8, 1920, 1080)
    sends = [s for s in plan["steps"] if s["op"] == "send"]
    assert len(sends) == 7
    assert sum(s["count"] for s in sends) * 4 == 1920 * (1080 - len(strip_rows(0, 8, 1080))) * 16


def random_partition(rng, n, H):
    """Every row once, in a random order, over n devices (some possibly empty)."""
    perm = rng.permutation(H).astype(np.uint32)
    cuts = np.sort(rng.integers(0, H + 1, n - 1))
    return [perm[a:b] for a, b in zip(np.r_[0, cuts], np.r_[cuts, H])]


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("H", [5, 27, 1080])
@pytest.mark.parametrize("accumulate", [False, True])
def test_plan_for_arbitrary_rows(rtvk, n, H, accumulate):
    """Any partition (a re-dealt one: rows in any order, devices of any size, empty ones): the plan
    keeps each device's rows in band order, pairs every send with one receive, and its numpy
    execution reproduces the frame (+ the running sums)."""
    rng = np.random.default_rng(n * 7919 + H + accumulate)
    for trial in range(3):
        parts = random_partition(rng, n, H)
        plan = rtvk.multi_plan(n, 1, H, accumulate=accumulate, parts=parts)
        assert len(plan["parts"]) == n
        for d, (dev, whole, rows) in enumerate(plan["parts"]):
            assert dev == d
            np.testing.assert_array_equal(rows, parts[d])
        live = [i for i, p in enumerate(plan["parts"]) if len(p[2])]
        assert sorted(s["part"] for s in plan["steps"] if s["op"] == "render") == live
        assert all(s["dev"] != s["peer"] for s in plan["steps"] if s["op"] == "send")
        acc0 = rng.integers(0, 1000, (H, 1, 4)).astype(np.float64) if accumulate else np.full((H, 1, 4), np.nan)
        frame = rng.integers(0, 1000, (H, 1, 4)).astype(np.float64)
        acc, resolved = simulate(plan, 1, H, n, accumulate, acc0, frame)
        np.testing.assert_array_equal(acc, acc0 + frame if accumulate else frame)
        assert resolved.all()


def test_plan_rows_rejects_bad_partitions(rtvk):
    with pytest.raises(rtvk.RtError):
        rtvk.multi_plan(2, 4, 6, parts=[np.array([0, 1, 2]), np.array([2, 3, 4, 5])])   # row 2 twice
    with pytest.raises(rtvk.RtError):
        rtvk.multi_plan(2, 4, 6, parts=[np.array([0, 1, 2]), np.array([3, 4])])          # row 5 missing
    with pytest.raises(rtvk.RtError):
        rtvk.multi_plan(2, 4, 6, parts=[np.array([0, 1, 2]), np.array([3, 4, 9])])       # row 9 of 6


def loads(parts, cost):
    return np.array([cost[p].sum() for p in parts])


@pytest.mark.parametrize("n,H", [(2, 1080), (3, 1080), (8, 1080), (8, 2160), (7, 1080), (8, 27), (8, 7)])
def test_rebalance_properties(rtvk, n, H):
    """rt_partition_rebalance: every row still once; rows leave only from a band's last 8 rows (a
    device that gives k rows changes from index len - 8 - k on) and join at its end, so every other
    tile keeps its index and LPT record; each step lowers the most loaded device's load;
    deterministic; a balanced partition is left alone."""
    rng = np.random.default_rng(n * 31 + H)
    parts = rtvk.partition_strips(n, H)
    true = 1.0 + rng.random(H) * 2.0   # per-row ms, sky-to-sphere spread
    cost = true.copy()
    prev_max = loads(parts, cost).max()
    for it in range(6):
        before = [p.copy() for p in parts]
        new, moved, pred = rtvk.partition_rebalance(parts, cost, tolerance=0.0)
        again, moved2, pred2 = rtvk.partition_rebalance(before, cost.copy(), tolerance=0.0)
        for a, b in zip(new, again):   # deterministic
            np.testing.assert_array_equal(a, b)
        assert (moved, pred) == (moved2, pred2)
        assert sorted(np.concatenate(new).tolist()) == list(range(H))
        for old, nw in zip(before, new):
            gave = len(set(old.tolist()) - set(nw.tolist()))
            keep = max(0, len(old) - 8 - gave) if gave else len(old)
            np.testing.assert_array_equal(nw[:keep], old[:keep])
        L = loads(new, cost)
        assert L.max() <= prev_max + 1e-9
        assert pred == pytest.approx(L.max() / L.mean(), rel=1e-9)
        prev_max = L.max()
        parts = new
        if not moved:
            break
    if H >= 8 * n:   # enough rows: within one row's cost of the mean
        L = loads(parts, cost)
        assert L.max() - L.mean() <= true.max() + 1e-9


def test_rebalance_measured_feedback(rtvk):
    """Config 4's shape: the device times of round 5's N = 8 band probe (rank 7 faster) fed as a
    measurement of the row-exact strips: rows leave the slow devices, the predicted imbalance drops
    below the measured one, and an even measurement moves nothing."""
    parts = rtvk.partition_strips(8, 1080)
    ms = [139.0, 138.5, 138.7, 139.2, 138.4, 138.9, 139.1, 131.4]
    cost = np.zeros(1080)
    new, moved, pred = rtvk.partition_rebalance(parts, cost, measured=parts, device_ms=ms)
    assert moved > 0 and pred < max(ms) / np.mean(ms)
    for p, t in zip(parts, ms):   # the estimates sum to each device's measured time
        assert cost[p].sum() == pytest.approx(float(np.float32(t)), rel=1e-9)   # times travel as f32
    assert len(new[7]) > len(parts[7])
    cost2 = np.zeros(1080)
    same, moved0, pred0 = rtvk.partition_rebalance(parts, cost2, measured=parts, device_ms=[100.0] * 8)
    assert moved0 == 0 and pred0 == pytest.approx(1.0)
    for a, b in zip(same, parts):
        np.testing.assert_array_equal(a, b)


def test_rebalance_rejects_bad_input(rtvk):
    parts = rtvk.partition_strips(2, 16)
    dup = parts[1].copy()
    dup[-1] = parts[0][0]
    with pytest.raises(rtvk.RtError):
        rtvk.partition_rebalance([parts[0], dup], np.zeros(16))               # a row twice, one missing
    with pytest.raises(ValueError):
        rtvk.partition_rebalance([parts[0], parts[1][:-1]], np.zeros(16))     # a row missing
    with pytest.raises(ValueError):
        rtvk.partition_rebalance(parts, np.zeros(16, np.float32))             # cost not float64
