"""The N>1 bench's gather grouping (bench.gather_plan / gather_schedule).

bench.py asserts at run time that the gathers it issued equal gather_schedule; this checks the
schedule itself on CPU: every step's slab goes to rank 0 exactly once, no slot is overwritten
before the gather that carries it was issued, and a region ends with at most about half of its
slabs still to send."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_gather_plan_sizes():
    assert bench.gather_plan(20, 5, 64) == 2  # the driver's region: 4 steps per stream, 2 per group
    assert bench.gather_plan(2000, 5, 64) == 64
    assert bench.gather_plan(1, 5, 64) == 1
    assert bench.gather_plan(0, 5, 64) == 1
    assert bench.gather_plan(7, 1, 64) == 4
    assert bench.gather_plan(100, 5, 3) == 3


@pytest.mark.parametrize("streams", [1, 2, 3, 5])
@pytest.mark.parametrize("steps", [1, 2, 4, 5, 7, 10, 20, 21, 64, 200])
def test_gather_schedule_delivers_every_step_once(steps, streams):
    G = bench.gather_plan(steps, streams, 64)
    sched = bench.gather_schedule(steps, streams, G)
    # replay: slot (stream, group, j) holds the step written last; a gather of (stream, group, k)
    # sends slots j < k of that group
    slot = {}
    sent = []
    ev = sorted(sched, key=lambda e: e[0])
    e = 0
    for i in range(steps):
        si, q = i % streams, i // streams
        g, j = (q // G) % 2, q % G
        assert (si, g, j) not in slot, f"step {i} overwrites slot {(si, g, j)} before it was sent"
        slot[(si, g, j)] = i
        while e < len(ev) and ev[e][0] == i:
            _, s2, g2, k = ev[e]
            for jj in range(k):
                sent.append(slot.pop((s2, g2, jj)))
            e += 1
    tail = 0
    for _, s2, g2, k in ev[e:]:  # the drain
        for jj in range(k):
            sent.append(slot.pop((s2, g2, jj)))
            tail += 1
    assert not slot
    assert sorted(sent) == list(range(steps))
    # the drain carries at most about half the region (one partly filled group per stream)
    assert tail <= streams * G
    if steps >= 4 * streams:
        assert tail <= (steps + 1) // 2 + streams
