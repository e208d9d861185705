"""The N>1 bench's gather rounds (bench.gather_plan / gather_schedule).

bench.py asserts at run time that the gathers it issued equal gather_schedule; this checks the
schedule itself on CPU: every step's slab goes to rank 0 exactly once, no slab is overwritten
before the gather that carries it was issued, and a region ends with at most about half of its
slabs still to send."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_gather_plan_sizes():
    assert bench.gather_plan(20, 5, 64) == 10  # the driver's region: two rounds of 10 steps
    assert bench.gather_plan(2000, 5, 64) == 64
    assert bench.gather_plan(1, 5, 64) == 5
    assert bench.gather_plan(0, 5, 64) == 5
    assert bench.gather_plan(7, 1, 64) == 4
    assert bench.gather_plan(100, 5, 3) == 3


@pytest.mark.parametrize("streams", [1, 2, 3, 5])
@pytest.mark.parametrize("steps", [1, 2, 4, 5, 7, 10, 20, 21, 64, 200])
def test_gather_schedule_delivers_every_step_once(steps, streams):
    R = bench.gather_plan(steps, streams, 64)
    sched = bench.gather_schedule(steps, R)
    slot = {}
    sent = []
    ev = {e[0]: e for e in sched}
    assert len(ev) == len(sched)
    for r in range(steps):
        b, j = (r // R) % 2, r % R
        assert (b, j) not in slot, f"step {r} overwrites slab {(b, j)} before it was sent"
        slot[(b, j)] = r
        if r in ev:
            _, b2, m = ev[r]
            assert b2 == b
            for jj in range(m):
                sent.append(slot.pop((b2, jj)))
    assert not slot
    assert sorted(sent) == list(range(steps))
    # the last gather carries at most about half the region
    assert sched[-1][2] <= max(streams, (steps + 1) // 2)
    if steps >= 2 * streams:
        assert len(sched) <= max(2, -(-steps // 64))  # few collectives: 2 per region up to 128 steps
