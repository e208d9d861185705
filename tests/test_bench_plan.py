"""The N>1 bench's gather rounds (bench.gather_plan / gather_schedule).

bench.py asserts at run time that the gathers it issued equal gather_schedule; this checks the
schedule itself on CPU: every step's slab goes to rank 0 exactly once, no slab is overwritten
before the round that carries it was sent, and the region ends with a short round in flight."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_gather_plan_sizes():
    assert bench.gather_plan(20, 64, 5) == [10, 5, 5]  # the driver's region
    assert bench.gather_plan(1, 64, 5) == [1]
    assert bench.gather_plan(0, 64, 5) == []
    p = bench.gather_plan(2000, 64, 5)
    assert sum(p) == 2000 and max(p) == 64 and p[-1] == 5 and len(p) <= 2000 // 64 + 8
    assert bench.gather_plan(100, 3, 5)[:3] == [3, 3, 3]


@pytest.mark.parametrize("streams", [1, 5])
@pytest.mark.parametrize("every", [1, 3, 64])
@pytest.mark.parametrize("steps", [1, 2, 4, 5, 7, 10, 20, 21, 64, 200, 2000])
def test_gather_schedule_delivers_every_step_once(steps, every, streams):
    rounds = bench.gather_plan(steps, every, streams)
    assert sum(rounds) == steps and all(1 <= r <= every for r in rounds)
    # at most one round below the floor (the last: a region's remainder under the cap)
    assert sum(r < min(streams, every) for r in rounds) <= 1
    assert all(r >= min(streams, every) for r in rounds[:-1])
    sched = bench.gather_schedule(rounds)
    ev = {e[0]: e for e in sched}
    assert len(ev) == len(sched) == len(rounds)
    slot, sent, r = {}, [], 0
    for k, n in enumerate(rounds):
        for j in range(n):
            b = k % 2
            assert (b, j) not in slot, f"step {r} overwrites slab {(b, j)} before it was sent"
            slot[(b, j)] = r
            if r in ev:
                _, b2, m = ev[r]
                assert b2 == b and m == n
                for jj in range(m):
                    sent.append(slot.pop((b2, jj)))
            r += 1
    assert not slot and sorted(sent) == list(range(steps))
    assert sched[-1][2] <= max(min(streams, every), 1) * 2  # a short last round
