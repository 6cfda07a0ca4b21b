"""tools/block_sim.py, the replay of dist.BlockSync's dependencies that turns
measured cell times into the predicted N-GPU epoch: equal
cells never stall, a transfer longer than a cell stalls the ring, and one slow
block stalls its neighbours only when its excess exceeds the two-block slack."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import block_sim  # noqa: E402


def _uniform(n, ms):
    return [[ms] * (2 * n) for _ in range(n)]


def test_equal_cells_no_stall():
    for n in (2, 4, 8):
        ep = block_sim.simulate(n, _uniform(n, 7.0), 2.5)
        assert abs(ep - 2 * n * 7.0) < 1e-9


def test_transfer_longer_than_a_cell_stalls():
    n = 4
    # a rotation must land before the cell two sub-rounds later: with a
    # transfer of 3 cells the ring runs at one transfer per sub-round pair
    ep = block_sim.simulate(n, _uniform(n, 1.0), 3.0)
    assert ep > 2 * n * 1.0 + 1.0


def test_one_slow_block():
    n = 8
    d = _uniform(n, 7.0)
    for r in range(n):
        d[r][10] = 8.0      # within the slack: no stall
    ep = block_sim.simulate(n, d, 2.5)
    assert abs(ep - (15 * 7.0 + 8.0)) < 1e-6
    for r in range(n):
        d[r][10] = 30.0     # far beyond it: the epoch grows past every rank's own sum
    ep = block_sim.simulate(n, d, 2.5)
    assert ep > 15 * 7.0 + 30.0 + 1.0
