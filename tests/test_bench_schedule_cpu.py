"""bench.py's step schedule (run_step) without a GPU: which global samples each
rank trains per step, and where the replica exchanges sit."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class FakeProNet:
    def __init__(self, log):
        self.log = log

    def train_edges(self, model, begin, count, total, K, alpha, reg, seed, mode, sync=False):
        assert model == "line2" and not sync
        self.log.append(("train", begin, count))


class FakeSync:
    def __init__(self, log, hot=False):
        self.log = log
        self.hot_idx = [object()] if hot else []

    def begin(self):
        self.log.append(("begin",))

    def hot(self):
        self.log.append(("hot",))


def _run(world, rank, steps, S, n_launch, n_ex, sync_every=1, hot=False, with_sync=True):
    log = []
    pn = FakeProNet(log)
    sync = FakeSync(log, hot) if with_sync else None
    for k in range(steps):
        bench.run_step(pn, sync, k, world, rank, S, n_launch, n_ex, steps * S * world, 5, 1, "hybrid",
                       sync_every)
    return log


def test_one_gpu_one_launch_per_step_no_exchange():
    S = 1 << 27
    log = _run(1, 0, 3, S, 1, 1, with_sync=False)
    assert log == [("train", k * S, S) for k in range(3)]


def test_two_exchanges_per_step_default_n_gt_1():
    S = 1 << 27
    log = _run(4, 2, 2, S, 2, 2)
    expect = []
    for k in range(2):
        b = (k * 4 + 2) * S
        expect += [("train", b, S // 2), ("begin",), ("train", b + S // 2, S // 2), ("begin",)]
    assert log == expect


def test_sum_rule_hub_rows_after_every_launch():
    S = 1 << 20
    log = _run(2, 1, 1, S, 8, 1, hot=True)
    trains = [e for e in log if e[0] == "train"]
    assert [e[0] for e in log] == ["train", "hot"] * 8 + ["begin"]
    assert sum(e[2] for e in trains) == S and trains[0][1] == S


def test_sync_every_two_steps_and_uneven_split():
    S = 1000
    log = _run(2, 0, 4, S, 3, 1, sync_every=2)
    trains = [e for e in log if e[0] == "train"]
    assert [e[2] for e in trains[:3]] == [333, 333, 334]
    # one exchange at the end of steps 1 and 3 only
    begins = [i for i, e in enumerate(log) if e[0] == "begin"]
    assert len(begins) == 2 and begins[0] == 6 and begins[1] == 13


def test_ranks_and_steps_tile_the_global_sample_range():
    S, world, steps = 4096, 3, 3
    ranges = []
    for r in range(world):
        ranges += [(b, b + n) for _, b, n in (e for e in _run(world, r, steps, S, 2, 2) if e[0] == "train")]
    ranges.sort()
    assert ranges[0][0] == 0 and ranges[-1][1] == world * steps * S
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
