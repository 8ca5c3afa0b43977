"""The bounding-box pass's work queue (k_mbr.hip k_mbr_order): y tiles above the average cost
are split into up to kMbrSplitMax items.  The item count must fit the queue the host sizes
(sky_internal.h mbr_items_max = ytiles + max(ytiles, 4096)) for ANY cost distribution: the
per-item cost c0 is total / max(ytiles, 4096) rounded UP (rounded down, c0 = 1 split every tile
into c_t items and overflowed the queue: an illegal address on the GPU in round 4).  This is
the rule restated in Python over adversarial cost vectors."""
import random


def _items(costs, split_max=64):
    nyt = len(costs)
    total = sum(costs)
    m = max(nyt, 4096)
    c0 = max(1, (total + m - 1) // m)
    return sum(min(c, split_max, (c + c0 - 1) // c0) for c in costs if c), nyt + max(nyt, 4096)


def test_split_items_fit_the_queue():
    rng = random.Random(4)
    for _ in range(300):
        nyt = rng.choice([1, 3, 100, 800, 4095, 4096, 4097, 31000, 160000])
        kind = rng.randrange(5)
        if kind == 0:
            costs = [rng.randrange(0, 20) for _ in range(nyt)]
        elif kind == 1:
            costs = [rng.randrange(0, 100000) for _ in range(nyt)]
        elif kind == 2:
            costs = [0] * (nyt - 1) + [10 ** 7]
        elif kind == 3:
            costs = [int(rng.paretovariate(1.1)) for _ in range(nyt)]
        else:
            costs = [5000] * nyt
        n, cap = _items(costs)
        assert n <= cap, (n, cap, nyt, kind)
