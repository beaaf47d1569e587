"""The incremental region update of the W = 1 rule audit (RegionSet1, sparc_rules.hpp; the
k_rollout1r INC shapes) restated on the CPU (tools/inc_regions_sim.py) equals the full flood of
every region after every step of random walks with pops, resets and gaps, and exercises every
case (rebuild, simple remove, split, add)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_incremental_regions_equal_full_flood():
    import inc_regions_sim
    rebuilds, simple, splits, adds = inc_regions_sim.main(200)
    assert min(rebuilds, simple, splits, adds) > 100


def test_ring_simple_table():
    import inc_regions_sim
    lut = inc_regions_sim.LUT
    assert len(lut) == 512
    assert lut[0] == 1                      # nothing allowed around: no split
    assert lut[0b111101111] == 1            # the whole ring allowed
    # (0, -1) and (0, 1) allowed, the sides blocked: two runs, each with a 4-neighbour
    assert lut[(1 << 3) | (1 << 5)] == 0
    # only diagonals allowed: no 4-neighbour, no split
    assert lut[(1 << 0) | (1 << 2) | (1 << 6) | (1 << 8)] == 1
