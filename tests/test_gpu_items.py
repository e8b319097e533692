"""The per-divide item list of the tiled interactions (csrc/sph_items.hpp): the count pass
stages each row's items in a slot of `ricap` items, the place pass copies them, and a row
whose items overflow its slot is walked again.  With tiny slots (SPH_ITEMS_RICAP, a test
hook read at solver creation) nearly every row takes the second walk: the list, and so the
run, must be bitwise the same — single domain (full and half cells) and two item lists
(slab ghost overlap)."""
import os

import numpy as np
import pytest

from dualsphysics_multilayer_amd.case import DamBreakCase


def _run(make, ricap):
    old = os.environ.pop("SPH_ITEMS_RICAP", None)
    try:
        if ricap is not None:
            os.environ["SPH_ITEMS_RICAP"] = str(ricap)
        return make()
    finally:
        os.environ.pop("SPH_ITEMS_RICAP", None)
        if old is not None:
            os.environ["SPH_ITEMS_RICAP"] = old


@pytest.mark.gpu
@pytest.mark.parametrize("cellmode", [1, 2])
def test_item_slots_overflow_is_bitwise(cellmode):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    case = DamBreakCase(0.02, step_algorithm=2, tdensity=2, cellmode=cellmode)

    def make():
        s = SphGpuSingle(case, device=0)
        s.run(15)
        return s.particles()

    ref = _run(make, None)
    for ricap in (1, 3):
        got = _run(make, ricap)
        for k in ("idp", "pos", "vel", "rhop"):
            assert np.array_equal(got[k], ref[k]), (ricap, k)


@pytest.mark.gpu
def test_item_slots_overflow_two_lists_is_bitwise():
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    case = DamBreakCase(0.025)
    case.vel[case.npb:, 0] = 2.0

    def make():
        grp = SphSlabGroup(case, slab_partition(case, 3))
        grp.set_overlap(True)  # interior + face item lists
        grp.run(10)
        return grp.particles()

    ref = _run(make, None)
    got = _run(make, 2)
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(got[k], ref[k]), k
