"""Incremental divide (sph_divide.hip, k_inc_classify / k_inc_boxes / k_inc_push).

Every divide after the first merges the previous stable order with the particles whose
box changed instead of re-sorting all keys.  The reference defines the order as the
stable sort by box key (JCellDivCpuSingle.cpp:203-234, the CPU counting sort); the radix
path (SPH_DIVIDE=full) is pinned to the oracle's order bit for bit
(test_gpu_parity.py::test_initial_divide_order_is_the_oracles, and through every
reference-PART test).  Here the incremental path must give the radix path's state BIT
FOR BIT after every step — particle order, positions, velocities, densities, counts and
the dt trace — on cases that move particles across cells in every direction, exclude
particles (far movers to the out boxes), move bodies, and on 2-D (one y row), half
cells and the NN solver.
"""
import copy

import numpy as np
import pytest

from dualsphysics_multilayer_amd.case import DamBreak2DCase, DamBreakCase, WaveFlumeCase, WetDambreakNNCase

pytestmark = pytest.mark.gpu


def _solver(case, mode, monkeypatch, dbg=0):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    if mode == "full":
        monkeypatch.setenv("SPH_DIVIDE", "full")
    else:
        monkeypatch.delenv("SPH_DIVIDE", raising=False)
    if dbg:
        monkeypatch.setenv("SPH_INC_DBG", str(dbg))
    s = SphGpuSingle(case, device=0)
    monkeypatch.delenv("SPH_DIVIDE", raising=False)
    monkeypatch.delenv("SPH_INC_DBG", raising=False)
    return s


def _same(case, nsteps, chunk, monkeypatch, dbg=0):
    a = _solver(case, "inc", monkeypatch, dbg)
    b = _solver(case, "full", monkeypatch)
    done = 0
    while done < nsteps:
        a.run(chunk)
        b.run(chunk)
        done += chunk
        sa, sb = a.stats(), b.stats()
        for k in ("np", "npb", "npbok", "nout", "nstep", "error_flags"):
            assert sa[k] == sb[k], (done, k, sa[k], sb[k])
        pa, pb = a.particles(), b.particles()
        for k in ("idp", "pos", "vel", "rhop"):  # device order: the divide's order itself
            assert np.array_equal(pa[k], pb[k]), (done, k)
    assert np.array_equal(a.dt_trace(), b.dt_trace())
    return a.stats()


def _stirred(case, frac, speed, seed=3):
    """Fluid particles given random velocities so that many cross cell faces in every
    direction (x, y, z and diagonals) within a few steps."""
    c = copy.copy(case)
    c.vel = case.vel.copy()
    rng = np.random.default_rng(seed)
    fl = np.arange(case.npb, case.np)
    pick = rng.choice(fl, int(frac * len(fl)), replace=False)
    c.vel[pick] = rng.uniform(-speed, speed, size=(len(pick), 3))
    return c


@pytest.mark.parametrize("dbg", [0, 48, 64, 112])
def test_inc_divide_verlet_stirred(monkeypatch, dbg):
    case = _stirred(DamBreakCase(0.02, celldomfixed=True), 0.5, 3.0)
    _same(case, 60, 5, monkeypatch, dbg)


def test_inc_divide_symplectic_ddt1(monkeypatch):
    case = _stirred(DamBreakCase(0.025, step_algorithm=2, tdensity=1, celldomfixed=True), 0.3, 2.0)
    _same(case, 40, 4, monkeypatch)


@pytest.mark.parametrize("nfast,dbg", [(40, 0), (40, 48), (40, 64), (900, 0)])
def test_inc_divide_exclusions(monkeypatch, nfast, dbg):
    """Far movers: OUTMOVE / OUTPOS / OUTRHOP exclusions go to the out boxes (and leave np).
    900 at once exceed the far arrivals a block keeps in LDS (IB_FCAP); dbg 48 forces the
    global-memory paths of the tile prefixes and far arrivals, 64 the chunked ranking pass."""
    case = DamBreakCase(0.03, celldomfixed=True, rhopoutmax=1010.0)
    rng = np.random.default_rng(7)
    pick = rng.choice(np.arange(case.npb, case.np), nfast, replace=False)
    q = nfast // 4
    case.vel[pick[:q]] = [0, 0, 400.0]
    case.vel[pick[q:2 * q]] = [0, 0, -30.0]
    case.vel[pick[2 * q:3 * q]] = [-120.0, 0, 0]
    case.vel[pick[3 * q:]] = [0, 25.0, 0]
    st = _same(case, 30, 1, monkeypatch, dbg)
    assert st["nout"] >= q


def test_inc_divide_first_particle_excluded(monkeypatch):
    """No boundary particles (npb = 0) and np not a multiple of the 1024-particle tile: the
    particle that sorts first is a far mover to the out boxes.  The push kernel's tail lanes
    (index >= np) read particle 0's slot; they must not take its far-mover word."""
    case = copy.copy(DamBreakCase(0.03, celldomfixed=True))
    fl = slice(case.npb, case.np)
    case.pos = case.pos[fl].copy()
    case.vel = case.vel[fl].copy()
    case.rhop = case.rhop[fl].copy()
    case.np -= case.npb
    case.npb = 0
    case.idp = np.arange(case.np, dtype=np.uint32)
    assert case.np % 1024 != 0
    first = np.lexsort((case.pos[:, 0], case.pos[:, 1], case.pos[:, 2]))[0]
    case.vel[first] = [0.0, 0.0, -400.0]
    st = _same(case, 6, 1, monkeypatch)
    assert st["nout"] >= 1 and st["npb"] == 0


def test_inc_divide_half_cells(monkeypatch):
    case = _stirred(DamBreakCase(0.025, cellmode=2, celldomfixed=True), 0.3, 2.0)
    _same(case, 30, 5, monkeypatch)


def test_inc_divide_2d(monkeypatch):
    case = _stirred(DamBreak2DCase(0.01), 0.3, 2.0)
    _same(case, 60, 10, monkeypatch)


def test_inc_divide_bodies(monkeypatch):
    """Piston, flap (moving boundaries) and a floating box (particles moved by the body)."""
    _same(WaveFlumeCase(0.025), 40, 8, monkeypatch)


def test_inc_divide_nn(monkeypatch):
    _same(WetDambreakNNCase(0.025, width=0.2, scale=0.5), 20, 5, monkeypatch)


def test_inc_divide_1m(monkeypatch):
    """BASELINE cfg2 size: 1,025,964 particles, 20 steps (one Euler step at 40 is not
    reached; the Verlet steps carry VelrhopM1 through the push)."""
    case = DamBreakCase(0.0045)
    assert case.np == 1025964
    _same(case, 20, 10, monkeypatch)


# ---- slabs: the exchange appends migrants + ghosts after the previous order; stale ghosts
# leave through the discard box (k_inc_classify DROP / APP classes) ------------------------
def _group(case, nslabs, mode, monkeypatch, repart=0):
    from dualsphysics_multilayer_amd.core import SphSlabGroup, case_derive, slab_partition

    if mode == "full":
        monkeypatch.setenv("SPH_DIVIDE", "full")
    else:
        monkeypatch.delenv("SPH_DIVIDE", raising=False)
    if repart:  # an uneven start, so that the first re-partition moves the bounds
        ncx = case_derive(case.case_def())["dom_cells"][0]
        bounds = np.array([0] + [ncx - 2 * (nslabs - r) for r in range(1, nslabs)] + [ncx], np.int32)
    else:
        bounds = slab_partition(case, nslabs)
    g = SphSlabGroup(case, bounds)
    monkeypatch.delenv("SPH_DIVIDE", raising=False)
    if repart:
        g.set_repartition(repart, 0.3, 0.0)
    return g


def _same_slabs(case, nslabs, nsteps, chunk, monkeypatch, repart=0):
    a = _group(case, nslabs, "inc", monkeypatch, repart)
    b = _group(case, nslabs, "full", monkeypatch, repart)
    done = 0
    while done < nsteps:
        a.run(chunk)
        b.run(chunk)
        done += chunk
        for r, (ma, mb) in enumerate(zip(a.members, b.members)):
            sa, sb = ma.stats(), mb.stats()
            for k in ("np", "npb", "npbok", "nout", "nstep", "error_flags"):
                assert sa[k] == sb[k], (done, r, k, sa[k], sb[k])
            pa, pb = ma.particles(), mb.particles()
            for k in ("idp", "pos", "vel", "rhop"):  # each slab's device order
                assert np.array_equal(pa[k], pb[k]), (done, r, k)
    if repart:
        assert [m["repartitions"] for m in a.slab_info()] == [m["repartitions"] for m in b.slab_info()]
    return a


@pytest.mark.parametrize("nslabs", [2, 3])
def test_inc_divide_slabs_verlet_stirred(monkeypatch, nslabs):
    case = _stirred(DamBreakCase(0.025, celldomfixed=True), 0.5, 3.0)
    _same_slabs(case, nslabs, 40, 5, monkeypatch)


def test_inc_divide_slabs_symplectic_exclusions(monkeypatch):
    case = _stirred(DamBreakCase(0.03, step_algorithm=2, tdensity=1, celldomfixed=True, rhopoutmax=1010.0), 0.3, 2.0)
    rng = np.random.default_rng(5)
    pick = rng.choice(np.arange(case.npb, case.np), 40, replace=False)
    case.vel[pick[:20]] = [0, 0, 400.0]
    case.vel[pick[20:]] = [-120.0, 0, 0]
    _same_slabs(case, 3, 30, 3, monkeypatch)


def test_inc_divide_slabs_bodies_and_nn(monkeypatch):
    _same_slabs(WaveFlumeCase(0.025), 3, 24, 8, monkeypatch)
    _same_slabs(WetDambreakNNCase(0.025, width=0.2, scale=0.5), 2, 12, 4, monkeypatch)


def test_inc_divide_slabs_repartition(monkeypatch):
    """A re-partition changes the slab grids: that divide sorts from scratch, later ones merge."""
    case = _stirred(DamBreakCase(0.025, celldomfixed=True), 0.5, 3.0)
    g = _same_slabs(case, 3, 30, 5, monkeypatch, repart=5)
    assert max(m["repartitions"] for m in g.slab_info()) >= 1
