"""GPU parity of the slab decomposition.

The decomposed run (x-slabs, ghost columns, migration, max-allreduced dt) must give
the single-domain answer: the merged owned particles are held to the same
tolerances as the single-GPU path against the reference's PART fixtures and the
oracle, the excluded set and the particle count are exact, and the run is
bitwise deterministic.  Slabs run as an in-process group on one GPU
(SphSlabGroup: the same pack/exchange/divide/reduce code as the RCCL path, with
device-to-device copies as the transport — RCCL refuses two ranks on one device).
"""
import numpy as np
import pytest

from golden_io import cellmode, tol, by_idp, load, maxdiff, meta, snapshot, steps

from dualsphysics_multilayer_amd.case import DamBreakCase

pytestmark = pytest.mark.gpu

oracle = pytest.importorskip("oracle.pyoracle")


def group(case, nslabs, bounds=None):
    from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition

    if bounds is None:
        bounds = slab_partition(case, nslabs)
    return SphSlabGroup(case, bounds)


def single(case):
    from dualsphysics_multilayer_amd.core import SphGpuSingle

    return SphGpuSingle(case, device=0)


def check_close(got, ref, step):
    assert np.array_equal(got["idp"], ref["idp"]), "excluded-particle set differs"
    tp, tv, tr = tol(step)
    assert maxdiff(got, ref, "pos") <= tp, (step, maxdiff(got, ref, "pos"))
    assert maxdiff(got, ref, "vel") <= tv, (step, maxdiff(got, ref, "vel"))
    assert maxdiff(got, ref, "rhop") <= tr, (step, maxdiff(got, ref, "rhop"))


@pytest.mark.parametrize("name,nslabs", [("verlet_ddt2_dp0.02", 2), ("verlet_ddt2_dp0.02", 3),
                                         ("symplectic_ddt1_dp0.025", 3)])
def test_slabs_match_reference_parts(name, nslabs):
    g_ = load(name)
    dp, step_alg, ddt, _ = meta(g_)
    grp = group(DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt), nslabs)
    done = 0
    for k in steps(g_):
        grp.run(k - done)
        done = k
        ref = snapshot(g_, k)
        check_close(grp.particles(), ref, k)
        times = [s["time"] for s in grp.stats()]
        assert max(times) == min(times), "slabs disagree on dt"
        assert abs(times[0] - float(ref["time"])) <= 1e-8 * max(1.0, k)


def test_slabs_match_single_gpu_and_conserve_count():
    case = DamBreakCase(0.025)
    grp, one = group(case, 4), single(case)
    grp.run(30)
    one.run(30)
    pg, p1 = grp.particles(), by_idp(one.particles())
    st = grp.stats()
    assert sum(s["np"] for s in st) == one.stats()["np"] == case.np
    check_close(pg, p1, 30)
    assert np.array_equal(np.array([s["nstep"] for s in st]), np.full(4, 30))


def test_heavy_migration_matches_oracle():
    """Every fluid particle pushed along +x at 3 m/s: many cross slab faces every few
    steps (migration + ghost refresh on both faces); result vs the single-domain oracle."""
    case = DamBreakCase(0.03, celldomfixed=True)
    case.vel[case.npb:, 0] = 3.0
    grp = group(case, 3)
    o = oracle.OracleSolver(case, nthreads=4)
    b0 = [s["np"] for s in grp.stats()]
    done = 0
    for k in (10, 40):
        grp.run(k - done)
        o.run(k - done)
        done = k
        check_close(grp.particles(), by_idp(o.particles()), k)
    b1 = [s["np"] for s in grp.stats()]
    assert b0 != b1, "no particle changed slab"


def test_narrowest_slabs_and_exclusion():
    """The narrowest slabs (two columns between two neighbours: every owned column is a
    face column) and excluded particles (OUTPOS through x < MapRealPosMin, OUTRHOP) in a
    slab run."""
    case = DamBreakCase(0.03, celldomfixed=True, rhopoutmax=1010.0)
    rng = np.random.default_rng(7)
    pick = rng.choice(np.arange(case.npb, case.np), 12, replace=False)
    case.vel[pick[:4]] = [0, 0, 400.0]
    case.vel[pick[4:8]] = [0, 0, -30.0]
    case.vel[pick[8:]] = [-120.0, 0, 0]
    from dualsphysics_multilayer_amd.core import case_derive

    ncx = case_derive(case.case_def())["dom_cells"][0]
    bounds = np.array([0, 2, 4, 6, 8, ncx], np.int32)
    grp = group(case, 5, bounds)
    o = oracle.OracleSolver(case, nthreads=4)
    for k in range(1, 7):
        grp.run(1)
        o.run(1)
        st, so = grp.stats(), o.stats()
        assert sum(s["np"] for s in st) == so["np"]
        assert sum(s["nout"] for s in st) == so["nout"]
        assert np.array_equal(grp.particles()["idp"], np.sort(o.particles()["idp"]))
    check_close(grp.particles(), by_idp(o.particles()), 6)


def test_slabs_deterministic_bitwise():
    case = DamBreakCase(0.025)
    case.vel[case.npb:, 0] = 2.0
    a, b = group(case, 3), group(case, 3)
    a.run(25)
    b.run(25)
    pa, pb = a.particles(), b.particles()
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(pa[k], pb[k]), k


def test_large_case_slabs_properties():
    """1M particles (cfg2 size) in 4 slabs against one domain: count conserved, same
    simulated time, fields within the rounding noise after 10 steps."""
    case = DamBreakCase(0.0045)
    grp, one = group(case, 4), single(case)
    grp.run(10)
    one.run(10)
    st = grp.stats()
    assert sum(s["np"] for s in st) == case.np
    assert abs(st[0]["time"] - one.stats()["time"]) <= 1e-9
    pg, p1 = grp.particles(), by_idp(one.particles())
    assert np.array_equal(pg["idp"], p1["idp"])
    assert maxdiff(pg, p1, "pos") <= 1e-7 and maxdiff(pg, p1, "vel") <= 5e-5


def test_rccl_transport_single_rank():
    """The RCCL transport end to end on one GPU: a 1-rank slab (ncclCommInitRank; with no
    neighbour it exchanges nothing and its own dt maxima are the domain's) must step like
    the single-domain solver."""
    from dualsphysics_multilayer_amd.core import SphGpuSlab, case_derive, comm_unique_id

    case = DamBreakCase(0.025)
    ncx = case_derive(case.case_def())["dom_cells"][0]
    s = SphGpuSlab(case, 0, 1, [0, ncx], comm_unique_id(), device=0)
    one = single(case)
    s.run(20)
    one.run(20)
    assert s.stats()["np"] == one.stats()["np"]
    assert s.stats()["time"] == pytest.approx(one.stats()["time"], rel=1e-9)
    check_close(by_idp(s.particles()), by_idp(one.particles()), 20)
    s.close()


def test_cfg3_10m_slabs_match_single_domain():
    """BASELINE cfg3 at its full size (9,969,118 particles, Symplectic + DDT Molteni): four
    in-process slabs against one domain over 5 steps — particle count conserved, the same
    excluded set and simulated time, fields within the 5-step noise tolerance."""
    case = DamBreakCase(0.00205, step_algorithm=2, tdensity=1)
    assert case.np == 9969118
    one = single(case)
    one.run(5)
    s1 = one.stats()
    p1 = by_idp(one.particles())
    one.close()
    del one
    grp = group(case, 4)
    grp.run(5)
    st = grp.stats()
    assert sum(s["np"] for s in st) == s1["np"] == case.np
    assert sum(s["nout"] for s in st) == s1["nout"] == 0
    assert abs(st[0]["time"] - s1["time"]) <= 1e-9
    pg = grp.particles()
    assert np.array_equal(pg["idp"], p1["idp"])
    check_close(pg, p1, 5)


def test_cfg3_10m_eight_slabs_with_repartition_match_single_domain():
    """BASELINE cfg3's own split: the 10M case in 8 slabs (6 interior slabs with both faces,
    the ghost exchange beside the interior items' interaction), re-partitioned every 2 steps
    from step 4 on, against one domain after 8 steps: the same particles and simulated time,
    fields within the 8-step noise tolerance."""
    case = DamBreakCase(0.00205, step_algorithm=2, tdensity=1)
    one = single(case)
    one.run(8)
    s1 = one.stats()
    p1 = by_idp(one.particles())
    one.close()
    del one
    grp = group(case, 8)
    grp.run(4)
    grp.set_repartition(2, 0.3, 0.0)
    grp.run(4)
    st = grp.stats()
    assert sum(s["np"] for s in st) == s1["np"] == case.np
    assert len({s["time"] for s in st}) == 1 and abs(st[0]["time"] - s1["time"]) <= 1e-9
    assert all(s["error_flags"] == 0 for s in st)
    assert max(i["repartitions"] for i in grp.slab_info()) >= 1
    pg = grp.particles()
    assert np.array_equal(pg["idp"], p1["idp"])
    check_close(pg, p1, 8)


@pytest.mark.parametrize("cfg", ["verlet_full", "symplectic_half", "verlet_repartition", "flume_bodies"])
def test_ghost_overlap_is_bitwise_the_in_place_exchange(cfg, monkeypatch):
    """The ghost records of a divide sent beside the interaction of the items that reach no
    ghost column, or put in place before the interaction with the same (cut) items
    (SPH_SLAB_CUT=1): bitwise the same run."""
    from dualsphysics_multilayer_amd.case import WaveFlumeCase
    from dualsphysics_multilayer_amd.core import case_derive

    rep = None
    if cfg == "verlet_full":
        case = DamBreakCase(0.025)
        case.vel[case.npb:, 0] = 2.0
        nslabs, bounds = 4, None
    elif cfg == "symplectic_half":
        case = DamBreakCase(0.03, step_algorithm=2, tdensity=1, cellmode=2, celldomfixed=True)
        case.vel[case.npb:, 0] = -2.0
        ncx = case_derive(case.case_def())["dom_cells"][0]
        nslabs, bounds = 4, np.array([0, 4, 8, 12, ncx], np.int32)
    elif cfg == "verlet_repartition":
        case = DamBreakCase(0.025)
        case.vel[case.npb:, 0] = 1.5
        nslabs, bounds, rep = 3, None, (3, 0.3, 0.0)
    else:  # moving boundaries + a floating body: ghosts in place before the interaction
        case = WaveFlumeCase(0.03)
        nslabs, bounds = 3, None
    res = []
    monkeypatch.setenv("SPH_SLAB_CUT", "1")
    for ov in (True, False):
        grp = group(case, nslabs, bounds)
        grp.set_overlap(ov)
        if rep:
            grp.set_repartition(*rep)
        grp.run(12)
        res.append(grp.particles())
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(res[0][k], res[1][k]), k


@pytest.mark.parametrize("name", ["verlet_ddt2_dp0.02", "symplectic_ddt1_dp0.025"])
def test_repartition_matches_reference_parts(name):
    """Periodic re-balancing: three slabs started far from balance (slab 0
    holds all but the last four columns), re-partitioned every 3 steps with no tolerance,
    so whole columns are handed over while the fluid moves; the merged state stays on the
    reference PARTs and the loads end near balance."""
    g_ = load(name)
    dp, step_alg, ddt, _ = meta(g_)
    case = DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt)
    from dualsphysics_multilayer_amd.core import case_derive

    ncx = case_derive(case.case_def())["dom_cells"][0]
    start = np.array([0, ncx - 4, ncx - 2, ncx], np.int32)
    grp = group(case, 3, start)
    loads0 = [s["np"] for s in grp.stats()]
    grp.set_repartition(3, 0.3, 0.0)
    done = 0
    for k in steps(g_):
        grp.run(k - done)
        done = k
        check_close(grp.particles(), snapshot(g_, k), k)
    info = grp.slab_info()
    assert all(i["repartitions"] >= 1 for i in info)
    assert [i["cx_begin"] for i in info] != list(start[:3])
    loads = [s["np"] for s in grp.stats()]
    assert max(loads) / max(min(loads), 1) < max(loads0) / max(min(loads0), 1)
    assert max(loads) < 3.0 * min(loads), loads


def test_repartition_deterministic_and_matches_single():
    case = DamBreakCase(0.025)
    case.vel[case.npb:, 0] = 1.5
    a, b, one = group(case, 4), group(case, 4), single(case)
    for gr in (a, b):
        gr.set_repartition(5, 0.3, 0.02)
    a.run(30)
    b.run(30)
    one.run(30)
    pa, pb = a.particles(), b.particles()
    for k in ("idp", "pos", "vel", "rhop"):
        assert np.array_equal(pa[k], pb[k]), k
    check_close(pa, by_idp(one.particles()), 30)
    assert [i["cx_begin"] for i in a.slab_info()] == [i["cx_begin"] for i in b.slab_info()]


# ---- CellMode=half: cells of h, two ghost columns per face (the support 2h) -----------------
@pytest.mark.parametrize("nslabs", [2, 3])
def test_half_cell_slabs_match_reference_parts(nslabs):
    g_ = load("verlet_ddt2_half_dp0.025")
    dp, step_alg, ddt, _ = meta(g_)
    assert cellmode(g_) == 2
    grp = group(DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt, cellmode=2), nslabs)
    info = grp.slab_info()
    assert min(i["cx_end"] - i["cx_begin"] for i in info) >= 2
    done = 0
    for k in steps(g_):
        grp.run(k - done)
        done = k
        check_close(grp.particles(), snapshot(g_, k), k)
        times = [s["time"] for s in grp.stats()]
        assert max(times) == min(times)


def test_half_cell_narrowest_slabs_migration_and_repartition():
    """Slabs of exactly four half-cell columns (two face columns towards each neighbour),
    fluid pushed along +x so particles migrate every few steps, then re-balancing every 4
    steps: against the single-domain oracle."""
    from dualsphysics_multilayer_amd.core import case_derive

    case = DamBreakCase(0.03, cellmode=2, celldomfixed=True)
    case.vel[case.npb:, 0] = 2.0
    ncx = case_derive(case.case_def())["dom_cells"][0]
    grp = group(case, 4, np.array([0, 4, 8, 12, ncx], np.int32))
    o = oracle.OracleSolver(case, nthreads=4)
    done = 0
    for k in (4, 12):
        grp.run(k - done)
        o.run(k - done)
        done = k
        check_close(grp.particles(), by_idp(o.particles()), k)
    grp.set_repartition(4, 0.3, 0.0)
    grp.run(12)
    o.run(12)
    check_close(grp.particles(), by_idp(o.particles()), 24)
    info = grp.slab_info()
    assert all(i["cx_end"] - i["cx_begin"] >= 4 for i in info)
    assert max(i["repartitions"] for i in info) >= 1


def test_half_cell_partition_keeps_disjoint_faces():
    """slab_partition with CellMode=half gives every slab at least 2W = 4 columns (two
    disjoint sets of two face columns); narrower slabs are refused: below W = 2 at a map
    end, below 4 between two neighbours."""
    from dualsphysics_multilayer_amd.core import SphSlabGroup, case_derive, slab_partition

    case = DamBreakCase(0.03, cellmode=2)
    ncx = case_derive(case.case_def())["dom_cells"][0]
    b = slab_partition(case, ncx // 4)
    assert (np.diff(b) >= 4).all() and b[-1] == ncx
    with pytest.raises(Exception):
        SphSlabGroup(case, np.array([0, 1, ncx], np.int32))
    with pytest.raises(Exception):
        SphSlabGroup(case, np.array([0, 4, 7, ncx], np.int32))


def test_half_cell_one_slab_matches_single_domain():
    """One slab holding every column with CellMode=half: its grid is the domain plus
    W = 2 ghost columns per face, the widest a slab grid gets, so the grid-sized buffers
    (begincell, items, the incremental divide's box table) must hold it; the run must
    equal the single domain within the 20-step noise tolerance."""
    case = DamBreakCase(0.025, cellmode=2)
    from dualsphysics_multilayer_amd.core import case_derive

    ncx = case_derive(case.case_def())["dom_cells"][0]
    grp, one = group(case, 1, np.array([0, ncx], np.int32)), single(case)
    grp.run(20)
    one.run(20)
    assert grp.stats()[0]["np"] == one.stats()["np"] == case.np
    check_close(grp.particles(), by_idp(one.particles()), 20)


def test_fatal_error_halts_every_slab_at_the_same_step():
    """ERR_BOUNDOUT raised by ONE slab's divide (the piston of the wave flume driven out of
    the map through x < MapRealPosMin: AbortBoundOut) travels with the dt maxima's
    all-reduce, so every slab stops at the same step and the group run raises, as the one
    reference domain stops the whole run."""
    from dualsphysics_multilayer_amd.case import WaveFlumeCase
    from dualsphysics_multilayer_amd.core import SphError

    case = WaveFlumeCase(0.03)
    pist = dict(case.motion["movs"][0])
    pist["vec"], pist["vec2"] = (5.0, 0.0, 0.0), (-0.5, 0.0, 0.0)  # 5 Hz, 0.5 m towards -x
    case.motion = dict(case.motion, movs=[pist] + list(case.motion["movs"][1:]))
    grp = group(case, 3)
    with pytest.raises(SphError, match="boundary particles were excluded"):
        grp.run(80)
    st = grp.stats()
    assert len({s["nstep"] for s in st}) == 1 and 0 < st[0]["nstep"] < 80, [s["nstep"] for s in st]
    assert len({s["time"] for s in st}) == 1
    assert all(s["error_flags"] & 2 for s in st), [s["error_flags"] for s in st]


@pytest.mark.parametrize("turns,overlap", [("1", True), ("2", False), ("2", True)])
def test_turns_measurement_modes_are_bitwise_the_normal_run(turns, overlap, monkeypatch):
    """The turns measurement modes (SPH_SLAB_TURNS=1: interactions and divides one slab at a
    time; 2: updates and the exchange's pack too) only order the slabs' kernels on the GPU:
    the run is bitwise the normal one, Verlet and Symplectic, ghosts in place or beside the
    interaction."""
    res = []
    for step_alg, ddt, dp in ((1, 2, 0.025), (2, 1, 0.03)):
        case = DamBreakCase(dp, step_algorithm=step_alg, tdensity=ddt)
        case.vel[case.npb:, 0] = 1.5  # migration across the faces
        out = []
        for env in (None, turns):
            if env is None:
                monkeypatch.delenv("SPH_SLAB_TURNS", raising=False)
            else:
                monkeypatch.setenv("SPH_SLAB_TURNS", env)
            grp = group(case, 3)
            grp.set_overlap(overlap)
            grp.run(10)
            out.append(grp.particles())
            grp.close()
        res.append(out)
    for a, b in res:
        for k in ("idp", "pos", "vel", "rhop"):
            assert np.array_equal(a[k], b[k]), k
