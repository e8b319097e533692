"""The N>1 (slab-decomposed) path on CPU: world_size-2 torch.distributed/gloo runs.

1. Halo sufficiency (no GPU): each rank keeps its owned columns of the partition
   (sph_slab_partition, the C++ host function the GPU path uses), receives its
   neighbours' border columns over gloo as ghosts — the exchange rule of
   sph_slab.hip — and runs the CPU oracle's Interaction_Forces on owned + ghosts.
   Every owned particle must get exactly (bit for bit) the single-domain oracle's
   ar/ace, and the max-allreduced AceMax must equal the single-domain one: this is
   the property the slab decomposition rests on (one column = 2h = the support).
2. Exchange protocol under motion (no GPU): a numpy model of the pack rules of
   sph_slab.hip (pack_class: stale ghosts dropped, migrants handed over and kept as
   ghosts, border columns copied) driven over gloo through random moves of up to
   0.9 cell per step (MovLimit); after every exchange each particle is owned by
   exactly one rank and every rank's ghost set is exactly its neighbours' particles
   in its ghost columns.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _sendrecv_arrays(arrays, peer_send, peer_recv, dtypes):
    """Send a list of numpy arrays to peer_send and receive the same layout from
    peer_recv (either may be None).  Counts first, then one tensor per field."""
    reqs = []
    if peer_send is not None:
        n = torch.tensor([len(arrays[0])], dtype=torch.int64)
        dist.send(n, peer_send)
        for a in arrays:
            if len(a):
                dist.send(torch.from_numpy(np.ascontiguousarray(a)), peer_send)
    out = None
    if peer_recv is not None:
        n = torch.zeros(1, dtype=torch.int64)
        dist.recv(n, peer_recv)
        out = []
        for dt, a in zip(dtypes, arrays):
            shape = (int(n.item()),) + a.shape[1:]
            t = torch.from_numpy(np.zeros(shape, dt))
            if shape[0]:
                dist.recv(t, peer_recv)
            out.append(t.numpy())
    del reqs
    return out


class _SubCase:
    """A rank's particle subset with the full case's constants and map limits."""

    def __init__(self, case, idx):
        self._cdef = dict(case.case_def())
        self.idp = case.idp[idx]
        self.pos = case.pos[idx]
        self.vel = case.vel[idx]
        self.rhop = case.rhop[idx]
        self.npb = int((idx < case.npb).sum())
        self.np = len(idx)
        self._cdef.update(npb=self.npb, np=self.np)

    def case_def(self):
        return self._cdef


def _columns(case, k, axis=0):
    # JSph::LoadDcellParticles: unsigned(dx / double(float scell)) with the map minimum
    dx = case.pos[:, axis] - k["dom_posmin"][axis]
    return np.floor(dx / np.float64(np.float32(k["scell"]))).astype(np.int64)


def _halo_worker(rank, world, port, axis=0):
    _init(rank, world, port)
    from dualsphysics_multilayer_amd.case import DamBreakCase
    from dualsphysics_multilayer_amd.core import case_derive, slab_partition
    from oracle.pyoracle import OracleSolver

    case = DamBreakCase(0.03, celldomfixed=True)
    bounds = slab_partition(case, world, 0.3, axis)
    allb = [None] * world
    dist.all_gather_object(allb, bounds.tolist())
    assert all(b == allb[0] for b in allb), "ranks disagree on the partition"
    k = case_derive(case.case_def())
    cx = _columns(case, k, axis)  # cells along the slab axis (x columns or y rows)
    c0, c1 = int(bounds[rank]), int(bounds[rank + 1])
    own = np.nonzero((cx >= c0) & (cx < c1))[0]
    # ghost exchange: my first column to the left, my last column to the right
    ghosts = []
    for step in (0, 1):  # left-going then right-going, ordered to avoid deadlock
        send_to = rank - 1 if step == 0 else rank + 1
        recv_from = rank + 1 if step == 0 else rank - 1
        col = c0 if step == 0 else c1 - 1
        sel = own[cx[own] == col]
        got = _sendrecv_arrays([sel.astype(np.int64)], send_to if 0 <= send_to < world else None,
                               recv_from if 0 <= recv_from < world else None, [np.int64])
        if got is not None:
            ghosts.append(got[0])
    local = np.sort(np.concatenate([own] + ghosts))
    expect_ghost_cols = set()
    if rank > 0:
        expect_ghost_cols.add(c0 - 1)
    if rank + 1 < world:
        expect_ghost_cols.add(c1)
    assert set(np.unique(cx[np.setdiff1d(local, own)]).tolist()) <= expect_ghost_cols
    # interaction on owned + ghosts vs the single domain
    sub = OracleSolver(_SubCase(case, local), nthreads=1)
    isub, psub = sub.interaction(), sub.particles()
    full = OracleSolver(case, nthreads=1)
    ifull, pfull = full.interaction(), full.particles()
    pos_full = {int(i): j for j, i in enumerate(pfull["idp"])}
    owned_ids = set(case.idp[own].tolist())
    rows = [(j, pos_full[int(i)]) for j, i in enumerate(psub["idp"]) if int(i) in owned_ids]
    assert len(rows) == len(own)
    a, b = np.array([r[0] for r in rows]), np.array([r[1] for r in rows])
    assert np.array_equal(isub["ar"][a], ifull["ar"][b]), "owned ar differs from the single domain"
    assert np.array_equal(isub["ace"][a], ifull["ace"][b]), "owned ace differs from the single domain"
    # AceMax over owned fluid, max-reduced over ranks = single-domain AceMax
    fl = a[a >= sub.stats()["npb"]]
    ace2 = float((isub["ace"][fl].astype(np.float64) ** 2).sum(axis=1).max()) if len(fl) else 0.0
    t = torch.tensor([ace2], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert abs(np.sqrt(t.item()) - ifull["acemax"]) <= 1e-6 * ifull["acemax"]
    # every particle owned exactly once
    counts = torch.tensor([len(own)], dtype=torch.int64)
    dist.all_reduce(counts)
    assert int(counts.item()) == case.np
    dist.destroy_process_group()


def _pack_class_model(lcx, xown0, xown1, has_left, has_right):
    """numpy model of sph_slab.hip pack_class (live particles): bit0 record to the
    left, bit1 record to the right, bit2 stays owned."""
    c = np.zeros(len(lcx), np.int64)
    left, right = lcx < xown0, lcx >= xown1
    c[left] = 1 if has_left else 0
    c[right] = 2 if has_right else 0
    mid = ~left & ~right
    c[mid] = 4 + (((lcx[mid] == xown0) & has_left) * 1) + (((lcx[mid] == xown1 - 1) & has_right) * 2)
    return c


def _protocol_worker(rank, world, port):
    _init(rank, world, port)
    rng = np.random.default_rng(1234)  # same stream on every rank: global truth is shared
    ncx, n = 12, 600
    bounds = [0, 5, 12] if world == 2 else None
    c0, c1 = bounds[rank], bounds[rank + 1]
    xoff, xown0, xown1 = c0 - 1, 1, 1 + c1 - c0
    gx = rng.uniform(0.0, ncx, n)  # global x in cell units, all particles
    ids = np.arange(n)
    mine = (np.floor(gx) >= c0) & (np.floor(gx) < c1)
    ghost_cols = [c for c in (c0 - 1, c1) if 0 <= c < ncx and not (c == c0 - 1 and rank == 0)
                  and not (c == c1 and rank + 1 == world)]
    held_ids = ids[mine | np.isin(np.floor(gx), ghost_cols)]
    held_x = gx[held_ids]
    for step in range(25):
        # motion: every particle moves < 0.9 cell (MovLimit); owners move theirs, the
        # global truth moves all (same rng stream on both ranks)
        d = rng.uniform(-0.85, 0.85, n)
        gx = np.clip(gx + d, 0.0, ncx - 1e-9)
        lcx_before = np.floor(held_x).astype(np.int64) - xoff
        owned_now = (lcx_before >= xown0) & (lcx_before < xown1)
        held_x = np.where(owned_now, gx[held_ids], held_x)  # update kernels skip ghosts
        lcx = np.floor(held_x).astype(np.int64) - xoff
        alive = owned_now  # stale ghosts -> DCELL_DISCARD
        cls = np.zeros(len(held_ids), np.int64)
        cls[alive] = _pack_class_model(lcx[alive], xown0, xown1, rank > 0, rank + 1 < world)
        keep = alive & (((cls & 4) != 0) | (lcx == xown0 - 1) | (lcx == xown1))  # migrants stay as ghosts
        send_l = np.nonzero((cls & 1) != 0)[0]
        send_r = np.nonzero((cls & 2) != 0)[0]
        recv = []
        for s_idx, to, frm in ((send_l, rank - 1, rank + 1), (send_r, rank + 1, rank - 1)):
            got = _sendrecv_arrays([held_ids[s_idx].astype(np.int64), held_x[s_idx]],
                                   to if 0 <= to < world else None, frm if 0 <= frm < world else None,
                                   [np.int64, np.float64])
            if got is not None:
                recv.append(got)
        held_ids = np.concatenate([held_ids[keep]] + [r[0] for r in recv])
        held_x = np.concatenate([held_x[keep]] + [r[1] for r in recv])
        # invariants
        assert len(np.unique(held_ids)) == len(held_ids), "a particle is held twice"
        lcx = np.floor(held_x).astype(np.int64) - xoff
        owned = held_ids[(lcx >= xown0) & (lcx < xown1)]
        assert np.array_equal(np.sort(owned), ids[(np.floor(gx) >= c0) & (np.floor(gx) < c1)])
        assert np.allclose(held_x, gx[held_ids])
        ghosts = np.sort(held_ids[(lcx < xown0) | (lcx >= xown1)])
        truth = ids[np.isin(np.floor(gx), ghost_cols)]
        assert np.array_equal(ghosts, truth), "ghost layer incomplete or stale"
        allown = [None] * world
        dist.all_gather_object(allown, owned.tolist())
        assert sorted(sum(allown, [])) == list(range(n)), "ownership is not a partition"
    dist.destroy_process_group()


def _spawn(fn, *extra):
    mp.spawn(fn, args=(WORLD, _free_port()) + extra, nprocs=WORLD, join=True)


@pytest.mark.parametrize("axis", [0, 1], ids=["x_slabs", "y_slabs"])
def test_halo_gives_single_domain_interaction(axis):
    pytest.importorskip("oracle.pyoracle")
    _spawn(_halo_worker, axis)


def test_exchange_protocol_invariants():
    _spawn(_protocol_worker)


def _bodies_worker(rank, world, port):
    """3. Floating bodies and mDBC on slabs (no GPU), on the wave flume (case.py
    WaveFlumeCase, the bench's cfg4 generator): (a) the body force/torque sums of
    k_ft_partial restated in numpy over each rank's OWNED floating particles, all-reduced
    (SUM) over gloo, equal the single-domain sums to float rounding; (b) the post-mDBC
    face records: the owned boundary particles a rank sends from its first/last W owned
    columns are exactly the boundary ghosts its neighbour holds in its W ghost columns
    (W = 2 with mDBC: a ghost node's search reaches one column past the face)."""
    _init(rank, world, port)
    from dualsphysics_multilayer_amd.case import WaveFlumeCase
    from dualsphysics_multilayer_amd.core import case_derive, slab_partition

    case = WaveFlumeCase(0.025, tboundary=2)
    k = case_derive(case.case_def())
    bounds = slab_partition(case, world, 0.3)
    col = _columns(case, k)
    c0, c1 = int(bounds[rank]), int(bounds[rank + 1])
    owned = (col >= c0) & (col < c1)
    # (a) floating sums: ace from a seeded generator, identical on every rank
    rng = np.random.default_rng(11)
    ace = rng.normal(size=(case.np, 3)).astype(np.float32)
    f = case.floatings[0]
    sel = np.arange(f["idbegin"], f["idbegin"] + f["count"])
    cen = np.array(f["center"])
    massp = np.float32(f["masspart"])

    def sums(idx):
        force = ace[idx] * massp
        d = (case.pos[idx] - cen).astype(np.float32)
        tq = np.cross(d, force)
        return np.concatenate([force.sum(axis=0, dtype=np.float64), tq.sum(axis=0, dtype=np.float64)])

    mine = sel[owned[sel]]
    t = torch.from_numpy(sums(mine).astype(np.float32))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    whole = sums(sel)
    assert np.allclose(t.numpy(), whole, rtol=1e-5, atol=1e-6 * np.abs(whole).max()), (t.numpy(), whole)
    cnt = torch.tensor([len(mine)], dtype=torch.int64)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    assert int(cnt.item()) == f["count"], "floating particles not partitioned"
    # (b) face records vs the neighbours' boundary ghosts
    isb = np.arange(case.np) < case.npb
    left = rank - 1 if rank > 0 else None
    right = rank + 1 if rank + 1 < world else None
    W = int(k["scelldiv"]) + 1  # ghost columns per face with mDBC (sph_solver.cpp ghost_width)
    send_l = case.idp[isb & owned & (col < c0 + W)] if left is not None else np.zeros(0, np.uint32)
    send_r = case.idp[isb & owned & (col >= c1 - W)] if right is not None else np.zeros(0, np.uint32)
    got_from_left = _sendrecv_arrays([send_r], right, left, [np.uint32])
    got_from_right = _sendrecv_arrays([send_l], left, right, [np.uint32])
    if left is not None:
        ghosts = case.idp[isb & (col >= c0 - W) & (col < c0)]
        assert np.array_equal(np.sort(got_from_left[0]), np.sort(ghosts))
    if right is not None:
        ghosts = case.idp[isb & (col >= c1) & (col < c1 + W)]
        assert np.array_equal(np.sort(got_from_right[0]), np.sort(ghosts))
    dist.destroy_process_group()


def test_bodies_and_mdbc_faces_on_slabs():
    _spawn(_bodies_worker)
