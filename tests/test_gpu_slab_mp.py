"""The slab decomposition across PROCESSES: one process per rank, as
bench.py --gpus N runs it, here on the shared-memory transport (sph_slab_create_shm)
because the test box has one GPU and RCCL refuses two ranks on one device.  Everything
but the transport is the RCCL ranks' code: per-process SphGpuSlab, pack / exchange /
unpack of ghosts and migrants, max-allreduced dt, re-partitioning collectives, the
deadline-bounded waits.  The merged owned particles must match the reference's PARTs."""
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

from golden_io import load, snapshot, steps, tol, maxdiff

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def run_ranks(tmp_path, nranks, golden, layout="balanced", every=0, die_rank=None, timeout_s=None, axis=0,
              commlog=None):
    name = "/sphtest_%s" % uuid.uuid4().hex[:12]
    env = dict(os.environ)
    if timeout_s:
        env["SPH_COMM_TIMEOUT_S"] = str(timeout_s)
    if commlog:
        env["SPH_COMM_LOG"] = str(commlog)
    procs, outs = [], []
    for r in range(nranks):
        out = str(tmp_path / ("rank%d.npz" % r))
        outs.append(out)
        args = [sys.executable, os.path.join(HERE, "slab_rank.py"), str(r), str(nranks), name, golden, out, layout,
                str(every)] + (["die-after-create"] if r == die_rank else []) + ["axis=%d" % axis]
        procs.append(subprocess.Popen(args, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = [p.communicate(timeout=240)[0] for p in procs]
    return [p.returncode for p in procs], outs, logs


def merged(outs, k):
    parts = [np.load(o) for o in outs]
    cat = {q: np.concatenate([p["s%d_%s" % (k, q)] for p in parts]) for q in ("idp", "pos", "vel", "rhop")}
    o = np.argsort(cat["idp"], kind="stable")
    return {q: v[o] for q, v in cat.items()}


@pytest.mark.parametrize("golden,nranks", [("verlet_ddt2_dp0.02", 2), ("symplectic_ddt1_dp0.025", 3),
                                           ("verlet_ddt2_dp0.02", 8)])
def test_processes_match_reference_parts(tmp_path, golden, nranks):
    rc, outs, logs = run_ranks(tmp_path, nranks, golden)
    assert rc == [0] * nranks, logs
    g = load(golden)
    for k in steps(g):
        got, ref = merged(outs, k), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"]), "excluded/duplicated particles"
        tp, tv, tr = tol(k)
        assert maxdiff(got, ref, "pos") <= tp, (k, maxdiff(got, ref, "pos"))
        assert maxdiff(got, ref, "vel") <= tv, (k, maxdiff(got, ref, "vel"))
        assert maxdiff(got, ref, "rhop") <= tr, (k, maxdiff(got, ref, "rhop"))
        times = [float(np.load(o)["s%d_time" % k]) for o in outs]
        assert max(times) == min(times)  # every rank stepped with the same dt


def test_processes_repartition_match_reference_parts(tmp_path):
    """Ranks started far from balance, re-partitioned every 3 steps across processes."""
    golden = "verlet_ddt2_dp0.02"
    rc, outs, logs = run_ranks(tmp_path, 3, golden, layout="skew", every=3)
    assert rc == [0, 0, 0], logs
    g = load(golden)
    for k in steps(g):
        got, ref = merged(outs, k), snapshot(g, k)
        assert np.array_equal(got["idp"], ref["idp"])
        tp, tv, tr = tol(k)
        assert maxdiff(got, ref, "pos") <= tp and maxdiff(got, ref, "vel") <= tv and maxdiff(got, ref, "rhop") <= tr
    info = [np.load(o)["info"] for o in outs]
    assert all(i[2] >= 1 for i in info)


def test_lost_rank_ends_the_others(tmp_path):
    """A rank that disappears after creation: the survivors' next collective times out
    and they end with SPH_ERR_COMM (status 3 of slab_rank.py), not a hang."""
    rc, outs, logs = run_ranks(tmp_path, 2, "verlet_ddt2_dp0.02", die_rank=1, timeout_s=5)
    assert rc[1] == 0 and rc[0] == 3, (rc, logs)
    assert "shm transport" in str(np.load(outs[0])["error"])


def read_comm_logs(d, nranks):
    """Per rank: the list of its transport calls ('X', nsl, nsr, nrl, nrr) / ('M'|'S', n)."""
    logs = []
    for r in range(nranks):
        calls = []
        for line in open(os.path.join(d, "rank%d.log" % r)):
            f = line.split()
            assert int(f[0]) == len(calls) + 1, "calls out of sequence"
            calls.append((f[1],) + tuple(int(x) for x in f[2:]))
        logs.append(calls)
    return logs


@pytest.mark.parametrize("nranks,axis,layout,every", [(8, 0, "balanced", 0), (4, 1, "balanced", 0),
                                                      (8, 0, "skew", 3)],
                         ids=["x_slabs_8", "y_slabs_4", "x_repartition_8"])
def test_transport_conformance(tmp_path, nranks, axis, layout, every):
    """The precondition of the RCCL transport (whose ncclSend / ncclRecv pairs hang instead
    of failing when sizes or order differ), checked on the same host code over 8 processes:
    the shm transport checks every call online (same collective and sequence number on the
    peers, every message sent exactly the size the peer receives, zero-size sides included)
    and logs it; offline, from the ranks' logs: the same sequence of call kinds on every rank,
    (the y split of the 10-row golden case holds 4 ranks of the minimum 2 rows)
    each exchange's send to rank r+1 / r-1 equal to what that rank receives in the same call,
    every reduction of the same length on all ranks."""
    logdir = tmp_path / "comm"
    logdir.mkdir()
    rc, outs, logs = run_ranks(tmp_path, nranks, "verlet_ddt2_dp0.02", layout=layout, every=every, axis=axis,
                               commlog=logdir)
    assert rc == [0] * nranks, logs
    calls = read_comm_logs(str(logdir), nranks)
    n = len(calls[0])
    assert n > 50 and all(len(c) == n for c in calls), [len(c) for c in calls]
    nexch = 0
    for k in range(n):
        kinds = {c[k][0] for c in calls}
        assert len(kinds) == 1, (k, kinds)
        if calls[0][k][0] == "X":
            nexch += 1
            for r in range(nranks):
                _, nsl, nsr, nrl, nrr = calls[r][k]
                if r + 1 < nranks:
                    assert nsr == calls[r + 1][k][3], (k, r, "right send vs its left receive")
                else:
                    assert nsr == 0 and nrr == 0
                if r > 0:
                    assert nsl == calls[r - 1][k][4], (k, r, "left send vs its right receive")
                else:
                    assert nsl == 0 and nrl == 0
        else:
            assert len({c[k] for c in calls}) == 1, (k, [c[k] for c in calls])
    assert nexch > 20
    g = load("verlet_ddt2_dp0.02")
    k = steps(g)[-1]
    got, ref = merged(outs, k), snapshot(g, k)
    assert np.array_equal(got["idp"], ref["idp"])
    tp, tv, tr = tol(k)
    assert maxdiff(got, ref, "pos") <= tp and maxdiff(got, ref, "vel") <= tv and maxdiff(got, ref, "rhop") <= tr
