"""bench.py's N>1 path as the driver runs it (python -m torch.distributed.run ... bench.py
--gpus N), here with 2 ranks sharing the box's one GPU over the shared-memory transport
(RCCL refuses two ranks on one device; everything but the transport is the RCCL ranks'
code): the one JSON line carries the weak-scaling headline of the N ranks AND the
strong-scaling cfg3 measurement (`strong_scaling_cfg3`) beside it, both on slabs."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_emits_weak_and_strong_scaling_lines():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--transport", "shm", "--ranks-per-gpu", "2", "--steps", "3", "--warmup", "1",
           "--cfg3-steps", "2", "--no-cpu-baseline", "--developed-presteps", "0", "--repartition", "0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["parallelism"].startswith("slab-y2")
    assert sum(d["config"]["owned_np_per_rank"]) == d["config"]["np"]
    s3 = d["strong_scaling_cfg3"]
    assert s3 is not None and s3["n_gpus"] == 2 and s3["np"] == 9969118
    assert s3["parallelism"].startswith("slab-y2") and sum(s3["owned_np_per_rank"]) == s3["np"]
    assert s3["value"] > 0 and s3["ms_per_step"] > 0
