"""Which particles the 512 x 2 fused update gets wrong (profiles/r06/gpu18.sh): one Verlet
step with the incremental divide (fused update) vs the radix divide (per-particle update),
compared by idp; the differing particles' slots p before the step (p % 1024 >= 512: the
thread's second particle)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dualsphysics_multilayer_amd.case import DamBreakCase  # noqa: E402
from dualsphysics_multilayer_amd.core import SphGpuSingle  # noqa: E402


def solver(case, mode):
    if mode == "full":
        os.environ["SPH_DIVIDE"] = "full"
    else:
        os.environ.pop("SPH_DIVIDE", None)
    s = SphGpuSingle(case, device=0)
    os.environ.pop("SPH_DIVIDE", None)
    return s


import copy  # noqa: E402

case = copy.copy(DamBreakCase(0.02, celldomfixed=True))
case.vel = case.vel.copy()
rng = np.random.default_rng(3)
fl = np.arange(case.npb, case.np)
pick = rng.choice(fl, int(0.5 * len(fl)), replace=False)
case.vel[pick] = rng.uniform(-3.0, 3.0, size=(len(pick), 3))  # tests/test_divide_inc.py's stirred case
a, b = solver(case, "inc"), solver(case, "full")
for step in range(8):
    pre = a.particles()
    slot = {int(i): k for k, i in enumerate(pre["idp"])}
    a.run(1)
    b.run(1)
    pa, pb = a.particles(), b.particles()
    oa, ob = np.argsort(pa["idp"]), np.argsort(pb["idp"])
    for key in ("pos", "vel", "rhop"):
        xa, xb = pa[key][oa], pb[key][ob]
        d = np.abs(xa - xb).reshape(len(oa), -1).max(axis=1)
        bad = np.nonzero(d > 0)[0]
        ids = pa["idp"][oa][bad]
        slots = np.array([slot[int(i)] for i in ids])
        if key == "pos" and len(bad):
            j = bad[0]
            print("  idp", int(ids[0]), "inc", xa[j].tolist(), "full", xb[j].tolist(), "code", int(pa["code"][oa][j]) if "code" in pa else None)
        print("step", step + 1, key, "differ", len(bad), "of", len(oa), "max", float(d.max()) if len(d) else 0,
              "slot%1024>=512:", int(np.sum(slots % 1024 >= 512)), "npb", case.npb,
              "first slots", slots[:12].tolist(), "first d", d[bad][:6].tolist())
a.close()
b.close()
