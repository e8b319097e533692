"""The slab ghost exchange beside the interior interaction, traced (run under rocprofv3).

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- \
        python3 profiles/slab_overlap.py [--slabs 8] [--steps 6] [--overlap 1]

BASELINE cfg3 (10M dam break, Symplectic + DDT) in in-process slabs on one GPU (the
LocalTransport: device-to-device copies instead of RCCL over xGMI).  Each slab runs on its
own host thread and streams, so the trace shows, per slab (launching thread), the ghost
copies of a divide on the exchange stream while that slab's interior k_fluid_tiled launch
(grid of nblocks - 64 blocks) runs on its solver stream.  profiles/overlap_summary.py reads
the trace.  Also prints the wall time per step of the timed steps.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from dualsphysics_multilayer_amd.case import DamBreakCase  # noqa: E402
from dualsphysics_multilayer_amd.core import SphSlabGroup, slab_partition  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slabs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--overlap", type=int, default=1)
    ap.add_argument("--dp", type=float, default=0.00205)
    a = ap.parse_args()
    case = DamBreakCase(a.dp, step_algorithm=2, tdensity=1)
    b = slab_partition(case, a.slabs)
    g = SphSlabGroup(case, np.asarray(b, np.int32))
    g.set_overlap(bool(a.overlap))
    g.run(a.warmup)
    t0 = time.time()
    g.run(a.steps)
    dt = time.time() - t0
    st = g.stats()
    print("slabs %d bounds %s np %d owned %s overlap %d: %.3f ms/step (wall, %d steps)" %
          (a.slabs, list(map(int, b)), case.np, [s["np"] for s in st], a.overlap, 1e3 * dt / a.steps, a.steps),
          flush=True)


if __name__ == "__main__":
    main()
