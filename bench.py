"""Benchmark: particle-steps/s of the SPH hot path on the dam break (BASELINE.json).

A "step" is one JSphGpuSingle::ComputeStep + RunCellDivide over the whole particle
set (interaction, dt, update, cell sort).  Inputs are resident in HBM when the
timed region starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2|cfg3|cfg4]
                    [--dp DP] [--no-cpu-baseline]

Workloads:
  cfg2 (default): 3D dam break, WCSPH + artificial viscosity + DDT2, Verlet.  N=1: the
        BASELINE cfg2 case (1,025,964 particles).  N>1 (torchrun, one process per GPU):
        weak scaling — a dam break of ~N x 1,025,964 particles slab-decomposed across the
        N ranks (y-slabs by default for the dam breaks, --slab-axis; RCCL halo/migration
        exchange + max-allreduce of the dt maxima inside libsphcore); value = all
        particles x steps / max rank time.
  cfg3: BASELINE cfg3, 3D dam break of ~10M particles (dp 0.00205), Symplectic + DDT
        (Molteni, delta-SPH) 0.1, slab-split over N ranks (strong scaling).
  cfg4: BASELINE cfg4, wave flume of ~4.0M particles (dp 0.00265): piston (mvrectsinu) +
        flap (mvrotsinu) moving boundaries, a floating box (RigidAlgorithm=1), mDBC,
        Verlet + DDT2; N>1: the same case slab-split over N ranks (strong scaling; body
        force sums summed over the ranks, mDBC face densities re-sent after the correction).
torch.distributed (gloo, host only) bootstraps the RCCL id, barriers and reduces the
timings; the data path never goes through torch.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "particle-steps/sec (whole node) + achieved HBM GB/s, dam-break 1M/10M"
PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector (= FP32 MFMA) peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
# Algorithmic work model: FP32 ops per fluid pair.
FLOP_REAL_FLUID_PAIR = 135
FLOP_REJECTED_CANDIDATE = 22
FLOP_REAL_BOUND_PAIR = 45  # bound p1: kernel fac + continuity + visc-dt only
# NN multiphase pair (sph_nn.hip nn_pair, Laminar + FDA, DDT Fourtakas, shifting; counted in
# DESIGN.md §4b): kernel 8, pressure 9, continuity 9, DDT 16, shifting 5, visc-dt 5, FDA
# gradient + strain-rate invariant 43, effective viscosity 17, Morris term 10 -> 126; a
# bound p1 pair (continuity + visc-dt) 25; rejected candidates as above.
FLOP_NN_PAIR = 126
FLOP_NN_BOUND_PAIR = 25
BYTES_PER_PARTICLE_STEP = {1: 356, 2: 712}  # Verlet / Symplectic, SURVEY.md §8(d)


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def usable_cpus() -> int:
    """CPUs this process may really use: the affinity mask, capped by the cgroup v2 CPU quota
    (a 16-CPU cgroup on a 256-thread host must not run 64 OpenMP threads)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q[0] != "max":
            n = min(n, max(1, int(float(q[0]) / float(q[1]))))
    except (OSError, ValueError, IndexError):
        pass
    return max(1, n)


def host_info(threads: int) -> dict:
    """What the CPU baseline ran on: logical CPUs of the machine, CPUs this process may use,
    the CPU model, and the thread rule (BASELINE.md asks for count and model)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    quota = None
    try:  # cgroup v2 CPU quota ("max" or "<quota> <period>"): the CPUs this job may really use
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q[0] == "max" else float(q[0]) / float(q[1])
    except (OSError, ValueError, IndexError):
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "cpu_model": model,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "thread_rule": "threads = min(usable CPUs, 64), usable = min(sched_getaffinity, cgroup CPU quota): "
                           "the reference at its best on the CPUs this job may use (it caps OpenMP at "
                           "OMP_MAXTHREADS=64, OmpDefs.h:39); `oversubscribed` times min(nproc, 64) threads "
                           "on the same CPUs, the literal BASELINE.md rule", "threads": threads}


def _ref_run(exe: str, case: str, out: str, nsteps: int, threads: int, extra=()) -> float:
    """Simulation Runtime (step loop, s) of one reference run of `nsteps` steps."""
    subprocess.run([exe, case, out, "-nsteps:%d" % nsteps, "-sv:none", "-svres:0", "-ompthreads:%d" % threads]
                   + list(extra), capture_output=True, text=True, check=True, timeout=900)
    log = open(os.path.join(out, "Run.out")).read()
    return float(re.search(r"Simulation Runtime\.*:\s*([0-9.eE+-]+)", log).group(1))


def reference_cpu_baseline(dp: float, nsteps: int, threads: int, step: int = 1, ddt: int = 2,
                           boundary: int = 1, flume: bool = False, first: int = 10, nn_width: float = 0.0,
                           cellmode: str = "full") -> dict | None:
    """Times the REFERENCE CPU solver (oracle/_ref, built from the reference sources)
    on the same dam break (or wave flume, or -- nn_width > 0 -- the v5.0 NN solver on the
    NN wet dam break) over the step window [first, first+nsteps) (steps
    10-110): two runs of `first` and `first+nsteps` steps, the difference of their
    'Simulation Runtime' (step loop only, no output) over nsteps.  `cellmode` is passed
    to the reference as -cellmode:<mode>, so both sides run the same cell division."""
    ref = os.path.join(ROOT, "oracle", "_ref")
    exe = os.path.join(ref, "DualSPHysics5.0NN_CPU_ref" if nn_width else "DualSPHysics5.2CPU_ref")
    gen = os.path.join(ref, "gennn_ref" if nn_width else "genflume_ref" if flume else "gencase_ref")
    name = "CaseNN" if nn_width else "CaseFlume" if flume else "CaseDambreak"
    if not (os.path.exists(exe) and os.path.exists(gen)):
        return None
    tmp = tempfile.mkdtemp(prefix="sphref_")
    try:
        if nn_width:
            args = [gen, repr(dp), tmp, repr(nn_width), "1", "5", name]
        else:
            args = [gen, repr(dp), tmp, str(step), str(ddt), "1.5", name, str(boundary)]
        out = subprocess.run(args, capture_output=True, text=True, check=True).stdout
        np_ = int(re.search(r"np=(\d+)", out).group(1))
        case = os.path.join(tmp, name)
        extra = () if nn_width else ("-cellmode:%s" % cellmode,)
        t_a = _ref_run(exe, case, os.path.join(tmp, "a"), first, threads, extra)
        t_b = _ref_run(exe, case, os.path.join(tmp, "b"), first + nsteps, threads, extra)
        sec = t_b - t_a
        return {"value": np_ * nsteps / sec, "unit": "particle-steps/s", "cores": threads, "kind": "reference",
                "window_steps": [first, first + nsteps], "window_seconds": sec,
                "sample": "reference %s CPU (built from /root/reference sources, -O3 -fopenmp "
                          "-ffast-math), %d-particle %s (%s), %s, -cellmode:%s, steps %d-%d (Simulation Runtime "
                          "of a %d-step run minus that of a %d-step run), -ompthreads:%d"
                          % ("DualSPHysics5.0 NNewtonian" if nn_width else "DualSPHysics5.2", np_,
                             "NN 3-phase wet dam break" if nn_width else "wave flume" if flume else "dam break",
                             "mDBC" if boundary == 2 else "DBC",
                             "Verlet" if step == 1 else "Symplectic", cellmode, first, first + nsteps,
                             first + nsteps, first, threads)}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write("reference CPU baseline failed: %r\n" % (e,))
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def port_cpu_baseline(case, nsteps: int, threads: int) -> dict:
    from oracle.pyoracle import OracleSolver

    o = OracleSolver(case, nthreads=threads)
    o.run(nsteps)
    sec = o.run_seconds()
    return {"value": case.np * nsteps / sec, "unit": "particle-steps/s", "cores": o.threads(), "kind": "port",
            "sample": "oracle restatement of JSphCpu (C++/OpenMP, -O3 -ffast-math), %d particles, %d steps"
                      % (case.np, nsteps)}


def profiled_traffic(kernel_prefix, np_: int, workload: str):
    """HBM bytes per launch of the dominant kernel from the latest committed PMC passes
    (profiles/<round>/pmc_traffic.json: 2*FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md
    §HBM) of the same workload on one GPU; None if there is none."""
    import glob

    found = None
    for d in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*"))):
        tj, bj = os.path.join(d, "pmc_traffic.json"), os.path.join(d, "bench.json")
        if not (os.path.exists(tj) and os.path.exists(bj)):
            continue
        try:
            b = json.load(open(bj))
            if b["config"]["np"] != np_ or b["n_gpus"] != 1 or not b["config"]["workload"].startswith(workload):
                continue
            prefixes = (kernel_prefix,) if isinstance(kernel_prefix, str) else tuple(kernel_prefix)
            for k, v in json.load(open(tj)).items():
                if k.startswith(prefixes):
                    found = {"bytes": v["traffic_bytes_per_launch"], "avg_ns": v.get("avg_ns"),
                             "source": os.path.relpath(tj, ROOT) + " (2*FETCH_SIZE + WRITE_SIZE, %s)" % k}
        except (KeyError, ValueError):
            continue
    return found


def profiled_valu_flop(kernel_prefix, np_: int, workload: str):
    """EXECUTED FP32 flop per launch of the dominant kernel from the latest committed PMC
    passes of the same workload (profiles/<round>/pmc/counters.json, per-dispatch averages):
    64 lanes x (ADD + MUL + TRANS + 2 FMA) F32 wave-instructions, the
    counter-based counterpart of the algorithmic flop model; None if there is none."""
    import glob

    found = None
    for d in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*"))):
        cj, bj = os.path.join(d, "pmc", "counters.json"), os.path.join(d, "bench.json")
        if not (os.path.exists(cj) and os.path.exists(bj)):
            continue
        try:
            b = json.load(open(bj))
            if b["config"]["np"] != np_ or b["n_gpus"] != 1 or not b["config"]["workload"].startswith(workload):
                continue
            prefixes = (kernel_prefix,) if isinstance(kernel_prefix, str) else tuple(kernel_prefix)
            for k, v in json.load(open(cj)).items():
                if (k[5:] if k.startswith("void ") else k).startswith(prefixes):
                    fl = 64.0 * (v["SQ_INSTS_VALU_ADD_F32"] + v["SQ_INSTS_VALU_MUL_F32"] + v["SQ_INSTS_VALU_TRANS_F32"]
                                 + 2.0 * v["SQ_INSTS_VALU_FMA_F32"])
                    found = {"flop": fl, "source": os.path.relpath(cj, ROOT) + " (%s)" % k}
        except (KeyError, ValueError):
            continue
    return found


CFG2_DP, CFG2_NP = 0.0045, 1025964
CFG3_DP = 0.00205  # 9,969,118 particles (BASELINE cfg3: ~10M)
CFG4_DP = 0.00265  # 4,007,978 particles (BASELINE cfg4: wave flume ~4M)
CFG5_DP, CFG5_WIDTH = 0.01, 0.70  # ~2.0M particles (BASELINE cfg5: NN multiphase 2M), the example's dp


def weak_dp(target_np: int) -> float:
    """Largest dp whose dam break has >= target_np particles (np falls as dp grows)."""
    from dualsphysics_multilayer_amd.case import dambreak_np

    lo, hi = 1e-4, CFG2_DP  # np(lo) >= target >= ... ; bisect on the step function
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        if dambreak_np(mid) >= target_np:
            lo = mid
        else:
            hi = mid
    return float("%.6g" % lo)


def measure(case, args, rank: int, world: int, device: int, dist, use_slab: bool, steps: int, warmup: int,
            presteps: int) -> dict:
    """Build the solver (one domain, or this rank's x-slab), run presteps + warmup untimed
    steps, then time exactly `steps` steps between barriers + device syncs; the elapsed
    time is the max over ranks and the units (particles x steps) their sum."""
    from dualsphysics_multilayer_amd.core import SphGpuSingle, SphGpuSlab, comm_unique_id, slab_partition

    bounds = None
    s = None
    t_setup = time.perf_counter()
    if use_slab:
        import torch

        # A failed slab setup on any rank ends every rank with a non-zero status: the run
        # never degrades into per-GPU replicas.
        err = None
        try:
            bounds = slab_partition(case, world, args.bound_weight, args.axis)
            if args.transport == "shm":
                import uuid

                ids = ["/sphbench_%s" % uuid.uuid4().hex[:12] if rank == 0 else None]
            else:
                ids = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(ids, src=0)
            s = SphGpuSlab(case, rank, world, bounds, ids[0], device=device, transport=args.transport,
                           slot_bytes=256 << 20, axis=args.axis)
            if args.repartition and world > 1:
                s.set_repartition(args.repartition, args.bound_weight, 0.05)
            s.run(presteps + warmup)
            s.sync()
            ok = torch.tensor([1], dtype=torch.int32)
        except Exception as e:  # noqa: BLE001
            err = e
            ok = torch.tensor([0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            sys.stderr.write("rank %d: slab run failed: %r\n" % (rank, err if err else "failed on another rank"))
            raise SystemExit(3)
    else:
        s = SphGpuSingle(case, device=device)
        s.run(presteps + warmup)
        s.sync()
    setup_s = time.perf_counter() - t_setup
    pairs0 = s.count_pairs()

    def barrier():
        if dist is not None:
            import torch

            if world > 1:  # a one-rank slab run (--force-slab) has no one to wait for
                dist.barrier()
            torch.cuda.synchronize(device)

    # The timed region records HIP events around the interaction only (the roofline's launch
    # time): every timed phase puts two markers in the stream, and timing all four costs
    # ~18 us per 1M-particle Verlet step.  The per-phase breakdown comes from a second,
    # untimed run of the same length right after.
    s.set_timing(True, phases=1)
    s.sync()
    barrier()
    t0 = time.perf_counter()
    s.run(steps)
    s.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    inter_ms, nlaunch = s.timing()
    pairs1 = s.count_pairs()
    s.set_timing(True)
    s.run(steps)
    phase_ms, _ = s.timing()
    phase_ms[0] = inter_ms[0]  # the interaction as timed inside the timed region
    st = s.stats()
    units = float(st["np"]) * steps
    per_rank_np = [int(st["np"])]
    slab_info = None
    if dist is not None:
        import torch

        tmax = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tot = torch.tensor([units], dtype=torch.float64)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        nps = [None] * world
        dist.all_gather_object(nps, int(st["np"]))
        infos = [None] * world
        dist.all_gather_object(infos, s.slab_info() if bounds is not None else None)
        elapsed, units, per_rank_np, slab_info = float(tmax.item()), float(tot.item()), nps, infos
    s.close()
    return dict(setup_s=setup_s, elapsed=elapsed, units=units, phase_ms=phase_ms, nlaunch=nlaunch, pairs0=pairs0,
                pairs1=pairs1, st=st, bounds=bounds, per_rank_np=per_rank_np, slab_info=slab_info)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=("cfg2", "cfg3", "cfg4", "cfg5"), default="cfg2")
    ap.add_argument("--dp", type=float, default=None, help="override the particle spacing")
    ap.add_argument("--boundary", choices=("dbc", "mdbc"), default=None,
                    help="boundary conditions (mdbc: modified DBC, Vel0, normals to the wall limit)")
    ap.add_argument("--bound-weight", type=float, default=0.3, help="slab balance weight of a bound particle")
    ap.add_argument("--cellmode", choices=("full", "half"), default="full",
                    help="cfg2/cfg3 cell size: full = 2h (the reference default), half = h (-cellmode:half)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=100,
                    help="reference CPU steps timed (window 10 .. 10+K, BASELINE.md: 10-110)")
    ap.add_argument("--repartition", type=int, default=20,
                    help="N>1: re-balance the slab bounds every K steps when the load is >5%% off (0: never)")
    ap.add_argument("--transport", choices=("rccl", "shm"), default="rccl",
                    help="N>1 slab transport: rccl (one process per GPU, the product path) or shm "
                         "(host-staged shared memory: ranks of one node without RCCL)")
    ap.add_argument("--ranks-per-gpu", type=int, default=1,
                    help="ranks sharing one GPU (device = LOCAL_RANK // this; needs --transport shm)")
    ap.add_argument("--presteps", type=int, default=None,
                    help="untimed steps before the warmup (default: 10 - warmup, so the timed window starts "
                         "at step 10 as BASELINE.md's 10-110); large values time a developed flow")
    ap.add_argument("--developed-presteps", type=int, default=8000,
                    help="cfg2 N=1: also time the same steps after this many steps (a developed flow, key "
                         "`developed_flow`; 0: skip)")
    ap.add_argument("--no-cfg3", action="store_true",
                    help="cfg2: skip the extra cfg3 (10M, Symplectic) timing (keys cfg3_1gpu / strong_scaling_cfg3)")
    ap.add_argument("--cfg3-steps", type=int, default=10, help="timed steps of the extra cfg3 measurement")
    ap.add_argument("--slab-axis", choices=("auto", "x", "y"), default="auto",
                    help="N>1 slab axis: y keeps every x row of cells whole on one rank (the dam breaks: "
                         "their load is spread evenly along y; DESIGN.md §6); auto = y for cfg2/cfg3, x otherwise")
    ap.add_argument("--force-slab", action="store_true",
                    help="run the N>1 code path (gloo bootstrap + RCCL slab) even with one rank")
    args = ap.parse_args()
    if args.presteps is None:
        args.presteps = max(0, 10 - args.warmup)
    if args.boundary is None:
        args.boundary = "mdbc" if args.workload == "cfg4" else "dbc"
    args.axis = {"x": 0, "y": 1}.get(args.slab_axis, 1 if args.workload in ("cfg2", "cfg3") else 0)

    rank, world, local = dist_env()
    if args.gpus != world and world > 1:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.ranks_per_gpu > 1 and args.transport == "rccl":
        raise SystemExit("--ranks-per-gpu > 1 needs --transport shm (RCCL refuses two ranks on one device)")
    device = local // max(1, args.ranks_per_gpu)
    use_slab = world > 1 or args.force_slab
    dist = None
    if use_slab:
        import torch
        import torch.distributed as dist

        # host-side bootstrap only (RCCL id broadcast, barriers, timing reduction)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from dualsphysics_multilayer_amd.case import DamBreakCase, WaveFlumeCase, WetDambreakNNCase

    cmode = 2 if args.cellmode == "half" else 1
    if cmode == 2 and args.workload not in ("cfg2", "cfg3"):
        raise SystemExit("--cellmode half applies to the dam-break workloads (cfg2, cfg3)")
    if args.workload == "cfg2":
        dp = args.dp or (CFG2_DP if world == 1 else weak_dp(world * CFG2_NP))
        case = DamBreakCase(dp, tboundary=2 if args.boundary == "mdbc" else 1, cellmode=cmode)
    elif args.workload == "cfg3":
        dp = args.dp or CFG3_DP
        case = DamBreakCase(dp, step_algorithm=2, tdensity=1, tboundary=2 if args.boundary == "mdbc" else 1,
                            cellmode=cmode)
    elif args.workload == "cfg4":
        dp = args.dp or CFG4_DP
        case = WaveFlumeCase(dp, tboundary=2 if args.boundary == "mdbc" else 1)
    else:
        dp = args.dp or CFG5_DP
        case = WetDambreakNNCase(dp, width=CFG5_WIDTH)
    wall = {}
    t_setup = time.perf_counter()
    m = measure(case, args, rank, world, device, dist, use_slab, args.steps, args.warmup, args.presteps)
    wall["setup_and_warmup_s"] = m["setup_s"]
    elapsed, units, phase_ms, nlaunch = m["elapsed"], m["units"], m["phase_ms"], m["nlaunch"]
    pairs0, pairs1, st, bounds, per_rank_np, slab_info = (m["pairs0"], m["pairs1"], m["st"], m["bounds"],
                                                          m["per_rank_np"], m["slab_info"])
    del t_setup
    # North star's strong-scaling target is cfg3 (~10M, Symplectic + DDT) from 1 to 8 GPUs:
    # time it beside the headline line -- on one GPU as `cfg3_1gpu`, on N ranks as
    # `strong_scaling_cfg3` -- so one scaling run yields the 1 -> N strong-scaling ratio.
    cfg3_extra = None
    if args.workload == "cfg2" and not args.no_cfg3 and args.dp is None and args.cellmode == "full":
        t3 = time.perf_counter()
        c3 = DamBreakCase(CFG3_DP, step_algorithm=2, tdensity=1)
        a3 = argparse.Namespace(**vars(args))
        a3.axis = {"x": 0, "y": 1}.get(args.slab_axis, 1)  # the cfg3 dam break: y-slabs unless told otherwise
        m3 = measure(c3, a3, rank, world, device, dist, world > 1 or args.force_slab, args.cfg3_steps, 2, 0)
        cfg3_extra = {"workload": "BASELINE cfg3: 3D dam break, %d particles (dp=%g), Symplectic, DDT (Molteni) "
                                  "0.1, DBC, CellMode full" % (c3.np, CFG3_DP),
                      "np": c3.np, "n_gpus": world, "steps": args.cfg3_steps, "warmup": 2,
                      "ms_per_step": m3["elapsed"] / args.cfg3_steps * 1e3,
                      "value": m3["units"] / m3["elapsed"], "unit": "particle-steps/s",
                      "interaction_ms_per_call": float(m3["phase_ms"][0]),
                      "divide_ms_per_call": float(m3["phase_ms"][2]),
                      "parallelism": ("slab-%s%d (%s)" % ("xy"[a3.axis], world,
                                                           "RCCL" if args.transport == "rccl" else "shared-memory"))
                                     if m3["bounds"] is not None else "single",
                      "slab_bounds_cells": None if m3["bounds"] is None else [int(b) for b in m3["bounds"]],
                      "owned_np_per_rank": m3["per_rank_np"],
                      "wall_s": time.perf_counter() - t3}

    # The flow after --developed-presteps steps (the surge under way: more particles change
    # cells, so the incremental divide does more work than in the first steps from rest).
    developed = None
    if (args.workload == "cfg2" and world == 1 and not args.force_slab and args.developed_presteps > 0
            and args.presteps < args.developed_presteps):
        t4 = time.perf_counter()
        m4 = measure(case, args, rank, world, device, dist, False, args.steps, args.warmup, args.developed_presteps)
        developed = {"presteps": args.developed_presteps, "steps": args.steps,
                     "timed_window": [args.developed_presteps + args.warmup,
                                      args.developed_presteps + args.warmup + args.steps],
                     "ms_per_step": m4["elapsed"] / args.steps * 1e3, "value": m4["units"] / m4["elapsed"],
                     "unit": "particle-steps/s", "interaction_ms_per_call": float(m4["phase_ms"][0]),
                     "divide_ms_per_call": float(m4["phase_ms"][2]), "wall_s": time.perf_counter() - t4}

    if rank == 0:
        pairs = (pairs0.astype("float64") + pairs1.astype("float64")) / 2.0
        ff_chk, ff_real, fb_chk, fb_real, bf_chk, bf_real = pairs
        nn = args.workload == "cfg5"
        fpair, fbound = (FLOP_NN_PAIR, FLOP_NN_BOUND_PAIR) if nn else (FLOP_REAL_FLUID_PAIR, FLOP_REAL_BOUND_PAIR)
        flops = (fpair * (ff_real + fb_real) + FLOP_REJECTED_CANDIDATE * (ff_chk - ff_real + fb_chk - fb_real)
                 + fbound * bf_real + FLOP_REJECTED_CANDIDATE * (bf_chk - bf_real))
        inter_ms = float(phase_ms[0])
        achieved = flops / (inter_ms * 1e-3) / 1e12 if inter_ms > 0 else None
        value = units / elapsed
        hbm_achieved = value * BYTES_PER_PARTICLE_STEP[case.step_algorithm] / 1e9
        # the tiled kernel's instantiation: DDT mode (| 8: Fourtakas term as its series),
        # floating records, cell mode (sph_interaction_tiled.hip launch_fluid_tiled_s)
        ftb = "true" if getattr(case, "floatings", None) else "false"
        kname = (["sphx::k_nn_tiled<%d, %d, true," % (case.tvisco, case.tdensity)] if nn else
                 ["sphx::k_fluid_tiled%s<%d, %s, %d>" % (w4, td, ftb, case.cellmode)
                  for td in ((case.tdensity | 8, case.tdensity) if case.tdensity >= 2 else (case.tdensity,))
                  for w4 in ("", "_w4")])  # _w4: the 4-wave register budget (DDT1)
        traffic = profiled_traffic(kname, case.np, "BASELINE " + args.workload) if world == 1 else None
        vflop = profiled_valu_flop(kname, case.np, "BASELINE " + args.workload) if world == 1 else None
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "particle-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.workload == "cfg2" else "strong",
            "vs_baseline": None,
            "dtype": "f32 (f64 positions/time integration)",
            "data": ("synthetic: generated wave-flume lattice (case.py WaveFlumeCase = oracle/tools/genflume_ref)"
                     if args.workload == "cfg4" else
                     "synthetic: the NN wet dam break example extruded to 3D (case.py WetDambreakNNCase = "
                     "oracle/tools/gennn_ref)" if nn else
                     "synthetic: generated 3D dam-break lattice (SURVEY.md §8(c) recipe)"),
            "timed_window": [args.presteps + args.warmup, args.presteps + args.warmup + args.steps],
            "config": {
                "workload": (("BASELINE cfg2: 3D dam break, %d particles (dp=%g), Verlet, Wendland, artificial "
                              "viscosity 0.1, DDT2 0.1, %s, CFL 0.2, CellMode %s"
                              % (case.np, dp, args.boundary.upper(), args.cellmode))
                             if args.workload == "cfg2" else
                             ("BASELINE cfg3: 3D dam break, %d particles (dp=%g), Symplectic, Wendland, artificial "
                              "viscosity 0.1, DDT (Molteni delta-SPH) 0.1, %s, CFL 0.2, CellMode %s"
                              % (case.np, dp, args.boundary.upper(), args.cellmode)) if args.workload == "cfg3" else
                             ("BASELINE cfg4: wave flume, %d particles (dp=%g): piston mvrectsinu + flap mvrotsinu "
                              "moving boundaries, floating box (RigidAlgorithm=1, %d particles), %s, Verlet, "
                              "Wendland, artificial viscosity 0.1, DDT2 0.1, CFL 0.2"
                              % (case.np, dp, case.case_nfloat, args.boundary.upper())) if args.workload == "cfg4" else
                             ("BASELINE cfg5: NN multiphase (v5.0 NNewtonian solver), 3-phase wet dam break extruded to "
                              "3D, %d particles (dp=%g, width %g m), Symplectic, Wendland, FDA velocity gradients, "
                              "Laminar viscosity with the HBP effective viscosity, DDT Fourtakas full 0.1, shifting "
                              "Full (-10, TFS 2.75), CFL 0.1, RelaxationDt 0.2" % (case.np, dp, CFG5_WIDTH))),
                "np": case.np,
                "presteps": args.presteps,
                "npb": case.npb,
                "parallelism": (("slab-%s%d (%s halo + migration, max-allreduce dt%s)"
                                 % ("xy"[args.axis], world, "RCCL" if args.transport == "rccl" else "shared-memory",
                                    "" if args.ranks_per_gpu == 1 else ", %d ranks per GPU" % args.ranks_per_gpu))
                                if bounds is not None else "single"),
                "slab_bounds_cells": None if bounds is None else [int(b) for b in bounds],
                "slab_repartition_every": args.repartition if bounds is not None and world > 1 else None,
                "slab_final_info": slab_info,
                "owned_np_per_rank": per_rank_np,
            },
            "roofline": {
                "kernel": ("k_nn_tiled<tvisco=%d, tdensity=%d> (Interaction_Forces NN)" % (case.tvisco, case.tdensity)
                           if nn else
                           ("k_fluid_tiled<tdensity=%d, floating records> (Interaction_Forces)"
                            if getattr(case, "floatings", None) else "k_fluid_tiled<tdensity=%d> (Interaction_Forces)")
                           % case.tdensity),
                "bound": "valu",
                "bound_note": "FP32-VALU-bound pairwise kernel (no MFMA: irregular pairs); gfx950's FP32 vector "
                              "peak equals its FP32 MFMA peak, 157.3 TFLOP/s",
                "achieved": achieved,
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": (achieved / PEAK_FP32_TFLOPS) if achieved else None,
                "traffic": traffic["bytes"] if traffic else None,
                "traffic_unit": "bytes per launch (HBM, PMC)",
                "traffic_source": traffic["source"] if traffic else None,
                "traffic_profiled_avg_ms": (traffic["avg_ns"] / 1e6) if traffic and traffic["avg_ns"] else None,
                "frac_counters": (vflop["flop"] / (inter_ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS)
                                 if vflop and inter_ms > 0 else None,
                "executed_flop_per_launch_pmc": vflop["flop"] if vflop else None,
                "executed_flop_source": vflop["source"] if vflop else None,
                "avg_launch_ms": inter_ms,
                "launches": int(nlaunch),
                "algorithmic_flop_per_launch": flops,
                "pairs_per_launch": {"ff_checked": ff_chk, "ff_real": ff_real, "fb_checked": fb_chk,
                                     "fb_real": fb_real, "bf_checked": bf_chk, "bf_real": bf_real},
            },
            "roofline_hbm_step": {
                "bound": "hbm",
                "achieved": hbm_achieved,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": hbm_achieved / PEAK_HBM_GBS,
                "bytes_per_particle_step": BYTES_PER_PARTICLE_STEP[case.step_algorithm],
            },
            "phase_ms_per_call": {"interaction": float(phase_ms[0]), "update": float(phase_ms[1]),
                                  "divide": float(phase_ms[2]), "mdbc": float(phase_ms[3])},
            "cpu_baseline": None,
        }
        wall["timed_s"] = elapsed
        if not args.no_cpu_baseline and world == 1:
            # The reference at its best on the CPUs this job may use: min(usable CPUs, 64) threads
            # (it caps OpenMP at OMP_MAXTHREADS=64, OmpDefs.h:39; usable = affinity capped by the
            # cgroup quota, 16 on the GPU box) -> `value`; beside it, on a shorter window, the
            # literal min(nproc, 64) of BASELINE.md, oversubscribed on a CPU-capped box.
            threads = min(usable_cpus(), 64)
            literal = min(os.cpu_count() or 1, 64)
            t_cpu = time.perf_counter()

            def ref_baseline(nthreads, nsteps):
                if nn:  # the v5.0 NN CPU solver runs ~3 s per step at 2M particles: a bounded sample
                    return reference_cpu_baseline(dp, min(nsteps, 6), nthreads, nn_width=CFG5_WIDTH, first=1)
                return reference_cpu_baseline(dp, nsteps, nthreads, case.step_algorithm, case.tdensity,
                                              case.tboundary, flume=args.workload == "cfg4", cellmode=args.cellmode)

            cb = ref_baseline(threads, args.cpu_steps)
            if cb is None and not nn:  # the oracle restates the single-phase solver only
                cb = port_cpu_baseline(case, min(args.cpu_steps, 10), threads)
            if cb is not None:
                cb["gpu_over_cpu"] = value / cb["value"]
                cb["host"] = host_info(threads)
                if literal != threads:
                    cs = ref_baseline(literal, max(args.cpu_steps // 3, 1))
                    if cs is not None:
                        cs["gpu_over_cpu"] = value / cs["value"]
                        cb["oversubscribed"] = cs
            res["cpu_baseline"] = cb
            wall["cpu_baseline_s"] = time.perf_counter() - t_cpu
        wall["process_s"] = time.perf_counter() - T_START
        res["wall_breakdown"] = wall
        res["cfg3_1gpu" if world == 1 else "strong_scaling_cfg3"] = cfg3_extra
        if developed is not None:
            res["developed_flow"] = developed
        print(json.dumps(res))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
