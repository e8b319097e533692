"""The 8-GPU cfg3 strong-scaling estimate from measured terms.

    python3 profiles/t8_model.py <turns log> <trace breakdown json> <cfg3 single bench json> [out.json]

Inputs, all from one box: the 8 y-slab turns run (SPH_SLAB_TURNS=2: every kernel of a slab's
step alone on the GPU; profiles/slab_turns.py), the kernel trace of the same mode
(profiles/turns2_breakdown.py: per slab the kernel time and the GPU-idle time before its
kernels, split into idle after one of its own kernels and idle after another slab's), and the
single-domain cfg3 step (bench.py --workload cfg3).  Two estimates of T1 / T8:

  A (round 5's method): the heaviest slab's kernels per step (HIP events) + the whole run's
    GPU-idle time spread over the eight slabs, (wall - sum of all slabs' kernels) / 8 —
    including the turn chain's hand-overs, which a slab on its own GPU does not have;
  B (per-slab critical path): the heaviest slab's kernels + its own idle gaps per call, from
    the trace (launch gaps, the exchange's host wait), x 2 calls per Symplectic step —
    without the hand-overs between slabs of the measurement mode.

Neither includes the xGMI transfer time (the in-process copies of the face messages,
migrants and ghost records are in the kernel terms, as device-to-device blits) or the
latency of RCCL's dt all-reduce across eight GPUs; neither can be measured on one GPU.
"""
import json
import sys


def last_json(path):
    return json.loads([ln for ln in open(path) if ln.startswith("{")][-1])


def main():
    turns = last_json(sys.argv[1])
    trace = json.load(open(sys.argv[2]))["slabs"]
    single = last_json(sys.argv[3])
    t1 = float(single["ms_per_step"])
    summ = turns["summary_min_over_repeats"]["inplace"]
    kern = summ["slab_kernels_ms_per_step"]
    wall = summ["wall_ms_per_step"]
    rest = (wall - sum(kern)) / len(kern)
    t8a = max(kern) + rest
    # the timed run's threads: the trace holds the warm-up run's slab threads too (its own
    # threads, fewer calls); keep the last len(kern) threads
    thr = sorted(trace, key=int)[-len(kern):]
    per = [{"thread": t, "kernels_us_per_call": trace[t]["total_us_per_call"],
            "idle_own_us_per_call": trace[t]["idle_own_us_per_call"],
            "idle_handover_us_per_call": trace[t]["idle_handover_us_per_call"],
            "top_kernels_us_per_call": dict(list(trace[t]["us_per_call"].items())[:8])} for t in thr]
    crit = max(p["kernels_us_per_call"] + p["idle_own_us_per_call"] for p in per)
    t8b = 2.0 * crit / 1e3
    out = {
        "note": __doc__.strip().splitlines()[0],
        "t1_single_ms_per_step": round(t1, 4),
        "turns_wall_ms_per_step": wall,
        "owned_np": turns["runs"][0]["owned_np"],
        "bounds": turns["bounds"],
        "slab_kernels_ms_per_step_events": kern,
        "rest_ms_per_step_A": round(rest, 4),
        "per_slab_trace": per,
        "A": {"t8_ms_per_step": round(t8a, 4), "speedup": round(t1 / t8a, 3)},
        "B": {"critical_us_per_call": round(crit, 1), "t8_ms_per_step": round(t8b, 4),
              "speedup": round(t1 / t8b, 3)},
        "not_measured": ["xGMI transfer time (in-process blits stand in)", "RCCL dt all-reduce latency"],
    }
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("t1_single_ms_per_step", "turns_wall_ms_per_step", "A", "B")}))


if __name__ == "__main__":
    main()
