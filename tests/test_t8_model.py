"""The measurement scripts behind DESIGN §6's 8-GPU estimate (CPU only, synthetic inputs):
profiles/turns2_breakdown.py's per-slab kernel time and its attribution of GPU-idle time
(own gaps vs the turn chain's hand-overs), and profiles/t8_model.py's two estimates."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, timeline):
    """timeline: (thread, start_ns, end_ns, kernel) rows."""
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Thread_Id", "Start_Timestamp", "End_Timestamp",
                                          "Grid_Size_X"])
        w.writeheader()
        for thr, s, e, name in timeline:
            w.writerow({"Kernel_Name": "void sphx::%s(int)" % name, "Thread_Id": thr, "Start_Timestamp": s,
                        "End_Timestamp": e, "Grid_Size_X": 1})


def _turns_chain(nslab=2, ncalls=6, inter=1000, upd=100, own=30, hand=50):
    """Each call: slab 0 interaction, slab 1 interaction, slab 0 update, slab 1 update; a gap of
    `own` ns between a slab's interaction and its update when nothing else ran, `hand` ns at
    every change of slab."""
    rows, t = [], 0
    for _ in range(ncalls):
        for r in range(nslab):
            rows.append((str(100 + r), t, t + inter, "k_fluid_tiled_w4"))
            t += inter + hand
        t -= hand
        for r in range(nslab):
            t += own if r == 0 else hand
            rows.append((str(100 + r), t, t + upd, "k_update_cls"))
            t += upd
        t += hand
    return rows


def test_breakdown_splits_idle_into_own_and_handover(tmp_path):
    kt, out = tmp_path / "kt.csv", tmp_path / "b.json"
    _trace(kt, _turns_chain())
    subprocess.run([sys.executable, os.path.join(ROOT, "profiles", "turns2_breakdown.py"), str(kt), str(out)],
                   check=True, capture_output=True)
    b = json.load(open(out))["slabs"]
    assert set(b) == {"100", "101"}
    for thr, v in b.items():
        assert v["interaction_calls"] == 4  # from each slab's 3rd interaction on
        assert abs(v["us_per_call"]["k_fluid_tiled_w4"] - 1.0) < 1e-9
        assert abs(v["total_us_per_call"] - 1.1) < 0.051
    # slab 0's update follows slab 1's interaction (a hand-over), slab 1's update follows slab
    # 0's update; the interactions follow the other slab's kernels: no own gaps at all here
    assert b["100"]["idle_own_us_per_call"] == 0.0 and b["101"]["idle_own_us_per_call"] == 0.0
    assert b["100"]["idle_handover_us_per_call"] > 0 and b["101"]["idle_handover_us_per_call"] > 0


def test_breakdown_own_gap_is_the_slabs_own(tmp_path):
    """One slab alone: every idle interval sits between two of its own kernels."""
    kt, out = tmp_path / "kt.csv", tmp_path / "b.json"
    rows, t = [], 0
    for _ in range(6):
        rows.append(("7", t, t + 1000, "k_fluid_tiled_w4"))
        rows.append(("7", t + 1040, t + 1140, "k_update_cls"))  # 40 ns gap
        t += 1200  # 60 ns gap before the next call
    _trace(kt, rows)
    subprocess.run([sys.executable, os.path.join(ROOT, "profiles", "turns2_breakdown.py"), str(kt), str(out)],
                   check=True, capture_output=True)
    v = json.load(open(out))["slabs"]["7"]
    assert abs(v["idle_own_us_per_call"] - 0.1) < 0.051 and v["idle_handover_us_per_call"] == 0.0


def test_t8_model_estimates(tmp_path):
    turns = {"bounds": [0, 5, 10], "runs": [{"owned_np": [100, 100]}],
             "summary_min_over_repeats": {"inplace": {"wall_ms_per_step": 5.0,
                                                      "slab_kernels_ms_per_step": [2.0, 2.2]}}}
    (tmp_path / "turns.log").write_text("progress {}\n" + json.dumps(turns) + "\n")
    slabs = {}
    for thr, kern, own, hand in (("11", 1000.0, 20.0, 60.0), ("12", 1080.0, 30.0, 40.0), ("3", 9.0, 9.0, 9.0)):
        slabs[thr] = {"total_us_per_call": kern, "idle_own_us_per_call": own, "idle_handover_us_per_call": hand,
                      "us_per_call": {"k_fluid_tiled_w4": kern}}
    (tmp_path / "trace.json").write_text(json.dumps({"slabs": slabs}))
    (tmp_path / "single.json").write_text(json.dumps({"ms_per_step": 8.88}) + "\n")
    out = tmp_path / "summary.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "profiles", "t8_model.py"), str(tmp_path / "turns.log"),
                    str(tmp_path / "trace.json"), str(tmp_path / "single.json"), str(out)], check=True,
                   capture_output=True)
    d = json.load(open(out))
    # A: heaviest slab 2.2 + (5.0 - 4.2) / 2 = 2.6 ms; B: the timed threads (the last two by
    # id, not the warm-up's "3"), 2 x (1080 + 30) us = 2.22 ms
    assert abs(d["A"]["t8_ms_per_step"] - 2.6) < 1e-9 and abs(d["A"]["speedup"] - round(8.88 / 2.6, 3)) < 1e-9
    assert abs(d["B"]["critical_us_per_call"] - 1110.0) < 1e-9
    assert abs(d["B"]["t8_ms_per_step"] - 2.22) < 1e-9
    assert [p["thread"] for p in d["per_slab_trace"]] == ["11", "12"]
