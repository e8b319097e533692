#!/bin/bash
# Round 6: the divide's classification in the update kernel (single domain), alternating A/B
# against the separate k_inc_classify launch (SPH_CLS_SPLIT=1): cfg2 (Verlet) and cfg3 (Symplectic).
# (The GPU tests of the change: tests/test_motion.py, test_divide_inc.py, test_gpu_items.py,
# test_gpu_parity.py, test_bodies.py, test_restart_bodies.py, test_cpp_host.py: 98 passed.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 500 bash profiles/ab.sh 3 main:SPH_CLS_SPLIT=1 main -- --steps 40 --warmup 5 > gpurun_out/r06/ab9.log 2>&1 || exit $?
cat gpurun_out/r06/ab9.log
timeout -k 10 500 bash profiles/ab.sh 2 main:SPH_CLS_SPLIT=1 main -- --workload cfg3 --steps 8 --warmup 2 > gpurun_out/r06/ab9_cfg3.log 2>&1 || exit $?
cat gpurun_out/r06/ab9_cfg3.log
