#!/bin/bash
# Round 6: NN single-phase-unit A/B at cfg5 (headline-only builds), then the NN / restart / slab tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 600 bash profiles/ab.sh 2 scratch/nn_base scratch/nn_uni -- --workload cfg5 --steps 20 --warmup 3 > gpurun_out/r06/ab_nn.log 2>&1 || exit $?
cat gpurun_out/r06/ab_nn.log
timeout -k 10 900 python -u -m pytest tests/test_nn.py tests/test_restart_bodies.py tests/test_bodies.py tests/test_gpu_slab_mp.py tests/test_gpu_slab_y.py "tests/test_fullsize.py::test_cfg5_2m_nn_matches_reference" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/test5.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test5.log | tail -8
exit $rc
