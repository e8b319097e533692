#!/bin/bash
# Round 6: the motion tree (nested objects, circular / file / flash / null movements) vs the reference goldens.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_motion.py tests/test_bodies.py tests/test_restart_bodies.py tests/test_cpp_host.py tests/test_abi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/test8.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test8.log | tail -8
exit $rc
