#!/bin/bash
# Round 6: the incremental-divide tests with the fused update at 512 x 2 (the default build)
# and at 1024 x 1 (gpurun_var/u1024), after test_inc_divide_verlet_stirred[0] failed once at
# 512 x 2 (gpu15).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_divide_inc.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06/test16_512.log 2>&1
echo "512: rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/r06/test16_512.log | tail -6
SPH_LIB=$R/gpurun_var/u1024/libsphcore.so timeout -k 10 300 python -u -m pytest tests/test_divide_inc.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06/test16_1024.log 2>&1
echo "1024: rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/r06/test16_1024.log | tail -6
