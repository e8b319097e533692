#!/bin/bash
# Round 6: y-slab parity tests, then the 8-slab cfg3 turns measurement of the y split.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_y.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/test_y.log 2>&1
rc=$?; tail -25 gpurun_out/r06/test_y.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SPH_SLAB_TURNS=2 timeout -k 10 500 python -u profiles/slab_turns.py --axis 1 --modes inplace,overlap --repeat 2 --steps 8 > gpurun_out/r06/turns8_y.log 2>&1 || exit $?
tail -c 1200 gpurun_out/r06/turns8_y.log
