#!/bin/bash
# Round 6: the NN golden of the v5.0 external forces / ViscoTime, and the cfg3 y-slab turns
# measurement (ghosts in place and beside the interior items) for profiles/r06_turns8.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_nn.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r06/test6.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test6.log | tail -5
[ $rc -eq 0 ] || exit $rc
SPH_SLAB_TURNS=2 timeout -k 10 400 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace,overlap > gpurun_out/r06/turns8_y6.log 2>&1 || exit $?
tail -c 3000 gpurun_out/r06/turns8_y6.log
