#!/bin/bash
# Round 6: k_inc_boxes at 3 blocks per CU (52 KB LDS): divide parity, then A/B at cfg2 and the y-slab turns.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_divide_inc.py tests/test_gpu_items.py tests/test_gpu_slab_y.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r06/test7.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test7.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash profiles/ab.sh 3 scratch/v_base main -- --steps 40 --warmup 5 > gpurun_out/r06/ab7.log 2>&1 || exit $?
cat gpurun_out/r06/ab7.log
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 1 --modes inplace > gpurun_out/r06/turns8_y7.log 2>&1 || exit $?
tail -c 700 gpurun_out/r06/turns8_y7.log
