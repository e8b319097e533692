#!/bin/bash
# Round 6: the classification and (slabs) the exchange's count pass in the update kernels:
# the divide / slab / motion / turns GPU tests, then alternating A/B against the separate
# launches (SPH_CLS_SPLIT=1) at cfg2 and cfg3, and the cfg3 y-slab turns measurement.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 1000 python -u -m pytest tests/test_divide_inc.py tests/test_gpu_items.py tests/test_gpu_slab.py tests/test_gpu_slab_y.py tests/test_gpu_slab_mp.py tests/test_motion.py tests/test_slab_capacity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/test10.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test10.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash profiles/ab.sh 3 main:SPH_CLS_SPLIT=1 main -- --steps 40 --warmup 5 > gpurun_out/r06/ab10.log 2>&1 || exit $?
cat gpurun_out/r06/ab10.log
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace,overlap > gpurun_out/r06/turns8_y10.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r06/turns8_y10.log
