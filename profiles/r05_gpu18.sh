#!/bin/bash
# Round 5 A/B: the launch-tail queue (last fluid items from one shared queue in list order) vs
# the previous commit; cfg2, cfg5, cfg3; items and parity tests first.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_items.py tests/test_gpu_parity.py tests/test_nn.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t18.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t18.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh 3 scratch/prev main -- --steps 40 --warmup 5 > gpurun_out/ab18_cfg2.log 2>&1 || exit $?
cat gpurun_out/ab18_cfg2.log
timeout -k 10 300 bash profiles/ab.sh 2 scratch/prev main -- --workload cfg5 --steps 10 --warmup 3 > gpurun_out/ab18_cfg5.log 2>&1 || exit $?
cat gpurun_out/ab18_cfg5.log
timeout -k 10 300 bash profiles/ab.sh 1 scratch/prev main -- --workload cfg3 --steps 6 --warmup 2 > gpurun_out/ab18_cfg3.log 2>&1 || exit $?
cat gpurun_out/ab18_cfg3.log
