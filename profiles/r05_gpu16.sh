#!/bin/bash
# Round 5: A/B base vs the per-instantiation register budget (cfg2, cfg3); tiled-kernel parity;
# the 8-slab full-step turns (in-place vs overlap ghosts) on the final code.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize.py tests/test_gpu_items.py tests/test_cubic.py tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_r05m.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/parity_r05m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh 2 scratch/base main -- --steps 40 --warmup 5 > gpurun_out/ab16_cfg2.log 2>&1 || exit $?
cat gpurun_out/ab16_cfg2.log
timeout -k 10 400 bash profiles/ab.sh 2 scratch/base main -- --workload cfg3 --steps 8 --warmup 3 > gpurun_out/ab16_cfg3.log 2>&1 || exit $?
cat gpurun_out/ab16_cfg3.log
SPH_SLAB_TURNS=2 timeout -k 10 400 python -u profiles/slab_turns.py --slabs 8 --repeat 2 --steps 8 --modes inplace,overlap > gpurun_out/turns8_r05m.log 2>&1 || exit $?
grep -o '"summary_min_over_repeats".*' gpurun_out/turns8_r05m.log | cut -c1-1500
