#!/bin/bash
# Round 5 A/B (alternating, one box): the round's previous commit (base) vs grids of resident
# blocks + two-phase claims without / with the 4-wave register budget; cfg2, then cfg3.
mkdir -p gpurun_out
timeout -k 10 500 bash profiles/ab.sh 3 scratch/base scratch/nowaves main -- --steps 40 --warmup 5 > gpurun_out/ab15_cfg2.log 2>&1 || exit $?
cat gpurun_out/ab15_cfg2.log
timeout -k 10 600 bash profiles/ab.sh 2 scratch/base scratch/nowaves main -- --workload cfg3 --steps 8 --warmup 3 > gpurun_out/ab15_cfg3.log 2>&1 || exit $?
cat gpurun_out/ab15_cfg3.log
