#!/bin/bash
# Round 5 A/B at cfg5 (cfg5-only NN builds): the mirrored drain one vs two pairs per iteration,
# at the 4-wave register budget and at 3 waves.
mkdir -p gpurun_out
timeout -k 10 700 bash profiles/ab.sh 2 scratch/nn_d1 scratch/nn_d2 scratch/nn_d1w3 scratch/nn_d2w3 -- --workload cfg5 --steps 12 --warmup 3 > gpurun_out/ab25_cfg5.log 2>&1 || exit $?
cat gpurun_out/ab25_cfg5.log
