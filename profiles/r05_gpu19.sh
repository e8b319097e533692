#!/bin/bash
# Round 5 A/B at cfg5: the NN effective viscosity with the HB power / Papanastasiou exponential
# skipped per wave when no lane needs it (nn_skip) vs computed always (nn_noskip), cfg5-only builds.
mkdir -p gpurun_out
timeout -k 10 500 bash profiles/ab.sh 3 scratch/nn_noskip scratch/nn_skip -- --workload cfg5 --steps 12 --warmup 3 > gpurun_out/ab19_cfg5.log 2>&1 || exit $?
cat gpurun_out/ab19_cfg5.log
