#!/bin/bash
# Round 5 A/B at cfg5: the NN effective viscosity with the HB power / Papanastasiou exponential
# skipped per wave when no lane needs it (nn_skip) vs computed always (nn_noskip), cfg5-only builds;
# then the NN tests and the turns-mode bitwise test on the main build.
mkdir -p gpurun_out
timeout -k 10 500 bash profiles/ab.sh 3 scratch/nn_noskip scratch/nn_skip -- --workload cfg5 --steps 12 --warmup 3 > gpurun_out/ab19_cfg5.log 2>&1 || exit $?
cat gpurun_out/ab19_cfg5.log
timeout -k 10 500 python -u -m pytest tests/test_nn.py tests/test_gpu_slab.py -m gpu -x -q -k "nn or turns" --timeout 300 --timeout-method thread > gpurun_out/t19.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/t19.log
