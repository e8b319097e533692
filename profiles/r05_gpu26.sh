#!/bin/bash
# Round 5 A/B at cfg2 (cfg2-only builds of the tiled kernel): compiler scheduling options.
mkdir -p gpurun_out
timeout -k 10 900 bash profiles/ab.sh 2 scratch/t_base scratch/t_ilp scratch/t_bias0 scratch/t_bias100 scratch/t_mem -- --steps 40 --warmup 5 > gpurun_out/ab26_cfg2.log 2>&1 || exit $?
cat gpurun_out/ab26_cfg2.log
