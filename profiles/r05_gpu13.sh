#!/bin/bash
# Round 5: launch-tail diagnostic of k_fluid_tiled with block start times (cfg2, cfg3).
mkdir -p gpurun_out
L=$(pwd)/scratch/tail/libsphcore.so
SPH_LIB=$L timeout -k 10 200 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail2_cfg2.json 2> gpurun_out/tail2_cfg2.err || exit $?
grep TAIL gpurun_out/tail2_cfg2.err | tail -4
SPH_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg3 --steps 6 --warmup 2 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail2_cfg3.json 2> gpurun_out/tail2_cfg3.err || exit $?
grep TAIL gpurun_out/tail2_cfg3.err | tail -4
