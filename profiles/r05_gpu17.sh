#!/bin/bash
# Round 5: launch-tail diagnostic with the blocks' last items (cfg2).
mkdir -p gpurun_out
L=$(pwd)/scratch/tail/libsphcore.so
SPH_LIB=$L timeout -k 10 200 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail4_cfg2.json 2> gpurun_out/tail4_cfg2.err || exit $?
grep TAIL gpurun_out/tail4_cfg2.err | tail -6
