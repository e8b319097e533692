#!/bin/bash
# Round 5: launch-tail diagnostic of k_fluid_tiled (block start/end times) at cfg2, cfg3 and the 8-slab split.
mkdir -p gpurun_out
L=$(pwd)/scratch/tail/libsphcore.so
SPH_LIB=$L timeout -k 10 200 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail_cfg2.json 2> gpurun_out/tail_cfg2.err || exit $?
grep TAIL gpurun_out/tail_cfg2.err | tail -4
SPH_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg3 --steps 6 --warmup 2 --no-cpu-baseline --no-cfg3 --developed-presteps 0 > gpurun_out/tail_cfg3.json 2> gpurun_out/tail_cfg3.err || exit $?
grep TAIL gpurun_out/tail_cfg3.err | tail -4
SPH_LIB=$L SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --slabs 8 --repeat 1 --steps 4 --modes inplace > gpurun_out/tail_slab8.log 2>&1 || exit $?
grep TAIL gpurun_out/tail_slab8.log | tail -16
