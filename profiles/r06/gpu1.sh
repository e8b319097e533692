#!/bin/bash
# Round 6 baseline on a fresh box: the 8-slab cfg3 turns measurement (round-5 x-slabs) and the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
SPH_SLAB_TURNS=2 timeout -k 10 400 python -u profiles/slab_turns.py --modes inplace --repeat 2 --steps 8 > gpurun_out/r06/turns8_base.log 2>&1 || exit $?
tail -c 1500 gpurun_out/r06/turns8_base.log
timeout -k 10 300 python -u bench.py > gpurun_out/r06/bench_base.json 2> gpurun_out/r06/bench_base.err || exit $?
head -c 600 gpurun_out/r06/bench_base.json
