#!/bin/bash
# Round 5: one slab's own step in the turns mode (cfg3 8-slab split), three ghost modes, two repeats.
mkdir -p gpurun_out
SPH_SLAB_TURNS=1 timeout -k 10 500 python -u profiles/slab_turns.py --repeat 2 > gpurun_out/turns_r05i.log 2>&1
rc=$?; echo "turns rc=$rc"; tail -c 2500 gpurun_out/turns_r05i.log
exit $rc
