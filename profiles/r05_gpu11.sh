#!/bin/bash
# Round 5: cfg3 interaction per slab vs the number of slabs (full-step turns mode, in-place ghosts).
mkdir -p gpurun_out
for n in 1 2 4 8; do
  SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --slabs $n --repeat 1 --steps 6 --modes inplace > gpurun_out/turns_n${n}_r05k.log 2>&1 || exit $?
  echo "slabs $n"; grep -o '"summary_min_over_repeats".*' gpurun_out/turns_n${n}_r05k.log | cut -c1-700
done
