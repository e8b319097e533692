#!/bin/bash
# Round 5, first GPU call: the -m gpu suite + default bench (gpu_round.sh), then the turns
# measurement of the cfg3 8-slab split (profiles/slab_turns.py).
set -o pipefail
bash profiles/gpu_round.sh r05a || exit $?
SPH_SLAB_TURNS=1 timeout -k 10 400 python -u profiles/slab_turns.py --repeat 2 > gpurun_out/turns_r05a.log 2>&1
rc=$?
tail -c 2500 gpurun_out/turns_r05a.log
exit $rc
