#!/bin/bash
# Round 5: NN drain A/B at cfg5 (main vs diag builds without / with the read-ahead), then the
# full-step turns mode (SPH_SLAB_TURNS=2) of the cfg3 8-slab split, in-place vs overlap ghosts.
mkdir -p gpurun_out
timeout -k 10 400 bash profiles/ab.sh 2 main scratch/nn_p0 scratch/nn_p1 -- --workload cfg5 --steps 20 --warmup 3 > gpurun_out/ab_nn_r05j.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab_nn_r05j.log | tail -8
[ $rc -eq 0 ] || exit $rc
SPH_SLAB_TURNS=2 timeout -k 10 400 python -u profiles/slab_turns.py --repeat 2 --modes inplace,overlap > gpurun_out/turns2_r05j.log 2>&1
rc=$?; echo "turns rc=$rc"; tail -c 1800 gpurun_out/turns2_r05j.log
exit $rc
