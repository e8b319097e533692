#!/bin/bash
# Round 5: the full GPU suite, the turns measurement of the three ghost modes, the default bench.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r05f.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/gputest_r05f.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SPH_SLAB_TURNS=1 timeout -k 10 400 python -u profiles/slab_turns.py --repeat 2 > gpurun_out/turns_r05f.log 2>&1 || exit $?
tail -c 900 gpurun_out/turns_r05f.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r05f.json 2> gpurun_out/bench_r05f.err
echo "bench rc=$?"; head -c 1200 gpurun_out/bench_r05f.json
