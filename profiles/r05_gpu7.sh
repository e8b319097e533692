#!/bin/bash
# Round 5 (re-entry): the full GPU suite and the default bench on the last committed code.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r05g.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputest_r05g.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r05g.json 2> gpurun_out/bench_r05g.err
echo "bench rc=$?"; head -c 1500 gpurun_out/bench_r05g.json
