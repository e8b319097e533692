#!/bin/bash
# One GPU call: the -m gpu suite (no -x: every failure is listed), then -- unless the suite
# ended on a fault, abort or time limit -- the default bench.  Usage: gpu_round.sh TAG [pytest args]
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread "$@" \
  > gpurun_out/gputest_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/gputest_$tag.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
brc=$?
echo "bench rc=$brc"
tail -c 3000 gpurun_out/bench_$tag.json
exit $brc
