#!/bin/bash
# Round 6 profile sets (1): cfg2 and cfg5 — rocprofv3 kernel stats, FETCH/WRITE traffic, the
# PMC counter passes (frac_counters), then the bench line with the CPU baseline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
( while sleep 50; do date >> "$R/gpurun_out/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMC=1 timeout -k 10 900 bash profiles/collect.sh r06_a --steps 20 --warmup 3 || exit $?
PMC=1 timeout -k 10 900 bash profiles/collect.sh r06_a_cfg5 --workload cfg5 --steps 10 --warmup 2 || exit $?
cat profiles/r06_a/bench.json | head -c 600; echo
cat profiles/r06_a_cfg5/bench.json | head -c 400; echo
