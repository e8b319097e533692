#!/bin/bash
# Round 6 profile sets (2): cfg3 and cfg4 — kernel stats, traffic, bench line with CPU baseline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
( while sleep 50; do date >> "$R/gpurun_out/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 bash profiles/collect.sh r06_a_cfg3 --workload cfg3 --steps 6 --warmup 2 --cpu-steps 3 || exit $?
timeout -k 10 700 bash profiles/collect.sh r06_a_cfg4 --workload cfg4 --steps 10 --warmup 2 --cpu-steps 6 || exit $?
cat profiles/r06_a_cfg3/bench.json | head -c 400; echo
cat profiles/r06_a_cfg4/bench.json | head -c 400; echo
