#!/bin/bash
# One round's profile sets (kernel stats + FETCH/WRITE traffic + bench line) for the
# BASELINE workloads on one MI355X: profiles/round_sets.sh <round-tag> [cfg ...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:?round tag}
shift || true
# heartbeat: the reference CPU baseline of a 10M case runs minutes without output
mkdir -p "$R/gpurun_out"
( while sleep 50; do date >> "$R/gpurun_out/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for c in ${*:-cfg2 cfg5 cfg3 cfg4}; do
  case $c in
    cfg2) bash "$R/profiles/collect.sh" "$T" --steps 20 --warmup 3 ;;
    cfg5) bash "$R/profiles/collect.sh" "${T}_cfg5" --workload cfg5 --steps 10 --warmup 2 ;;
    cfg3) bash "$R/profiles/collect.sh" "${T}_cfg3" --workload cfg3 --steps 6 --warmup 2 --cpu-steps 3 ;;
    cfg4) bash "$R/profiles/collect.sh" "${T}_cfg4" --workload cfg4 --steps 10 --warmup 2 --cpu-steps 6 ;;
  esac
done
echo round-sets-done
