#!/bin/bash
# Round 5 profile sets, part 1: cfg2 and cfg5 (kernel stats, FETCH/WRITE traffic, bench line),
# then the SQ/TCC counter passes of both (MI355X_MICROARCH.md: one counter group per run).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/profiles/round_sets.sh" r05_a cfg2 cfg5
BENCH_ARGS="--steps 6 --warmup 2 --no-cpu-baseline --no-cfg3 --developed-presteps 0" bash "$R/profiles/pmc_passes.sh" "$R/gpurun_out/pmc_r05_a"
BENCH_ARGS="--workload cfg5 --steps 4 --warmup 2 --no-cpu-baseline --no-cfg3 --developed-presteps 0" bash "$R/profiles/pmc_passes.sh" "$R/gpurun_out/pmc_r05_a_cfg5"
mkdir -p "$R/gpurun_out/profiles/r05_a/pmc" "$R/gpurun_out/profiles/r05_a_cfg5/pmc"
python3 "$R/profiles/pmc_summary.py" "$R/gpurun_out/pmc_r05_a" "$R/gpurun_out/profiles/r05_a/pmc/counters.json" > "$R/gpurun_out/profiles/r05_a/pmc/counters.txt"
python3 "$R/profiles/pmc_summary.py" "$R/gpurun_out/pmc_r05_a_cfg5" "$R/gpurun_out/profiles/r05_a_cfg5/pmc/counters.json" > "$R/gpurun_out/profiles/r05_a_cfg5/pmc/counters.txt"
rm -rf "$R/gpurun_out/pmc_r05_a"/p*/ "$R/gpurun_out/pmc_r05_a_cfg5"/p*/
echo prof1-done
