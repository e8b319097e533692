#!/bin/bash
# Profiling recipe used for profiles/<round>/ (run on the MI355X box from the repo root).
#   1. kernel trace + stats of the bench command
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc passes, MI355X_MICROARCH.md §rocprofv3)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${1:-$R/gpurun_out/prof}
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline"}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1
echo done
