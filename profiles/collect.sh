#!/bin/bash
# Round profile collection (run on the MI355X box from the repo root):
#   profiles/collect.sh <tag> [bench args]
#   1. rocprofv3 --kernel-trace --stats of the bench            -> <tag>/kernel_stats.csv
#   2. rocprofv3 --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE passes    -> <tag>/pmc_traffic.json
#      (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass,
#       MI355X_MICROARCH.md §rocprofv3; never combined with sys/runtime traces)
#   (PMC=1: the counter passes of pmc_passes.sh                -> <tag>/pmc/counters.json)
#   4. bench.py (default flags, incl. the CPU baseline)        -> <tag>/bench.json
#   (the profiled passes 1-3 skip bench.py's extra cfg3 timing and its developed-flow run:
#    --no-cfg3 --developed-presteps 0; 8000 more steps under --pmc overran the tool's buffers)
#      (reads the traffic of step 2-3 from profiles/<tag>/)
# Results go to profiles/<tag>/ of the box copy and to gpurun_out/profiles/<tag>/.
set -e
TAG=${1:?tag}
shift || true
ARGS=${*:-"--steps 20 --warmup 3"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
DST=$R/profiles/$TAG
export TMPDIR=/tmp
mkdir -p "$OUT" "$DST"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $ARGS --no-cpu-baseline --no-cfg3 --developed-presteps 0 > "$OUT/kt.log" 2>&1
# provisional bench.json (workload, np) so step 4's bench finds this round's traffic
grep '^{' "$OUT/kt.log" | tail -1 > "$DST/bench.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS --no-cpu-baseline --no-cfg3 --developed-presteps 0 > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS --no-cpu-baseline --no-cfg3 --developed-presteps 0 > "$OUT/write.log" 2>&1
python3 "$R/profiles/summarize.py" "$OUT" "$DST"
# PMC=1: the counter passes of profiles/pmc_passes.sh (VALU mix, waits, LDS, L2) -> <tag>/pmc,
# read by step 4's bench for roofline.frac_counters
if [ -n "${PMC:-}" ]; then
  BENCH_ARGS="$ARGS --no-cpu-baseline --no-cfg3 --developed-presteps 0" bash "$R/profiles/pmc_passes.sh" "$OUT/pmc" > "$OUT/pmc.log" 2>&1
  mkdir -p "$DST/pmc"
  python3 "$R/profiles/pmc_summary.py" "$OUT/pmc" "$DST/pmc/counters.json" > "$DST/pmc/counters.txt"
fi
timeout -k 10 400 python3 "$R/bench.py" $ARGS > "$OUT/bench.log" 2>&1
grep '^{' "$OUT/bench.log" | tail -1 > "$DST/bench.json"
mkdir -p "$R/gpurun_out/profiles/$TAG"
cp -r "$DST"/* "$R/gpurun_out/profiles/$TAG/"
rm -rf "$OUT/kt" "$OUT/fetch" "$OUT/write" "$OUT/pmc"  # the raw traces (summarised above) stay on the box
echo collect-done
