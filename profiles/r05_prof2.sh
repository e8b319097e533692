#!/bin/bash
# Round 5 profile sets, part 2: cfg3 and cfg4; then the full GPU suite, smoke() and the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
bash "$R/profiles/round_sets.sh" r05_a cfg3 cfg4 > "$R/gpurun_out/prof2_sets.log" 2>&1 || { echo "sets rc=$?"; tail -20 "$R/gpurun_out/prof2_sets.log"; exit 1; }
tail -3 "$R/gpurun_out/prof2_sets.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$R/gpurun_out/gputest_r05p.log" 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$R/gpurun_out/gputest_r05p.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$R/gpurun_out/smoke_r05p.log" 2>&1; echo "smoke rc=$?"; tail -3 "$R/gpurun_out/smoke_r05p.log"
timeout -k 10 400 python -u bench.py > "$R/gpurun_out/bench_r05p.json" 2> "$R/gpurun_out/bench_r05p.err"
echo "bench rc=$?"; head -c 700 "$R/gpurun_out/bench_r05p.json"
