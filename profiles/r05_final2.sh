#!/bin/bash
# Round 5, last call: the full GPU suite, smoke() and the default bench on the final tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$R/gpurun_out/gputest_r05final.log" 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$R/gpurun_out/gputest_r05final.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$R/gpurun_out/smoke_r05final.log" 2>&1; echo "smoke rc=$?"; tail -2 "$R/gpurun_out/smoke_r05final.log"
timeout -k 10 400 python -u bench.py > "$R/gpurun_out/bench_r05final.json" 2> "$R/gpurun_out/bench_r05final.err"
echo "bench rc=$?"; head -c 400 "$R/gpurun_out/bench_r05final.json"
