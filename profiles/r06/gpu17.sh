#!/bin/bash
# Round 6, last: smoke() and the default bench line (the driver's round-end commands).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06/smoke17.log 2>&1 || { tail -20 gpurun_out/r06/smoke17.log; exit 1; }
tail -2 gpurun_out/r06/smoke17.log
start=$(date +%s)
timeout -k 10 600 python3 bench.py > gpurun_out/r06/bench17.json 2> gpurun_out/r06/bench17.err || { tail -20 gpurun_out/r06/bench17.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
grep '^{' gpurun_out/r06/bench17.json | tail -1 | head -c 1500
