#!/bin/bash
# Round 6, final build: the full GPU suite, then profile set 2 (cfg3, cfg4).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/test23.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test23.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash profiles/r06/prof2.sh
