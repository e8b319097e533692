#!/bin/bash
# Round 6: full GPU suite, then the cfg3 y split in turns mode (timing + one kernel trace).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/gputest4.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/gputest4.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
SPH_SLAB_TURNS=2 timeout -k 10 500 python -u profiles/slab_turns.py --axis 1 --modes inplace,overlap --repeat 2 --steps 8 > gpurun_out/r06/turns8_y4.log 2>&1 || exit $?
tail -c 700 gpurun_out/r06/turns8_y4.log
cd /tmp && export TMPDIR=/tmp
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y4" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --only overlap --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y4.log" 2>&1 || exit $?
cd "$R"
f=$(find gpurun_out/r06/trace_y4 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y4_breakdown.json | tail -3
