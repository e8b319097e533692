#!/bin/bash
# Round 6: the y-slab tests again, then a kernel trace of one turns run of the cfg3 y split.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab_y.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06/test_y.log 2>&1
rc=$?; tail -16 gpurun_out/r06/test_y.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --only inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y.log" 2>&1 || exit $?
cd "$R"
f=$(find gpurun_out/r06/trace_y -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y_breakdown.json
rm -f "$f"
