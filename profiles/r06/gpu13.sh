#!/bin/bash
# Round 6: update kernels with every load before the first store (one memory latency per
# particle) and the classification / pack count from registers; in-process slab reductions on
# the device.  Full GPU suite, cfg2 and cfg3 A/B against the previous commit's library
# (gpurun_var/base), the cfg3 8 y-slab turns run and its kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/test13.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test13.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash profiles/ab.sh 3 gpurun_var/base main -- --steps 40 --warmup 5 > gpurun_out/r06/ab13.log 2>&1 || exit $?
cat gpurun_out/r06/ab13.log
timeout -k 10 500 bash profiles/ab.sh 2 gpurun_var/base main -- --workload cfg3 --steps 8 --warmup 2 > gpurun_out/r06/ab13_cfg3.log 2>&1 || exit $?
cat gpurun_out/r06/ab13_cfg3.log
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace,overlap > gpurun_out/r06/turns8_y13.log 2>&1 || exit $?
tail -c 600 gpurun_out/r06/turns8_y13.log
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y13" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y13.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y13 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y13_breakdown.json | tail -8
rm -rf gpurun_out/r06/trace_y13
