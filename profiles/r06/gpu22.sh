#!/bin/bash
# Round 6: the in-process transport copies both faces in one kernel (as RCCL moves a group) —
# slab GPU tests, the cfg3 8 y-slab turns run, its trace, cfg3 single domain, T8 summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_slab.py tests/test_gpu_slab_y.py tests/test_gpu_slab_mp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/test22.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test22.log | tail -8
[ $rc -eq 0 ] || exit $rc
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace > gpurun_out/r06/turns8_y22.log 2>&1 || exit $?
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y22" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y22.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y22 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y22_breakdown.json | tail -8
rm -rf gpurun_out/r06/trace_y22
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06/cfg3_single22.json 2> gpurun_out/r06/cfg3_single22.err || exit $?
python3 profiles/t8_model.py gpurun_out/r06/turns8_y22.log gpurun_out/r06/trace_y22_breakdown.json gpurun_out/r06/cfg3_single22.json gpurun_out/r06/t8_summary22.json
