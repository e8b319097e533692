#!/bin/bash
# Round 6: the fused update (1024 x 1, every load first, registers) — full GPU suite, the cfg3 8 y-slab
# turns run, its kernel trace, the cfg3 single domain on the same box, the T8 summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/test15.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test15.log | tail -8
[ $rc -eq 0 ] || exit $rc
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace > gpurun_out/r06/turns8_y15.log 2>&1 || exit $?
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y15" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y15.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y15 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y15_breakdown.json | tail -8
rm -rf gpurun_out/r06/trace_y15
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06/cfg3_single15.json 2> gpurun_out/r06/cfg3_single15.err || exit $?
python3 profiles/t8_model.py gpurun_out/r06/turns8_y15.log gpurun_out/r06/trace_y15_breakdown.json gpurun_out/r06/cfg3_single15.json gpurun_out/r06/t8_summary15.json
