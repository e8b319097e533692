#!/bin/bash
# Round 6: the update's products kept out of multiply-add fusion, the fused update at 512 x 2 —
# full GPU suite, the cfg3 8 y-slab turns run, its trace, cfg3 single domain, T8 summary, and
# the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r06"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/test20.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/test20.log | tail -8
[ $rc -eq 0 ] || exit $rc
SPH_SLAB_TURNS=2 timeout -k 10 300 python -u profiles/slab_turns.py --axis 1 --slabs 8 --steps 8 --repeat 2 --modes inplace > gpurun_out/r06/turns8_y20.log 2>&1 || exit $?
SPH_SLAB_TURNS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r06/trace_y20" -o run -- python3 "$R/profiles/slab_turns.py" --axis 1 --modes inplace --repeat 1 --steps 6 > "$R/gpurun_out/r06/trace_y20.log" 2>&1 || exit $?
f=$(find gpurun_out/r06/trace_y20 -name "*kernel_trace.csv" | head -1)
python3 profiles/turns2_breakdown.py "$f" gpurun_out/r06/trace_y20_breakdown.json | tail -8
rm -rf gpurun_out/r06/trace_y20
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06/cfg3_single20.json 2> gpurun_out/r06/cfg3_single20.err || exit $?
python3 profiles/t8_model.py gpurun_out/r06/turns8_y20.log gpurun_out/r06/trace_y20_breakdown.json gpurun_out/r06/cfg3_single20.json gpurun_out/r06/t8_summary20.json
timeout -k 10 400 python3 bench.py > gpurun_out/r06/bench20.json 2> gpurun_out/r06/bench20.err || exit $?
grep '^{' gpurun_out/r06/bench20.json | tail -1 | head -c 400
